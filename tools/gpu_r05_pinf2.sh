# Round 5: lone-stream inflate — the tabulated walk stops where the parses agree; kernel stats per case.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05p2}
mkdir -p $OUT
timeout -k 10 300 python -u tools/probe_pinflate.py 10 > $OUT/probe.jsonl 2> $OUT/probe.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_pinflate.py 5 > $OUT/trace.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_pinflate.py > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
exit $rc
