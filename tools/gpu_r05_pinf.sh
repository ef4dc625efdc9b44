# Round 5: lone-stream inflate — declines back to the host, the tabulated walk, GNU gzip fixtures.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05p}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_pinflate.py tests/test_gpu_inflate.py > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/probe_pinflate.py 10 > $OUT/probe.jsonl 2> $OUT/probe.err
rc=$?
tail -3 $OUT/pytest.log
exit $rc
