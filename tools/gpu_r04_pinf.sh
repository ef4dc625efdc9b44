# GPU box (round 4): the single-stream parallel inflate — its GPU tests, the lone-chunk timing probe, a
# per-workgroup profile (RDX_PINF_PROF) and a kernel-trace profile of the probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r04pinf}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pinflate.py > $OUT/pytest_pinf.txt 2>&1
  rc=$?
  tail -4 $OUT/pytest_pinf.txt
  [ $rc -eq 0 ] || { tail -40 $OUT/pytest_pinf.txt; exit $rc; }
fi
timeout -k 10 300 python -u tools/probe_pinflate.py 10 > $OUT/probe.jsonl 2>$OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
RDX_PINF_PROF=1 timeout -k 10 300 python -u tools/probe_pinflate.py 1 > /dev/null 2>$OUT/wgprof.txt || { tail -20 $OUT/wgprof.txt; exit 1; }
grep pinf_prof $OUT/wgprof.txt | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/probe_pinflate.py 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/pinf_trace.py $OUT/prof/run_kernel_trace.csv 4
