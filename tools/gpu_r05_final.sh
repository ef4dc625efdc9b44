# Round-5 closing records, part 1 on the GPU box: smoke, the -m gpu suite (one pass), the bench line at its
# defaults and at the driver's --steps 20 --warmup 5.  Stops at the first failing step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05z}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err
rc=$?
tail -2 $OUT/pytest_gpu.log
exit $rc
