# Round-6 closing records on the GPU box: smoke, the -m gpu suite (one pass), the bench line at its defaults and at
# the driver's --steps 20 --warmup 5, the headline kernel's trace stats with FETCH_SIZE / WRITE_SIZE passes, the
# per-kernel passes over tools/pmc_configs.py (trace stats, FETCH_SIZE, WRITE_SIZE), and the phase timeline of the
# small single launches (probe build) in both fold forms.  Stops at the first failing step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06z}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 500 python3 -u bench.py --full-out $OUT/bench_full.json > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 --full-out $OUT/bench_driver_full.json > $OUT/bench_driver.json 2> $OUT/bench_driver.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2trace -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --primary-only --full-out '' > $OUT/c2trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --primary-only --full-out '' > $OUT/pmc.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --primary-only --full-out '' > $OUT/pmcw.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfgtrace -o run --output-format csv -- python3 tools/pmc_configs.py 20 > $OUT/cfgtrace.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/cfg_fetch -o run --output-format csv -- python3 tools/pmc_configs.py 10 > $OUT/cfg_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/cfg_write -o run --output-format csv -- python3 tools/pmc_configs.py 10 > $OUT/cfg_write.log 2>&1 &&
RDX_FOLD_LAST=2 timeout -k 10 120 python3 -u tools/probe_timeline.py > $OUT/timeline_fold2.json 2> $OUT/timeline.err &&
RDX_FOLD_LAST=1 timeout -k 10 120 python3 -u tools/probe_timeline.py > $OUT/timeline_fold1.json 2>> $OUT/timeline.err
rc=$?
tail -2 $OUT/pytest_gpu.log
exit $rc
