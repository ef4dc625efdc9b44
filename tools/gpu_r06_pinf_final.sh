# Round 6, after the k_pinflate work: smoke, the -m gpu suite (one pass), the bench line at its defaults and at the
# driver's --steps 20 --warmup 5, the lone-stream probe (tools/probe_pinflate.py, all cases) with its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06pf}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 500 python3 -u bench.py --full-out $OUT/bench_full.json > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 --full-out $OUT/bench_driver_full.json > $OUT/bench_driver.json 2> $OUT/bench_driver.err &&
timeout -k 10 300 python3 -u tools/probe_pinflate.py 20 > $OUT/pinflate_probe.jsonl 2> $OUT/pinflate_probe.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pinftrace -o run --output-format csv -- python3 tools/probe_pinflate.py 5 c4_shuffled_normal_f32_zlib1 > $OUT/pinftrace.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
exit $rc
