# Round-2 profiling pass on the GPU box: k_multi timeline, per-kernel kernel-trace stats,
# separate FETCH_SIZE / WRITE_SIZE passes over tools/pmc_configs.py, and the headline kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r02}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/mixtrace -o run --output-format csv -- python3 tools/probe_mixed.py 30 > $OUT/mixtrace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfgtrace -o run --output-format csv -- python3 tools/pmc_configs.py 20 > $OUT/cfgtrace.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/pmc_configs.py 10 > $OUT/pmc_fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 tools/pmc_configs.py 10 > $OUT/pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2trace -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --primary-only > $OUT/c2trace.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
