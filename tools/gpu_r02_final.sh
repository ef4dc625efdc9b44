# Round-2 final records on the GPU box: the bench line, the headline kernel's trace stats, and the blosc2
# decode probe with its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r02f}
mkdir -p $OUT
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2trace -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --primary-only > $OUT/c2trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/b2trace -o run --output-format csv -- python3 tools/probe_blosc2.py 256 > $OUT/probe_blosc2.jsonl 2> $OUT/b2trace.log
