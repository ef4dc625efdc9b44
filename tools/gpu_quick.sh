# Quick cycle: GPU parity tests, then the per-config measurements under a kernel trace
# (RDX_SMALL=1: also the small single-chunk probe).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 tools/bench_configs.py --no-cpu > $OUT/cfg.log 2>&1 || exit 1
if [ -n "$RDX_SMALL" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ts -o run --output-format csv -- python3 tools/probe_small.py > $OUT/small.log 2>&1 || exit 1
fi
