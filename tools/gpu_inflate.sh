# Device inflate: parity tests, then the throughput bench (tools/bench_inflate.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-zq}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 &&
timeout -k 10 400 python tools/bench_inflate.py ${RDX_BENCH_ARGS:-} > $OUT/bench.log 2>&1
