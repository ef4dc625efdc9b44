# A/B of two in-tree builds (librdx.so vs $RDX_B, default librdx_plain.so): parity tests on A, then the
# headline loop and the per-config measurements for both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-ab}
B=${RDX_B:-reductionist-rs_amd/librdx_plain.so}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_A.log 2>&1 &&
RDX_LIB_PATH=$PWD/$B timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_B.log 2>&1 &&
timeout -k 10 300 python tools/bench_configs.py --no-cpu > $OUT/cfg_A.log 2>&1 &&
RDX_LIB_PATH=$PWD/$B timeout -k 10 300 python tools/bench_configs.py --no-cpu > $OUT/cfg_B.log 2>&1
