# Axis kernels: parity tests, then lane width x fill target x phase probe (tools/probe_axis.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/sweep_axis2.log
: > $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_axis2_pytest.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
for vw in 4 2; do for c in 4 8 16; do for pr in 0 2; do
  RDX_AXIS_COLS_VW=$vw RDX_AXIS_PROBE=$pr RDX_AXIS_COLS_WGS_PER_CU=$c timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 || exit 1
done; done; done
