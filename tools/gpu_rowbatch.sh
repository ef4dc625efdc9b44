# Row-batch routing for axis reductions: parity, then the axis probe with it on and off.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/rowbatch.log
: > $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rowbatch_pytest.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
RDX_AXIS_ROWBATCH_KIB=0 timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
