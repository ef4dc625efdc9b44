# Axis probe (all configs, twice) + the GPU parity suite: A/B of a k_axis change.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/axisab.log
: > $OUT
timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 &&
timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/axisab_pytest.log 2>&1
