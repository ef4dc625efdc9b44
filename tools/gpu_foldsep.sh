# Separate cols fold launch: parity (auto and forced on), then the axis probe (auto, off, on).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/foldsep.log
: > $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/foldsep_pytest.log 2>&1 || exit 1
RDX_AXIS_FOLD_SEP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/foldsep_pytest.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
for f in 0 1; do
  RDX_AXIS_FOLD_SEP=$f timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 || exit 1
done
