# Two-level cols fold: parity, then the axis probe (auto, forced lane widths, fold groups, phase probes).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/axisfold.log
: > $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/axisfold_pytest.log 2>&1 || exit 1
timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
for vw in 4 2; do for kn in "RDX_AXIS_PROBE=0" "RDX_AXIS_PROBE=1" "RDX_AXIS_PROBE=2" "RDX_AXIS_FOLD_GROUP=8" "RDX_AXIS_FOLD_GROUP=1000000"; do
  env RDX_AXIS_COLS_VW=$vw $kn timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 || exit 1
done; done
