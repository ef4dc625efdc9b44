# cols max: phase probe and fold settings (axis probe --minmax under each knob set).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/colsmax.log
: > $OUT
for cfg in "RDX_AXIS_PROBE=2" "RDX_AXIS_PROBE=2 RDX_AXIS_FOLD_SEP=0" "RDX_AXIS_FOLD_SEP=0" "RDX_AXIS_FOLD_KIB=160" "RDX_AXIS_FOLD_KIB=160 RDX_AXIS_FOLD_SEP=0" "RDX_AXIS_COLS_VW=1"; do
  echo "== $cfg" >> $OUT
  env $cfg timeout -k 10 120 python tools/probe_axis.py --minmax >> $OUT 2>&1 || exit 1
done
