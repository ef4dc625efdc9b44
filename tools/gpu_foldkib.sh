# Cols fold budget sweep (RDX_AXIS_FOLD_KIB) x lane width.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/foldkib.log
: > $OUT
for kib in 8 16 32 64 128; do for vw in 0 2; do
  RDX_AXIS_FOLD_KIB=$kib RDX_AXIS_COLS_VW=$vw timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 || exit 1
done; done
