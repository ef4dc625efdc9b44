# Fill-target sweep for the axis kernels (tools/probe_axis.py), one process per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sweep_axis.log
: > $OUT
for c in 2 4 8; do for pr in 0 1 2; do
  RDX_AXIS_PROBE=$pr RDX_AXIS_COLS_WGS_PER_CU=$c timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 || exit 1
done; done
