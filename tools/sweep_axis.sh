# Fill-target sweep for the axis kernels (tools/probe_axis.py), one process per setting, then one
# kernel-trace pass at the defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sweep_axis.log
: > $OUT
timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
for c in 1 2 8; do
  RDX_AXIS_COLS_WGS_PER_CU=$c timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
done
for r in 4 8 32; do
  RDX_AXIS_ROWS_WAVES_PER_CU=$r timeout -k 10 120 python tools/probe_axis.py >> $OUT 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/axisprof -o run --output-format csv -- python3 tools/probe_axis.py > gpurun_out/axisprof.log 2>&1
