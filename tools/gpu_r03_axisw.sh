# GPU box: sliced column reductions — tile width W x lane width x workgroups-per-CU sweep (probe_axis.py --cols).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03axisw}
mkdir -p $OUT
timeout -k 10 120 python -u tools/probe_axis.py --cols > $OUT/axis_default.jsonl 2>>$OUT/axis.err || exit 1
for w in 32 16 8 4; do
  for vw in 2 4; do
    for g in 2 4; do
      RDX_AXIS_COLS_W=$w RDX_AXIS_COLS_VW=$vw RDX_AXIS_COLS_WGS_PER_CU=$g timeout -k 10 120 python -u tools/probe_axis.py --cols >> $OUT/axis_sweep.jsonl 2>>$OUT/axis.err || exit 1
    done
  done
done
