# GPU box: sliced column reductions — lane width x workgroups-per-CU sweep (probe_axis.py per setting).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03axis}
mkdir -p $OUT
timeout -k 10 120 python -u tools/probe_axis.py > $OUT/axis_default.jsonl 2>>$OUT/axis.err || exit 1
for vw in 2 4; do
  for w in 1 2 4; do
    RDX_AXIS_COLS_VW=$vw RDX_AXIS_COLS_WGS_PER_CU=$w timeout -k 10 120 python -u tools/probe_axis.py > $OUT/axis_vw${vw}_w$w.jsonl 2>>$OUT/axis.err || exit 1
  done
done
for fk in 32 128; do
  RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_WGS_PER_CU=1 RDX_AXIS_FOLD_KIB=$fk timeout -k 10 120 python -u tools/probe_axis.py > $OUT/axis_vw4_w1_fk$fk.jsonl 2>>$OUT/axis.err || exit 1
done
for rep in 1 2; do
  for v in "" _p2 _rot; do
    RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64${v}_$rep.jsonl 2>>$OUT/f64.err || exit 1
  done
done
