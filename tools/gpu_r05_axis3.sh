# Round 5: column reductions — 4-wide f32 lanes (512 B strips, 16 loads in flight) against the default
# 2-wide, with fold budgets, the separate fold launch and workgroups per CU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05ax3}
mkdir -p $OUT
run() { env "$@" timeout -k 10 200 python3 -u tools/probe_axis.py --cols >> $OUT/sweep.jsonl 2>> $OUT/sweep.err; }
run RDX_AXIS_COLS_VW=2 &&
run RDX_AXIS_COLS_VW=4 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_KIB=128 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_KIB=32 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_SEP=1 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_WGS_PER_CU=2 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_WGS_PER_CU=8 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_W=16 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_W=64 &&
run RDX_AXIS_COLS_VW=2 RDX_AXIS_FOLD_SEP=1 &&
run RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_SEP=1 RDX_AXIS_COLS_WGS_PER_CU=2
