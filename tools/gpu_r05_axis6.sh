# Round 5: column-kernel shapes after the load fixes: tile widths (RDX_AXIS_COLS_W), lane widths
# (RDX_AXIS_COLS_VW) and 32 loads in flight for 8-byte lanes (librdx_cu32.so); kernel stats per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05ax6}
mkdir -p $OUT
run() {   # $1 = label, rest = env assignments
  local label=$1; shift
  env "$@" timeout -k 10 120 python3 -u tools/probe_axis.py --cols 2>> $OUT/axis.err | sed "s/^{/{\"label\": \"$label\", /" >> $OUT/axis.jsonl
}
for rep in 1 2; do
  run default RDX_X=0 || exit 1
  run w16 RDX_AXIS_COLS_W=16 || exit 1
  run w8 RDX_AXIS_COLS_W=8 || exit 1
  run vw4w16 RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_W=16 || exit 1
  run vw4w8 RDX_AXIS_COLS_VW=4 RDX_AXIS_COLS_W=8 || exit 1
  run cu32 RDX_LIB_PATH=reductionist-rs_amd/librdx_cu32.so || exit 1
  run cu32w16 RDX_LIB_PATH=reductionist-rs_amd/librdx_cu32.so RDX_AXIS_COLS_W=16 || exit 1
done
