# Round 5: 4-wide f32 column lanes — streaming only / + publish / whole (probe build).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05ax4}
mkdir -p $OUT
P=$PWD/reductionist-rs_amd/librdx_probe.so
for vw in 2 4; do for pr in 2 1 0; do
  RDX_LIB_PATH=$P RDX_AXIS_COLS_VW=$vw RDX_AXIS_PROBE=$pr timeout -k 10 200 python3 -u tools/probe_axis.py --cols >> $OUT/probe.jsonl 2>> $OUT/err || exit 1
done; done
