# Round 5: f64 plain sums (one step per 4 elements), and where the axis-0 column reduction's time goes
# (probe build: RDX_AXIS_PROBE=2 streams only, =1 streams + publishes, 0 the whole kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PLANES_QUICK=1
OUT=gpurun_out/${RDX_TAG:-r05ax}
mkdir -p $OUT
for rep in 1 2; do
for b in 32 64; do
RDX_FORCE_BPC=$b PLANES_DTYPES=float64,int64 PLANES_OPS=sum timeout -k 10 200 python3 -u tools/probe_planes.py >> $OUT/f64.jsonl 2>> $OUT/f64.err || exit 1
done
done
P=$PWD/reductionist-rs_amd/librdx_probe.so
for pr in 0 1 2; do
  RDX_LIB_PATH=$P RDX_AXIS_PROBE=$pr timeout -k 10 200 python3 -u tools/probe_axis.py --cols >> $OUT/axis_probe.jsonl 2>> $OUT/axis.err || exit 1
done
timeout -k 10 200 python3 -u tools/probe_axis.py >> $OUT/axis_all.jsonl 2>> $OUT/axis.err
