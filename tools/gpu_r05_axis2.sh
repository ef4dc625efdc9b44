# Round 5: column reductions with 16 loads in flight per lane (librdx) vs 8 (librdx_u8); f64 plain sums at
# two workgroups per CU by default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PLANES_QUICK=1
OUT=gpurun_out/${RDX_TAG:-r05ax2}
mkdir -p $OUT
L=$PWD/reductionist-rs_amd
for rep in 1 2; do
for lib in librdx librdx_u8; do
  RDX_LIB_PATH=$L/$lib.so timeout -k 10 200 python3 -u tools/probe_axis.py >> $OUT/axis.jsonl 2>> $OUT/axis.err || exit 1
done
done
PLANES_DTYPES=float64 PLANES_OPS=sum timeout -k 10 200 python3 -u tools/probe_planes.py >> $OUT/f64.jsonl 2>> $OUT/f64.err
