# Round 5: plain f64 sums with a compensated step per 4 elements; 1 and 2 workgroups per CU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PLANES_QUICK=1
OUT=gpurun_out/${RDX_TAG:-r05f64c}
mkdir -p $OUT
for rep in 1 2 3; do
for b in 32 64; do
RDX_FORCE_BPC=$b PLANES_DTYPES=float64,int64 PLANES_OPS=sum timeout -k 10 200 python3 -u tools/probe_planes.py >> $OUT/ops.jsonl 2>> $OUT/ops.err || exit 1
done
done
