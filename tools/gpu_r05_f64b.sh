# Round 5: f64 sums — what the f64 arithmetic costs: the same bytes as f64 / i64 / u64 / f32 sums, min, count.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PLANES_QUICK=1
OUT=gpurun_out/${RDX_TAG:-r05f64b}
mkdir -p $OUT
for rep in 1 2; do
PLANES_DTYPES=float64,int64,uint64,float32 PLANES_OPS=sum,min,count timeout -k 10 200 python3 -u tools/probe_planes.py >> $OUT/ops.jsonl 2>> $OUT/ops.err || exit 1
done
