# Round 5: byte-shuffled f64 sums (the pipelined form) at 1 / 2 / 3 workgroups per CU (RDX_FORCE_BPC 32 / 64 / 96
# per chunk of the 8 x 64 MiB batch), against i64 over the same bytes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05f64d}
mkdir -p $OUT
for rep in 1 2; do for bpc in 32 64 96; do
  RDX_FORCE_BPC=$bpc PLANES_QUICK=1 PLANES_DTYPES=float64,int64 timeout -k 10 120 python3 -u tools/probe_planes.py >> $OUT/planes.jsonl 2>> $OUT/planes.err || exit 1
done; done
