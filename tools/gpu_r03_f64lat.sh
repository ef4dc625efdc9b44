# GPU box: f64 vs f32 batched all-axes variants at 1 / 2 workgroups per CU, and the small-launch latency
# probe (empty / load-only / hand-off variants, events over back-to-back launches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03f64lat}
mkdir -p $OUT
for b in 1 2; do
  RDX_BLOCKS_PER_CU=$b timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64_bpcu$b.jsonl 2>>$OUT/f64.err || exit 1
done
timeout -k 10 120 tools/probe_latency > $OUT/latency.txt 2>&1 || exit 1
