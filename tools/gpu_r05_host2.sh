# Round 5: host-memory requests, second pass — the host-read grid sweep without phase events, and the
# 15-thread rows with a per-thread CPU breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05h2}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
for w in 2 4 6 8 12 16; do
  for cfg in s1 c1; do
    RDX_HOST_READ_WGS=$w timeout -k 10 60 $B $cfg 1 2000 owned >> $OUT/wgs_sweep.jsonl || exit 1
  done
done &&
for cfg in s1 c1 h4f32 h4f64; do
  timeout -k 10 60 $B $cfg 1 2000 owned >> $OUT/one.jsonl || exit 1
  RDX_HOST_READ_KIB=0 timeout -k 10 60 $B $cfg 1 2000 owned >> $OUT/one_dma.jsonl || exit 1
done &&
timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c4 15 300 host >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c1 15 2000 resident >> $OUT/conc.jsonl &&
RDX_HOST_READ_KIB=0 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
RDX_HOST_SPIN_US=0 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl
