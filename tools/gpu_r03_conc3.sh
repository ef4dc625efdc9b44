# GPU box: where a coalesced request's time goes (RDX_DISPATCH_STATS: host launch cost, launch -> results
# seen, completion) for C1 / C3 at 15 threads and 1-4 lanes; then the axis-cols tile sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03conc3}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
for cfg in c1 c3; do
  for l in 1 2 3 4; do
    RDX_DISPATCH_STATS=1 timeout -k 10 60 $B $cfg 15 2000 resident 0 $l >> $OUT/conc.jsonl 2>>$OUT/conc_stats.jsonl || exit 1
  done
done
RDX_TAG=${RDX_TAG:-r03conc3} bash tools/gpu_r03_axisw.sh
