# GPU box: dispatcher timing + kernel trace of the coalesced resident path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-poolprof}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
export RDX_DISPATCH_STATS=1
for l in 1 2; do
  timeout -k 10 60 $B c1 15 2000 resident 0 $l >> $OUT/conc.jsonl 2>>$OUT/conc.err || exit 1
  timeout -k 10 60 $B c1 1 2000 resident 0 $l >> $OUT/conc.jsonl 2>>$OUT/conc.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B c1 15 1000 resident 0 2 > $OUT/trace.log 2>&1
