# GPU box: full -m gpu suite, hand-off A/B (fold-by-last-block vs arrival counters), coalesced concurrency.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03iter}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit 1
RDX_FOLD_LAST=0 timeout -k 10 200 python -u tools/probe_handoff.py > $OUT/handoff.jsonl 2>>$OUT/handoff.err &&
RDX_FOLD_LAST=1 timeout -k 10 200 python -u tools/probe_handoff.py >> $OUT/handoff.jsonl 2>>$OUT/handoff.err || exit 1
export RDX_DISPATCH_STATS=1
for cfg in c1 c3; do
  timeout -k 10 60 $B $cfg 15 2000 device >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 1 2000 resident >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 1 >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 2 >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 3 >> $OUT/conc.jsonl 2>>$OUT/conc.err || exit 1
done
