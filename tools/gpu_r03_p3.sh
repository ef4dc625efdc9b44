# GPU box: full -m gpu suite (snappy, f64 multi-accumulator sums, tree min/max, W-capped axis tiles),
# then the f64 / axis probes and the coalescer's caller-spin sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03p3}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64.jsonl 2>>$OUT/f64.err || exit 1
timeout -k 10 120 python -u tools/probe_axis.py > $OUT/axis.jsonl 2>>$OUT/axis.err || exit 1
for cfg in c1 c3; do
  for sp in 0 2000 20000 200000; do
    for l in 2 3; do
      RDX_WAIT_SPIN=$sp RDX_DISPATCH_STATS=1 timeout -k 10 60 $B $cfg 15 2000 resident 0 $l >> $OUT/conc.jsonl 2>>$OUT/conc_stats.jsonl || exit 1
    done
  done
done
