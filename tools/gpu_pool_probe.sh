# GPU box: the pool tests, then the native concurrency bench in its three paths (coalescer A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-pool}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_pool.log 2>&1 &&
for cfg in c1 c3; do
  timeout -k 10 60 $B $cfg 15 2000 device >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 1 2000 resident >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 1 >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 2 >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 3 >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
  timeout -k 10 60 $B $cfg 15 2000 resident 0 4 >> $OUT/conc.jsonl 2>>$OUT/conc.err || exit 1
done
timeout -k 10 60 $B c4 15 300 host >> $OUT/conc.jsonl 2>>$OUT/conc.err &&
timeout -k 10 60 $B c4 15 300 host 0,0 >> $OUT/conc.jsonl 2>>$OUT/conc.err
