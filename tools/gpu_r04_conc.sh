# GPU box (round 4): the coalescer's idle-queue fast path and the pool tests, then the native concurrency
# legs: C1 / C3 resident at 1 / 15 / 60 threads, 1 MiB host chunks through rdx_execute_owned at 1 / 15 threads,
# and the direct (own workspace + synchronize) form at 1 thread for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r04conc}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pool.py tests/test_gpu_epoch.py > $OUT/pytest_pool.txt 2>&1 || { tail -30 $OUT/pytest_pool.txt; exit 1; }
tail -3 $OUT/pytest_pool.txt
for rep in 1 2; do
  for cfg in c1 c3; do
    timeout -k 10 60 $B $cfg 1 2000 device >> $OUT/conc.jsonl || exit 1
    for t in 1 15 60; do
      timeout -k 10 60 $B $cfg $t 2000 resident >> $OUT/conc.jsonl || exit 1
    done
  done
  for t in 1 15; do
    timeout -k 10 60 $B s1 $t 2000 owned >> $OUT/conc.jsonl || exit 1
    RDX_DIRECT_MAX=0 timeout -k 10 60 $B s1 $t 2000 owned >> $OUT/conc.jsonl || exit 1
  done
  for d in 0 2 4; do
    RDX_DIRECT_MAX=$d timeout -k 10 60 $B c1 15 2000 resident >> $OUT/conc_direct_sweep.jsonl || exit 1
    RDX_DIRECT_MAX=$d timeout -k 10 60 $B c3 15 2000 resident >> $OUT/conc_direct_sweep.jsonl || exit 1
  done
done
cat $OUT/conc.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d['path'][:22], d['threads'], d['us_per_request_aggregate'], d['roofline_frac'], d['direct_requests'], d['coalesced_requests'], d['cpu_cores_busy'], d['errors'])"
