# Round 5: host-memory requests, fourth pass — coalesced host reads (no copy, no workspace lease).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05h4}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_host.py tests/test_gpu_pool.py > $OUT/pytest.log 2>&1 &&
timeout -k 10 60 $B s1 1 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c4 15 300 host >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c4 15 300 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c1 15 2000 resident >> $OUT/conc.jsonl &&
RDX_PHASES=1 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc_ph.jsonl 2>> $OUT/phases.jsonl
rc=$?
tail -3 $OUT/pytest.log
exit $rc
