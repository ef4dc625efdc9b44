# Round 5: host-memory requests — non-spinning waits, the direct host-read path, phase records; the GPU
# tests these touch.  Stops at the first failing step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05h}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_host.py tests/test_gpu_pinflate.py tests/test_gpu_pool.py "tests/test_gpu_configs.py::test_f64_sum_cancellation" \
  tests/test_gpu_inflate.py > $OUT/pytest.log 2>&1 &&
for cfg in s1 c1 h4f32 h4f64; do
  RDX_PHASES=1 timeout -k 10 60 $B $cfg 1 2000 owned >> $OUT/conc.jsonl 2>> $OUT/phases.jsonl || exit 1
  RDX_PHASES=1 RDX_HOST_READ_KIB=0 timeout -k 10 60 $B $cfg 1 2000 owned >> $OUT/conc_dma.jsonl 2>> $OUT/phases_dma.jsonl || exit 1
done &&
timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c4 15 300 host >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c1 15 2000 resident >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c3 15 2000 resident >> $OUT/conc.jsonl &&
for idle in 5 100; do
  RDX_DISPATCH_IDLE_US=$idle timeout -k 10 120 $B s1 15 2000 owned >> $OUT/idle_sweep.jsonl || exit 1
  RDX_DISPATCH_IDLE_US=$idle timeout -k 10 120 $B c1 15 2000 resident >> $OUT/idle_sweep.jsonl || exit 1
done
rc=$?
tail -3 $OUT/pytest.log
exit $rc
