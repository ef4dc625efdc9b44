# Round 6: fold-last for launches of many chunks of one or two blocks each (RDX_FOLD_LAST_PAIRS=1: C4's 1024 x 4
# MiB, bpc 1; the f64 4 MiB leg's 128 chunks, bpc 2) against the arrival counters they use above kFoldLastChunks;
# bench.py legs, interleaved, two reps; then the config and parity tests with it on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06pairs}
mkdir -p $OUT
for rep in 1 2; do for v in 0 1; do
  RDX_FOLD_LAST_PAIRS=$v timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --c4-steps 20 --no-cpu-baseline --no-inflate --no-configs --no-host --full-out $OUT/bench_p${v}_$rep.json > $OUT/bench_p${v}_$rep.line 2>> $OUT/bench.err || exit 1
done; done
RDX_FOLD_LAST_PAIRS=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_pool.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_pairs.log 2>&1 || exit 1
