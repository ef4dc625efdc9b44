# Round 6: order-free folds through atomics (RDX_FOLD_LAST=2, rdx_device.hpp atomic_fold) against the record
# fold (1): the GPU suite on the new default, then bench.py's small-launch legs, interleaved, two reps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06fold}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
fi
for rep in 1 2; do for fl in 2 1; do
  RDX_FOLD_LAST=$fl timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c4 --no-inflate --no-f64 --no-host --full-out $OUT/bench_fl${fl}_$rep.json > $OUT/bench_fl${fl}_$rep.line 2>> $OUT/bench.err || exit 1
done; done
