# Sweep of the blocks-per-CU fill target x tiles in flight for the contiguous kernel (headline
# batched C2 + single chunk).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-bpcu}
mkdir -p $OUT
for u in 2; do
for b in ${RDX_BPCU_LIST:-1 2 4}; do
  RDX_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-c4 --steps 200 --warmup 20 > $OUT/bench_${b}_$u.log 2>&1 || exit 1
done
done
