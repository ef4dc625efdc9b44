# f64 legs vs the k_all_contig fill target (workgroups per CU).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/f64bpc.log
: > $OUT
for b in 1 2 3 4; do
  echo "== RDX_BLOCKS_PER_CU=$b" >> $OUT
  RDX_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-c4 --no-inflate --no-cpu-baseline >> $OUT 2>&1 || exit 1
done
