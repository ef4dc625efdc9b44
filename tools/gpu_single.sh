# Single-chunk vs batched C2 across the k_all_contig fill target (RDX_BLOCKS_PER_CU).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/single.log
: > $OUT
for b in 1 2 3 4; do
  RDX_BLOCKS_PER_CU=$b timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-c4 --no-inflate --no-cpu-baseline > gpurun_out/single_$b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/single_$b.log') if l.startswith('{')][-1]); print('bpcu', $b, d['value'], d['extra']['c2_single_chunk']['value'], d['extra']['c2_single_chunk']['kernel_us_avg'])" >> $OUT
done
