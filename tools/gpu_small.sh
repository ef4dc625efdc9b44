# Small-launch configs (C1, C3) across the k_all fill knobs.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/small.log
: > $OUT
for kn in "RDX_MIN_TILES_PER_BLOCK=2" "RDX_MIN_TILES_PER_BLOCK=1" "RDX_MIN_TILES_PER_BLOCK=4" "RDX_MIN_TILES_PER_BLOCK=8" "RDX_BLOCKS_PER_CU=2"; do
  env $kn timeout -k 10 300 python tools/bench_configs.py 2>/dev/null | grep '"c1_\|"c3_' | sed "s/^/$kn /" >> $OUT || exit 1
done
