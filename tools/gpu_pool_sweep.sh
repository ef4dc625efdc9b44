# k_all_contig dynamic-pool A/B on the GPU box: parity first, then the C2 legs of bench.py per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-pool}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
for cfg in "0 2" "4 2" "8 2" "12 2" "16 2" "8 1" "8 4" "12 4"; do
  set -- $cfg
  RDX_POOL_PCT=$1 RDX_POOL_PIECE_TILES=$2 timeout -k 10 200 python3 bench.py --no-c4 --no-inflate --no-f64 --no-configs --no-host --no-cpu-baseline --steps 300 --warmup 30 > $OUT/bench_$1_$2.json 2>> $OUT/bench.err || exit 1
done
timeout -k 10 200 python3 tools/probe_timeline.py > $OUT/timeline.json 2>> $OUT/bench.err
