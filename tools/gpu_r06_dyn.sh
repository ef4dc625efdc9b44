# Round 6: the dynamic tail of k_all_contig (RDX_DYN_TAIL per mille of each chunk's tiles handed out at run time
# in pieces of RDX_DYN_PIECE tiles) against the static split, on the headline batch (8 x 64 MiB), the single
# 64 MiB chunk, C4 and the f64 legs; interleaved settings, two reps, bench.py's own legs; then the GPU tests of
# the all-axes path with the tail forced on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06dyn}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "0 4 32" "100 4 8" "150 2 8" "200 4 8"; do
    set -- $cfg
    RDX_DYN_TAIL=$1 RDX_DYN_PIECE=$2 RDX_DYN_MIN_TILES=$3 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-inflate --no-configs --no-host --full-out $OUT/bench_t$1_p$2_$rep.json > $OUT/bench_t$1_p$2_$rep.line 2>> $OUT/bench.err || exit 1
  done
done
RDX_DYN_TAIL=150 RDX_DYN_PIECE=2 RDX_DYN_MIN_TILES=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_dyn.log 2>&1 || exit 1
