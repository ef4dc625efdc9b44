# Inflate ring variants: parity under each forced ring, then throughput per batch size (auto vs 8 KiB).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ringsel
mkdir -p $OUT
for r in 8192 16384 32768; do
  RDX_INFLATE_RING=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$r.log 2>&1 || exit 1
done
for b in 256 512 1024 2048; do
  timeout -k 10 300 python tools/bench_inflate.py --batch $b --formats zlib > $OUT/auto_$b.log 2>&1 || exit 1
  RDX_INFLATE_RING=8192 timeout -k 10 300 python tools/bench_inflate.py --batch $b --formats zlib > $OUT/r8k_$b.log 2>&1 || exit 1
done
