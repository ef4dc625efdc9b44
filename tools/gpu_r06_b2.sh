# Round 6: blosc2 LZ decode occupancy.  k_blosc2_decode holds 40 KiB of LDS per workgroup (an 8 KiB output ring
# + 2 KiB input ring per wave), so 4 workgroups = 16 waves per CU run the serial token chains.  Variants (only
# k_blosc2.o differs): b2r4 = 4 KiB rings (5 workgroups per CU by VGPRs), b2r4w6 / b2r4w8 = 4 KiB + 1 KiB rings
# and the compiler asked for 6 / 8 waves per SIMD.  bench.py's decompression legs, interleaved, two reps; then
# the blosc2 GPU tests on each variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06b2}
mkdir -p $OUT
for rep in 1 2; do for lib in librdx.so librdx_b2r4.so librdx_b2r4w6.so librdx_b2r4w8.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --no-f64 --no-configs --no-host --full-out '' > $OUT/bench_${lib%.so}_$rep.line 2>> $OUT/bench.err || exit 1
done; done
for lib in librdx_b2r4.so librdx_b2r4w6.so librdx_b2r4w8.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_blosc2.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_${lib%.so}.log 2>&1 || exit 1
done
