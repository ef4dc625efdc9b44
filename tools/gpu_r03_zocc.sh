# zstd decoder occupancy A/B: ring 4 KiB x 2 waves per workgroup (librdx), 8 KiB x 4 (librdx_zA, the previous
# form), 2 KiB x 2 (librdx_zC); batch / lone timing per library, the phase probe, then the blosc2 GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-r03zo}
mkdir -p $OUT
R=$GRAFT_REPO_ROOT/reductionist-rs_amd
for lib in librdx librdx_zA librdx_zC librdx librdx_zA; do
  RDX_LIB_PATH=$R/$lib.so timeout -k 10 200 python3 -u tools/probe_blosc2.py 256 zstd > $OUT/p_$lib.jsonl 2> $OUT/p_$lib.err || exit 1
  sed "s/^/$lib /" $OUT/p_$lib.jsonl >> $OUT/ab.txt
done
RDX_LIB_PATH=$R/librdx_probe.so timeout -k 10 240 python3 -u tools/probe_zstd.py 64 65536 > $OUT/zprof.jsonl 2> $OUT/zprof.err &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_blosc2.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_blosc2.log 2>&1
