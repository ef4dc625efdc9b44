# zstd sequence-reader variant: phase probe, batch / lone timing, the blosc2 GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-r03zs}
mkdir -p $OUT
RDX_LIB_PATH=$GRAFT_REPO_ROOT/reductionist-rs_amd/librdx_probe.so timeout -k 10 240 python3 -u tools/probe_zstd.py 64 65536 > $OUT/zprof.jsonl 2> $OUT/zprof.err &&
timeout -k 10 200 python3 -u tools/probe_blosc2.py 256 zstd > $OUT/probe_blosc2.jsonl 2> $OUT/probe_blosc2.err &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_blosc2.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_blosc2.log 2>&1
