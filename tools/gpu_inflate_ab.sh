set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/z3
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/z3/pytest.log 2>&1 &&
RDX_LIB_PATH=$PWD/reductionist-rs_amd/librdx_r4k.so timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/z3/pytest_r4k.log 2>&1 &&
timeout -k 10 400 python tools/bench_inflate.py > gpurun_out/z3/bench.log 2>&1 &&
RDX_LIB_PATH=$PWD/reductionist-rs_amd/librdx_r4k.so timeout -k 10 400 python tools/bench_inflate.py > gpurun_out/z3/bench_r4k.log 2>&1
