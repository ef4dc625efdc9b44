# Parity tests, then per-config measurements, then the same measurements under a kernel trace
# (kernel durations vs event-timed per-call durations tell launch-bound from host-bound).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/cfg.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cfgprof -o run --output-format csv -- python3 tools/bench_configs.py --no-cpu > gpurun_out/cfgprof.log 2>&1
