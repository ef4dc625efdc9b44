set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python tools/probe_axis.py > gpurun_out/probe_axis.log 2>&1 &&
timeout -k 10 120 python tools/probe_small.py > gpurun_out/probe_small.log 2>&1 &&
timeout -k 10 900 python tools/bench_configs.py --no-cpu > gpurun_out/cfg3.log 2>&1
