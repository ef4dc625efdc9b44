set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 &&
bash tools/sweep_small.sh &&
timeout -k 10 900 python tools/bench_configs.py --no-cpu > gpurun_out/cfg2.log 2>&1
