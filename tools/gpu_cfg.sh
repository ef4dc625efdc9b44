set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/cfg.log 2>&1
