set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python tools/sweep2.py > gpurun_out/sweep2.log 2>&1 &&
timeout -k 10 300 python bench.py --cpu-seconds 3 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c4 > gpurun_out/prof_c2.log 2>&1
