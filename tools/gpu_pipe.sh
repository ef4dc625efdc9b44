# k_all_contig pipelining A/B: variant probe, headline bench (primary only), then parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/probe_f64.py > gpurun_out/probe_pipe.log 2>&1 &&
timeout -k 10 300 python bench.py --primary-only --steps 400 --warmup 40 > gpurun_out/bench_pipe.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_pytest.log 2>&1
