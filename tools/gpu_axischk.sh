# axis planner change: parity suite, then the default axis probe and the min/max probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/axischk_pytest.log 2>&1 &&
timeout -k 10 300 python tools/probe_axis.py > gpurun_out/axischk.log 2>&1 &&
timeout -k 10 300 python tools/probe_axis.py --minmax >> gpurun_out/axischk.log 2>&1
