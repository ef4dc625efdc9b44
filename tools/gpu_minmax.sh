# min/max change: parity suite, then the all-axes variant probe and the axis/strided min-max probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/minmax_pytest.log 2>&1 &&
timeout -k 10 300 python tools/probe_f64.py > gpurun_out/probe_minmax.log 2>&1 &&
timeout -k 10 300 python tools/probe_axis.py --minmax > gpurun_out/probe_minmax_axis.log 2>&1
