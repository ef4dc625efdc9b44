# word-major cols records (in-kernel fold): parity suite, default + min/max axis probes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/soa.log
: > $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/soa_pytest.log 2>&1 &&
timeout -k 10 300 python tools/probe_axis.py >> $OUT 2>&1 &&
timeout -k 10 300 python tools/probe_axis.py --minmax >> $OUT 2>&1 &&
RDX_AXIS_FOLD_SEP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/soa_pytest.log 2>&1
