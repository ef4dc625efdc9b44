set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/r1_smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/r1_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/r1_bench.log 2>&1
