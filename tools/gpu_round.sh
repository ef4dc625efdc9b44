# Full round check on the GPU box: smoke, parity tests, bench, kernel-trace profile, PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r01}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --primary-only > $OUT/trace.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --primary-only > $OUT/pmc.log 2>&1
