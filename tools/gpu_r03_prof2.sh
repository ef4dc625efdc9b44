# GPU box: fault test (probe build) and kernel traces of the coalesced path (1 / 2 lanes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03prof2}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 300 python -u -m pytest tests/test_gpu_fault.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fault.log 2>&1 || exit 1
for l in 1 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace_l$l -o run --output-format csv -- $B c1 15 1000 resident 0 $l > $OUT/trace_l$l.log 2>&1 || exit 1
done
