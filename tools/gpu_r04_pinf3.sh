# GPU box: the pinflate GPU tests alone, each test under its own time limit, RDX_PINF_PROF=1 so that any
# stream the parallel path declines says why on stderr (captured per test by pytest).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r04pinf3}
mkdir -p $OUT
RDX_PINF_PROF=1 timeout -k 10 240 python -u -m pytest -x -v -rA --timeout 60 --timeout-method thread tests/test_gpu_pinflate.py > $OUT/pytest_pinf.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_pinf.txt | tail -30
grep -h "pinf_declined" $OUT/pytest_pinf.txt | sort | uniq -c | head -20
exit $rc
