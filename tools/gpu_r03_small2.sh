# GPU box: parity of the changed fold (config tests, parity, multi, pool, fault), then small-launch timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03small2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_pool.py tests/test_gpu_fault.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probe_timeline.py > $OUT/timeline.json 2>>$OUT/err.log || exit 1
timeout -k 10 120 python -u tools/probe_small.py > $OUT/small.jsonl 2>>$OUT/err.log || exit 1
timeout -k 10 300 python3 -u bench.py --no-c4 --no-inflate --no-f64 --no-host --no-cpu-baseline --steps 100 --warmup 10 > $OUT/bench.json 2>>$OUT/err.log || exit 1
