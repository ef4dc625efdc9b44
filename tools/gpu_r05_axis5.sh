# Round 5: axis kernels with strength-reduced offsets and pinned load registers (no loads sunk into the
# clamped-row branches): parity, times, kernel stats (default and streaming-only probe builds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05ax5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multi.py > $OUT/pytest_axis.log 2>&1 || exit 1
for rep in 1 2; do
timeout -k 10 120 python3 -u tools/probe_axis.py >> $OUT/axis.jsonl 2>> $OUT/axis.err || exit 1
RDX_AXIS_COLS_VW=4 timeout -k 10 120 python3 -u tools/probe_axis.py --cols >> $OUT/axis_vw4.jsonl 2>> $OUT/axis.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/axtrace -o run --output-format csv -- python3 tools/probe_axis.py > $OUT/axtrace.log 2>&1 || exit 1
RDX_LIB_PATH=reductionist-rs_amd/librdx_probe.so RDX_AXIS_PROBE=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/axtrace2 -o run --output-format csv -- python3 tools/probe_axis.py --cols > $OUT/axtrace2.log 2>&1 &&
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -1 $OUT/pytest_axis.log
exit $rc
