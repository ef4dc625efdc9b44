# Round 5: shuffled 8-byte elements with the split-in-time plane loads (k_all RDX_F8_SPLIT) against the
# pipelined form, tiles in flight 1 / 2 / 4, 1 or 2 workgroups per CU; the CBOR pack fast path; parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05sp}
mkdir -p $OUT
L=reductionist-rs_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_cbor.py tests/test_gpu_configs.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
for lib in librdx.so librdx_nosplit.so librdx_s1.so librdx_s4.so; do
  PLANES_QUICK=1 PLANES_DTYPES=float64,int64 RDX_LIB_PATH=$L/$lib timeout -k 10 120 python3 -u tools/probe_planes.py >> $OUT/planes.jsonl 2>> $OUT/planes.err || exit 1
done
for lib in librdx.so librdx_s1.so; do
  RDX_FORCE_BPC=64 PLANES_QUICK=1 PLANES_DTYPES=float64 RDX_LIB_PATH=$L/$lib timeout -k 10 120 python3 -u tools/probe_planes.py >> $OUT/planes.jsonl 2>> $OUT/planes.err || exit 1
done
done
for st in 1 0; do
RDX_CBOR_STAGED=$st timeout -k 10 200 python3 -u tools/probe_cbor.py >> $OUT/cbor.jsonl 2>> $OUT/cbor.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_cbor.py > $OUT/trace.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/axtrace -o run --output-format csv -- python3 tools/probe_axis.py --cols > $OUT/axtrace.log 2>&1 &&
RDX_LIB_PATH=$L/librdx_probe.so RDX_AXIS_PROBE=2 RDX_AXIS_COLS_VW=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/axtrace2 -o run --output-format csv -- python3 tools/probe_axis.py --cols > $OUT/axtrace2.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
exit $rc
