# Round 5: the staged CBOR count array (pack -> place) against agg / scan / encode; parity tests; kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05cb}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_cbor.py > $OUT/pytest.log 2>&1 &&
for rep in 1 2; do for st in 1 0; do
RDX_CBOR_STAGED=$st timeout -k 10 200 python3 -u tools/probe_cbor.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done; done &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_cbor.py > $OUT/trace.log 2>&1
rc=$?
[ $rc -eq 0 ] && { timeout -k 10 120 tools/probe_f64lds > $OUT/f64lds.jsonl 2> $OUT/f64lds.err; rc=$?; }
[ $rc -eq 0 ] && { timeout -k 10 60 tools/probe_cols random > $OUT/cols.txt 2>&1 && timeout -k 10 60 tools/probe_cols >> $OUT/cols.txt 2>&1; rc=$?; }
for vw in 2 4; do for pr in 0 2; do
[ $rc -eq 0 ] && { RDX_LIB_PATH=reductionist-rs_amd/librdx_probe.so RDX_AXIS_PROBE=$pr RDX_AXIS_COLS_VW=$vw timeout -k 10 120 python3 -u tools/probe_axis.py --cols >> $OUT/axis.jsonl 2>> $OUT/axis.err; rc=$?; }
done; done
tail -2 $OUT/pytest.log
exit $rc
