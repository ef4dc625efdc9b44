# Round 5: k_cbor_pack without per-workgroup fences (tagged tile lengths); the sliceless column probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05cb2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_cbor.py > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do for st in 1 0; do
RDX_CBOR_STAGED=$st timeout -k 10 200 python3 -u tools/probe_cbor.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_cbor.py > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 120 tools/probe_cols2 > $OUT/cols2.jsonl 2> $OUT/cols2.err
rc=$?
tail -2 $OUT/pytest.log
exit $rc
