# Round 5: k_cbor_pack with the next tile's loads in flight while a tile is encoded; CBOR parity (incl. the
# unstaged form in a child process); times and kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05cb4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_cbor.py > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
timeout -k 10 200 python3 -u tools/probe_cbor.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_cbor.py > $OUT/trace.log 2>&1
rc=$?
tail -1 $OUT/pytest.log
exit $rc
