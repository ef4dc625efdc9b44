# Round 5: the rows kernel with 16 loads in flight for long rows (RDX_AXIS_ROWS_DEEP, librdx.so) against 4
# (librdx_shallow.so) on the axis configs, then smoke() and the full -m gpu suite on librdx.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05rows}
mkdir -p $OUT
for rep in 1 2; do for lib in librdx.so librdx_shallow.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 120 python3 -u tools/probe_axis.py 2>> $OUT/axis.err | sed "s/^{/{\"lib\": \"$lib\", /" >> $OUT/axis.jsonl || exit 1
done; done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
exit $rc
