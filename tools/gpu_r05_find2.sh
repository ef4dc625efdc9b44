# Round 5: the finder's survivor header decode through per-lane code tables (RDX_PINF_FIND_LUT) against
# the register form, then the single-stream inflate tests and the lone-stream probe on the product build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05fd2}
mkdir -p $OUT
python3 - <<'PY' || exit 1
import zlib, numpy as np
rng = np.random.default_rng(0x5EED2000)
v = rng.standard_normal(1 << 20).astype(np.float32)
sh = v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
ints = np.random.default_rng(3).integers(-8, 9, 1 << 20).astype(np.float32).tobytes()
for name, raw, lvl in (("c4z1", sh, 1), ("intz6", ints, 6)):
    open(f"/tmp/{name}.zlib", "wb").write(zlib.compress(raw, lvl))
PY
for rep in 1 2; do for v in lut nolut nohdr; do for f in c4z1 intz6; do
  echo "{\"find_variant\": \"$v\", \"stream\": \"$f\"}" >> $OUT/find.jsonl
  timeout -k 10 60 tools/probe_pinf_find_$v /tmp/$f.zlib >> $OUT/find.jsonl 2>> $OUT/find.err || exit 1
done; done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_pinflate.py tests/test_gpu_inflate.py > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/probe_pinflate.py > $OUT/pinflate_probe.jsonl 2> $OUT/pinflate_probe.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_pinflate.py 5 > $OUT/trace.log 2>&1 || exit 1
# axis kernels counting once per load (MK_NONE): parity, then times and kernel stats
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_configs.py > $OUT/pytest_axis.log 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/probe_axis.py > $OUT/axis.jsonl 2>> $OUT/axis.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/axtrace -o run --output-format csv -- python3 tools/probe_axis.py --cols > $OUT/axtrace.log 2>&1 || exit 1
RDX_LIB_PATH=reductionist-rs_amd/librdx_probe.so RDX_AXIS_PROBE=2 RDX_AXIS_COLS_VW=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/axtrace2 -o run --output-format csv -- python3 tools/probe_axis.py --cols > $OUT/axtrace2.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
exit $rc
