# Round 5: k_pinf_find variants (tools/probe_pinf_find_<variant>) on the bench chunk and an integer-valued
# chunk; the rows kernel with more loads in flight (librdx_ru8 / _ru16) on the axis configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05fd}
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
for rep in 1 2; do for v in base nohdr spread; do for f in c4z1 intz6; do
  echo "{\"find_variant\": \"$v\", \"stream\": \"$f\"}" >> $OUT/find.jsonl
  timeout -k 10 60 tools/probe_pinf_find_$v /tmp/$f.zlib >> $OUT/find.jsonl 2>> $OUT/find.err || exit 1
done; done; done
for lib in librdx.so librdx_ru8.so librdx_ru16.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 120 python3 -u tools/probe_axis.py >> $OUT/axis.jsonl 2>> $OUT/axis.err || exit 1
done
