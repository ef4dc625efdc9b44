# GPU box: k_pinf_find variants (tools/probe_pinf_find.hip) on the bench chunk and an integer-valued chunk
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-r04find}
mkdir -p $OUT
python3 - <<'PY'
import numpy as np, zlib
rng = np.random.default_rng(0x5EED2000)
v = rng.standard_normal(1 << 20).astype(np.float32)
raw = v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
c = zlib.compressobj(1, zlib.DEFLATED, 15); open("/tmp/c0.zlib", "wb").write(c.compress(raw) + c.flush())
raw = np.random.default_rng(3).integers(-8, 9, 1 << 20).astype(np.float32).tobytes()
open("/tmp/c3.zlib", "wb").write(zlib.compress(raw, 1))
PY
for f in c0 c3; do
  echo "== $f"; timeout -k 10 60 tools/probe_pinf_find /tmp/$f.zlib | tee -a $OUT/find_$f.jsonl || exit 1
done
