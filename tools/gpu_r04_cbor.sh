# GPU box: k_cbor variants (look-back polls before the one-round-trip fallback) — the device-encoder tests on
# the first variant, then bench.py's cbor leg per library, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-r04cbor}
mkdir -p $OUT
V=${VARIANTS:-base}
first=${V%% *}; [ "$first" = base ] && first=""
RDX_LIB_PATH=$PWD/reductionist-rs_amd/librdx$first.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cbor.py -x -q --timeout 100 --timeout-method thread > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for pass in 1 2; do
  for v in $V; do
    [ "$v" = base ] && v=""
    RDX_LIB_PATH=$PWD/reductionist-rs_amd/librdx$v.so timeout -k 10 200 python3 tools/probe_cbor.py 2>> $OUT/err.log | python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), lib='librdx$v', p=$pass))) for l in sys.stdin]" >> $OUT/sweep.jsonl || exit 1
  done
done
python3 - $OUT/sweep.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["lib"], r["p"], {k: (v.get("us_per_call"), v.get("roofline_frac")) for k, v in r["r"].items() if isinstance(v, dict) and "us_per_call" in v})
PY
