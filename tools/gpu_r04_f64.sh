# GPU box: f64 shuffled sums — tile orders (product, RDX_TILE_STRIDE, RDX_TILE_ROT builds), two passes each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r04f64}
mkdir -p $OUT
for pass in 1 2; do
  for v in ${VARIANTS:-base _ts _rot}; do
    [ "$v" = base ] && v=""
    RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py 2>>$OUT/err.log | python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), lib='librdx$v', p=$pass))) for l in sys.stdin if '\"float64\"' in l or 'float32' in l]" >> $OUT/f64.jsonl || exit 1
  done
done
python3 - $OUT/f64.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
for r in rows:
    k = tuple((kk, r[kk]) for kk in sorted(r) if kk not in ("us", "us_per_launch", "GiBs", "frac", "roofline_frac", "p", "lib") and not isinstance(r[kk], float))
    agg[(r["lib"],) + k].append(r.get("us_per_launch", r.get("us")))
for k, v in sorted(agg.items()):
    print(k, v)
PY
