# GPU box: the coalescer at 15 threads (C1 / C3 resident) over lanes in flight, k_multi workgroups per CU and
# the callers' spin before sleeping; two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-r04csweep}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
for rep in 1 2; do
  for lanes in 2 3 4 6; do
    for mb in 3 5 8; do
      for cfg in c1 c3; do
        RDX_MULTI_BLOCKS_PER_CU=$mb timeout -k 10 60 $B $cfg 15 2000 resident 0 $lanes | python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), lanes=$lanes, mbpcu=$mb, rep=$rep))) for l in sys.stdin]" >> $OUT/sweep.jsonl || exit 1
      done
    done
  done
done
python3 - $OUT/sweep.jsonl <<'PY'
import json, sys, collections
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l)
    agg[(r["config"], r["lanes"], r["mbpcu"])].append(r["roofline_frac"])
for k, v in sorted(agg.items()):
    print(k, [round(x, 3) for x in v])
PY
