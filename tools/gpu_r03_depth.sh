# GPU box: coalescer launch-ahead A/B (RDX_COALESCE_DEPTH 1 / 2) x lanes, C1 / C3 at 15 threads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03depth}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
for cfg in c1 c3; do
  for d in 1 2; do
    for l in 2 4 6; do
      RDX_COALESCE_DEPTH=$d RDX_WAIT_SPIN=0 RDX_DISPATCH_STATS=1 timeout -k 10 60 $B $cfg 15 2000 resident 0 $l > $OUT/tmp.json 2>$OUT/tmp.err || exit 1
      python3 -c "import json,sys; r=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1]); s=[json.loads(l) for l in open('$OUT/tmp.err') if l.startswith('{')]; r.update(depth=$d, lanes=$l, dispatch=s[-1]['rdx_dispatch'] if s else None); print(json.dumps(r))" >> $OUT/depth.jsonl || exit 1
    done
  done
done
