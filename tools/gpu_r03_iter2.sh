# GPU box: full -m gpu suite, then the coalesced resident path (grouped launches) for C1 / C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03iter2}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit 1
export RDX_DISPATCH_STATS=1
for cfg in c1 c3 c4; do
  for l in 1 2 3; do
    timeout -k 10 60 $B $cfg 15 2000 resident 0 $l > $OUT/one.json 2>$OUT/one.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/one.json')); d['lanes']=$l; e=[json.loads(x) for x in open('$OUT/one.err') if 'rdx_dispatch' in x]; d['dispatch']=e[-1]['rdx_dispatch'] if e else None; print(json.dumps(d))" >> $OUT/conc.jsonl
  done
  timeout -k 10 60 $B $cfg 1 2000 resident >> $OUT/conc1.jsonl 2>/dev/null || exit 1
done
