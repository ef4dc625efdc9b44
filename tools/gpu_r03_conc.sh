# GPU box: the coalesced resident path across thread counts, lanes and caller wait modes; f64 variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03conc}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
export RDX_DISPATCH_STATS=1
for spin in 0 200 2000 20000; do
  for l in 1 2; do
    for t in 8 15; do
      RDX_WAIT_SPIN=$spin timeout -k 10 60 $B c1 $t 2000 resident 0 $l > $OUT/one.json 2>$OUT/one.err || exit 1
      python3 -c "import json,sys; d=json.load(open('$OUT/one.json')); d['spin']=$spin; d['lanes']=$l; e=[json.loads(x) for x in open('$OUT/one.err') if 'rdx_dispatch' in x]; d['dispatch']=e[-1]['rdx_dispatch'] if e else None; print(json.dumps(d))" >> $OUT/conc.jsonl
    done
  done
done
timeout -k 10 200 python -u tools/probe_batch_sizes.py > $OUT/batch_sizes.jsonl 2>$OUT/batch_sizes.err || exit 1
for v in "" _u1 _u3; do
  RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64$v.jsonl 2>$OUT/f64$v.err || exit 1
done
RDX_BLOCKS_PER_CU=2 timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64_bpcu2.jsonl 2>$OUT/f64_bpcu2.err
