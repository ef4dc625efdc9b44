# GPU box: coalesced resident path vs callers / lanes / wait mode, a kernel trace, and f64 UNR variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03conc2}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
export RDX_DISPATCH_STATS=1
for cfg in c1 c3; do
 for spin in 0 200; do
  for l in 2 3; do
    for t in 15 31 63; do
      RDX_WAIT_SPIN=$spin timeout -k 10 60 $B $cfg $t 1000 resident 0 $l > $OUT/one.json 2>$OUT/one.err || exit 1
      python3 -c "import json,sys; d=json.load(open('$OUT/one.json')); d['spin']=$spin; d['lanes']=$l; e=[json.loads(x) for x in open('$OUT/one.err') if 'rdx_dispatch' in x]; d['dispatch']=e[-1]['rdx_dispatch'] if e else None; print(json.dumps(d))" >> $OUT/conc.jsonl
    done
  done
 done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B c1 15 1000 resident 0 2 > $OUT/trace.log 2>&1 || exit 1
for v in "" _u4 _u6; do
  RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64$v.jsonl 2>$OUT/f64$v.err || exit 1
done
