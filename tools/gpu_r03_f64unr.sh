# GPU box: f64 shuffled sums — tiles in flight per lane (RDX_UNR_F8 1/2/3/4 builds) x workgroups per CU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03f64unr}
mkdir -p $OUT
for v in "" _u1 _u3 _u4; do
  for b in 1 2; do
    RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so RDX_BLOCKS_PER_CU=$b timeout -k 10 200 python -u tools/probe_f64.py 2>>$OUT/err.log | python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), lib='librdx$v', bpcu=$b))) for l in sys.stdin if '\"float64\"' in l and ('sum' in l or 'min' in l)]" >> $OUT/f64unr.jsonl || exit 1
  done
done
