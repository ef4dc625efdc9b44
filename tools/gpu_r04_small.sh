# GPU box: small single-launch latency (tools/probe_small.py: C1, C3, a C3-sized run) per library, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-r04small}
mkdir -p $OUT
for pass in 1 2; do
  for v in ${VARIANTS:-base}; do
    [ "$v" = base ] && v=""
    RDX_LIB_PATH=$PWD/reductionist-rs_amd/librdx$v.so timeout -k 10 200 python3 tools/probe_small.py 2>> $OUT/err.log | python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), lib='librdx$v', p=$pass))) for l in sys.stdin]" >> $OUT/small.jsonl || exit 1
  done
done
cat $OUT/small.jsonl
