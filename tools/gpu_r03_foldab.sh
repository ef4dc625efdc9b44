# GPU box: the wave-fold variants A/B in one session (tools/probe_small.py per library, two rounds interleaved):
# 7f5de6f per-granule polls, fad87ec batched re-reads, 3fbdc4e + backoff by retry, cc19410 + granule-major,
# librdx (HEAD) backoff by the number of waiting lanes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03foldab}
mkdir -p $OUT
for r in 1 2; do
  for v in _7f5de6f _fad87ec _3fbdc4e _cc19410 ""; do
    RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 120 python -u tools/probe_small.py 2>>$OUT/err.log | sed "s/\"bpc\": \"auto\"/\"lib\": \"librdx$v\", \"round\": $r/" >> $OUT/foldab.jsonl || exit 1
  done
done
