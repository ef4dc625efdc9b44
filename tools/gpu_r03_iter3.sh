# GPU box: full -m gpu suite, phase timelines, hand-off probe, concurrency (coalesced).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03iter3}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probe_timeline.py > $OUT/timeline.json 2>>$OUT/timeline.err || exit 1
timeout -k 10 200 python -u tools/probe_handoff.py > $OUT/handoff.jsonl 2>>$OUT/handoff.err || exit 1
for cfg in c1 c3; do
  timeout -k 10 60 $B $cfg 15 2000 resident >> $OUT/conc.jsonl 2>/dev/null || exit 1
done
