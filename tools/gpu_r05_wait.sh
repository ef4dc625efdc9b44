# Round 5: host-wait primitives and host-memory reads (tools/probe_hostwait).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05w2}
mkdir -p $OUT
timeout -k 10 200 tools/probe_hostwait 1 > $OUT/wait.jsonl 2>&1 &&
timeout -k 10 200 tools/probe_hostwait 4 > $OUT/wait_blockingsync.jsonl 2>&1 &&
ROC_ACTIVE_WAIT_TIMEOUT=0 timeout -k 10 200 tools/probe_hostwait 1 > $OUT/wait_awt0.jsonl 2>&1 &&
timeout -k 10 200 tools/probe_hostwait 2 > $OUT/hread.jsonl 2>&1
