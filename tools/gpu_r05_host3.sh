# Round 5: host-memory requests, third pass — completion by event queries (no stream queries), the
# coalesced host path's phases (wall and caller CPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05h3}
mkdir -p $OUT
B=reductionist-rs_amd/rdx_conc_bench
timeout -k 10 60 $B s1 1 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
timeout -k 10 120 $B c4 15 300 host >> $OUT/conc.jsonl &&
RDX_PHASES=1 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc_ph.jsonl 2>> $OUT/phases.jsonl &&
RDX_PHASES=1 RDX_HOST_READ_KIB=0 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc_ph.jsonl 2>> $OUT/phases.jsonl &&
RDX_WAIT_SPIN=0 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl &&
RDX_DISPATCH_IDLE_US=2 timeout -k 10 120 $B s1 15 2000 owned >> $OUT/conc.jsonl
