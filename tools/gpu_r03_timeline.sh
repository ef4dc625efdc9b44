# GPU box: phase timelines (probe build) of C2 single / batch, C3, C1 in both hand-off forms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03tl}
mkdir -p $OUT
for fl in 1 0; do
  RDX_FOLD_LAST=$fl timeout -k 10 200 python -u tools/probe_timeline.py > $OUT/timeline_fl$fl.json 2>>$OUT/timeline.err || exit 1
done
timeout -k 10 200 python -u tools/probe_handoff.py > $OUT/handoff.jsonl 2>>$OUT/handoff.err
