# GPU box: phase timelines of the small launches (probe build) and grid sweeps for C1 / C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03small}
mkdir -p $OUT
timeout -k 10 200 python -u tools/probe_timeline.py > $OUT/timeline.json 2>>$OUT/err.log || exit 1
timeout -k 10 120 python -u tools/probe_small.py > $OUT/small.jsonl 2>>$OUT/err.log || exit 1
for b in 64 168 256 512; do
  RDX_FORCE_BPC=$b timeout -k 10 120 python -u tools/probe_small.py >> $OUT/small.jsonl 2>>$OUT/err.log || exit 1
done
RDX_MIN_TILES_PER_BLOCK=1 timeout -k 10 120 python -u tools/probe_small.py | sed 's/"bpc": "auto"/"bpc": "mintiles1"/' >> $OUT/small.jsonl 2>>$OUT/err.log || exit 1
