# Round 5: f64 byte-shuffled sums — plane spacing and workgroups per chunk.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05pl}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/probe_planes.py > $OUT/planes.jsonl 2> $OUT/planes.err &&
for b in 16 24 48 64; do RDX_FORCE_BPC=$b timeout -k 10 200 python3 -u tools/probe_planes.py >> $OUT/planes_bpc.jsonl 2>> $OUT/planes.err || exit 1; done
