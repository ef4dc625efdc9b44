# Blocks-per-chunk sweep for the small single-chunk configs (tools/probe_small.py), one process each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sweep_small.log
: > $OUT
for b in 0 16 32 64 128 256 512 1024; do
  if [ $b = 0 ]; then
    timeout -k 10 120 python tools/probe_small.py >> $OUT 2>&1 || exit 1
  else
    RDX_FORCE_BPC=$b timeout -k 10 120 python tools/probe_small.py >> $OUT 2>&1 || exit 1
  fi
done
