# Round 5: f64 sums — pipelining, tiles in flight, per-element compensation, workgroups per CU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PLANES_QUICK=1
OUT=gpurun_out/${RDX_TAG:-r05f64}
mkdir -p $OUT
L=$PWD/reductionist-rs_amd
for rep in 1 2; do
for lib in librdx librdx_pipe1 librdx_pipe1u3 librdx_nogroup; do
  for b in 32 64; do
    RDX_LIB_PATH=$L/$lib.so RDX_FORCE_BPC=$b timeout -k 10 120 python3 -u tools/probe_planes.py >> $OUT/f64.jsonl 2>> $OUT/f64.err || exit 1
  done
done
done
