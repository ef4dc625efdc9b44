# Inflate ring size x waves per workgroup, field and noise, 1024 and 2048 streams.  Measured with
# per-variant probe_inflate builds before the ring became a per-launch choice (RDX_INFLATE_RING forces
# one now: see tools/gpu_ringsel.sh); kept as the record of that sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ring.log
: > $OUT
for v in 8192_4 16384_4 16384_2 32768_2; do for k in field noise; do for n in 1024 2048; do
  echo "== $v" >> $OUT
  timeout -k 10 120 ./tools/build/probe_inflate_$v $k 1 $n 2 >> $OUT 2>&1 || exit 1
done; done; done
