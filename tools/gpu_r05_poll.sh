# Round 5: the fold_last folder's polling (RDX_FOLD_POLL_SHORT): small single launches (C1, C3, C2 one chunk,
# mixed) from bench.py's own legs, short polls (librdx.so) against the long back-off (librdx_longpoll.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05poll}
mkdir -p $OUT
for rep in 1 2; do for lib in librdx.so librdx_longpoll.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c4 --no-inflate --no-f64 --no-host > $OUT/bench_${lib%.so}_$rep.json 2>> $OUT/bench.err || exit 1
done; done
