# Concurrent single-chunk requests: streams / workspaces in flight.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/conc.log
: > $OUT
for n in 1 2 3 4 6 8; do
  echo "== RDX_BENCH_STREAMS=$n" >> $OUT
  RDX_BENCH_STREAMS=$n timeout -k 10 200 python bench.py --steps 2000 --warmup 20 --no-c4 --no-inflate --no-cpu-baseline --no-f64 >> $OUT 2>&1 || exit 1
done
