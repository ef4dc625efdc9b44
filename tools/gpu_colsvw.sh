# Cols lane width x separate fold launch sweep (axis probe, cols configs), plus the f64 bench legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/colsvw.log
: > $OUT
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-c4 --no-inflate --no-cpu-baseline > gpurun_out/bench_f64.log 2>&1 || exit 1
for cfg in "" "RDX_AXIS_FOLD_SEP=1" "RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_SEP=1" "RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_SEP=0" \
           "RDX_AXIS_COLS_VW=4 RDX_AXIS_FOLD_SEP=1 RDX_AXIS_PROBE=2" "RDX_AXIS_COLS_VW=2 RDX_AXIS_FOLD_SEP=1 RDX_AXIS_PROBE=2" \
           "RDX_AXIS_COLS_VW=1 RDX_AXIS_FOLD_SEP=1 RDX_AXIS_PROBE=2"; do
  echo "== $cfg" >> $OUT
  env $cfg timeout -k 10 120 python tools/probe_axis.py --cols >> $OUT 2>&1 || exit 1
done
