# Round 6: do FEWER concurrent plane streams help byte-shuffled f64?  8 planes per workgroup x 256 workgroups =
# 2048 concurrent DRAM streams (f32: 1024, plain: 256); forcing 16 / 24 workgroups per chunk (128 / 192 in all)
# halves / cuts them at the price of idle CUs.  bench.py's f64 and C2 legs under RDX_FORCE_BPC, interleaved, 2 reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06f64bpc}
mkdir -p $OUT
for rep in 1 2; do for bpc in 0 16 24 32; do
  if [ $bpc = 0 ]; then E=""; else E="RDX_FORCE_BPC=$bpc"; fi
  env $E timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-c4 --no-inflate --no-configs --no-host --full-out '' > $OUT/bench_bpc${bpc}_$rep.line 2>> $OUT/bench.err || exit 1
done; done
