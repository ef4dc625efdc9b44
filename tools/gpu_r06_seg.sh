# Round 6: odd XCDs stream the headline batch ~3 % slower than even ones in most launches
# (profiles/r06_xcd_stability.jsonl).  Does the slowness follow the XCD or the address range?  librdx_seg1.so:
# workgroup b streams segment b ^ 1 (odd XCDs get the even segments); librdx_seg2*.so: odd workgroups' ranges
# 3 % / 1.5 % shorter (their partners' longer).  bench.py's C2 legs, interleaved, three reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06seg}
mkdir -p $OUT
for rep in 1 2 3; do for lib in librdx.so librdx_seg1.so librdx_seg2.so librdx_seg2w15.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c4 --no-inflate --no-f64 --no-configs --no-host --full-out '' > $OUT/bench_${lib%.so}_$rep.line 2>> $OUT/bench.err || exit 1
done; done
