# Round 6: k_pinflate phase times (RDX_PINF_PROF=1: the slowest workgroup of find / block / emit, phase by
# phase) for the product library and the A/B variants tools/build_pinf_variant.sh built (PINF_LIBS), on the
# bench chunk and the integer-valued / periodic streams; then rocprofv3 kernel stats of the product library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06pinf}
mkdir -p $OUT
CASES=${PINF_CASES:-shuffled_normal_f32_zlib,int_valued_f32_zlib,periodic_f32_zlib6}
for lib in default ${PINF_LIBS:-}; do
  if [ $lib = default ]; then L=$PWD/reductionist-rs_amd/librdx.so; else L=$PWD/reductionist-rs_amd/librdx_pv_$lib.so; fi
  RDX_LIB_PATH=$L timeout -k 10 180 python3 -u tools/probe_pinflate.py 10 $CASES 2> $OUT/prof_$lib.err | sed "s/^{/{\"lib\": \"$lib\", /" >> $OUT/probe.jsonl || exit 1
  RDX_LIB_PATH=$L RDX_PINF_PROF=1 timeout -k 10 180 python3 -u tools/probe_pinflate.py 3 $CASES > $OUT/prof_$lib.jsonl 2> $OUT/prof_$lib.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/probe_pinflate.py 5 $CASES > $OUT/rocprof.jsonl 2> $OUT/rocprof.err
