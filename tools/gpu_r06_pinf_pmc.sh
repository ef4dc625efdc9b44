# Round 6: what bounds k_pinflate's block / emit / find kernels on the bench chunk: rocprofv3 --pmc passes of
# issue / wait / LDS / store / instruction-cache counters over tools/probe_pinflate.py (the zlib-1 bench chunk,
# 3 decodes), one pass per counter group (tools/pmc_pinf_summary.py sums them per kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06pinfpmc}
mkdir -p $OUT
L=${PINF_LIB:-$PWD/reductionist-rs_amd/librdx.so}
export RDX_LIB_PATH=$L
step() {   # $1 = name, $2 = seconds, rest = command
  local name=$1 secs=$2; shift 2
  timeout -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "{\"step\": \"$name\", \"rc\": $rc}" >> $OUT/steps.jsonl
  if [ $rc -gt 1 ]; then exit $rc; fi
}
P="python3 tools/probe_pinflate.py 3 c4_shuffled_normal_f32_zlib1"
step sq1 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/sq1 -o run --output-format csv -- $P
step sq2 90 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA -d $OUT/sq2 -o run --output-format csv -- $P
step sq3 90 rocprofv3 --pmc SQ_IFETCH SQC_ICACHE_MISSES SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM -d $OUT/sq3 -o run --output-format csv -- $P
step ta 90 rocprofv3 --pmc TA_BUSY_max TA_FLAT_WRITE_WAVEFRONTS_sum -d $OUT/ta -o run --output-format csv -- $P
exit 0
