# Round 6: what bounds the axis kernels: kernel trace stats, then one rocprofv3 --pmc pass
# each of wave occupancy / issue-stall / VALU counters and of HBM traffic, over tools/pmc_axis.py.  A pass
# that ends in an ordinary error (an unknown counter name: rc 1) does not stop the others; a kill, abort or
# time limit does.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06axpmc}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
step() {   # $1 = name, $2 = seconds, rest = command
  local name=$1 secs=$2; shift 2
  timeout -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "{\"step\": \"$name\", \"rc\": $rc}" >> $OUT/steps.jsonl
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step trace 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/pmc_axis.py 20
step sq1 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/sq1 -o run --output-format csv -- python3 tools/pmc_axis.py 10
step sq2 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/sq2 -o run --output-format csv -- python3 tools/pmc_axis.py 10
step fetch 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/pmc_axis.py 10
step write 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/pmc_axis.py 10
exit 0
