# Round 6: what bounds k_blosc2_decode (LZ4) and k_axis_cols: issue / stall counters, one rocprofv3 --pmc pass per
# group, over tools/pmc_b2.py and tools/pmc_axis.py.  An ordinary error (rc 1) does not stop the others; a kill does.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06b2pmc}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "{\"step\": \"$name\", \"rc\": $rc}" >> $OUT/steps.jsonl
  if [ $rc -gt 1 ]; then exit $rc; fi
}
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
B="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
step b2trace 120 rocprofv3 --kernel-trace --stats -d $OUT/b2trace -o run --output-format csv -- python3 tools/pmc_b2.py 5
step b2a 120 rocprofv3 --pmc $A -d $OUT/b2a -o run --output-format csv -- python3 tools/pmc_b2.py 3
step b2b 120 rocprofv3 --pmc $B -d $OUT/b2b -o run --output-format csv -- python3 tools/pmc_b2.py 3
step axa 90 rocprofv3 --pmc $A -d $OUT/axa -o run --output-format csv -- python3 tools/pmc_axis.py 10
step axb 90 rocprofv3 --pmc $B -d $OUT/axb -o run --output-format csv -- python3 tools/pmc_axis.py 10
exit 0
