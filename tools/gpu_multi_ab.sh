#!/bin/bash
# A/B of k_multi builds / fill targets: kernel durations per case (tools/probe_multi_kernel.py; case order:
# 20 x C3 multi, 20 x C3 batch, 20 x C1 multi, 20 x C1 batch, 10+10 mixed multi).  Every variant is a
# complete, correct build (same results), differing only in tuning.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-librdx librdx_k4}; do
  for b in ${BPCS:-4 5 8}; do
    RDX_LIB_PATH=reductionist-rs_amd/$v.so RDX_MULTI_BLOCKS_PER_CU=$b timeout -k 10 100 rocprofv3 --kernel-trace -d gpurun_out/prof_ab_${v}_$b -o mk -- python3 tools/probe_multi_kernel.py 20 > gpurun_out/prof_ab_${v}_$b.log 2>&1 || { echo "FAILED $v $b"; exit 1; }
    echo "== $v bpc $b"; python3 tools/kstats_by_case.py gpurun_out/prof_ab_${v}_$b/mk_results.db | grep -E "k_multi"
  done
done
