# Round 6: C3 with 8 vectors in flight per lane in half the workgroups (librdx_ku8.so: only k_all_f64.o differs,
# RDX_FORCE_BPC=168 = one round per lane) against 4 per lane in 336 workgroups (librdx.so); tools/probe_small.py
# (the c3_min / c3_sum lines), interleaved, three reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06ku8}
mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 120 python3 -u tools/probe_small.py 2>> $OUT/err | sed "s/^{/{\"lib\": \"default\", \"rep\": $rep, /" >> $OUT/small.jsonl || exit 1
  RDX_LIB_PATH=reductionist-rs_amd/librdx_ku8.so RDX_FORCE_BPC=168 timeout -k 10 120 python3 -u tools/probe_small.py 2>> $OUT/err | sed "s/^{/{\"lib\": \"ku8_bpc168\", \"rep\": $rep, /" >> $OUT/small.jsonl || exit 1
done
