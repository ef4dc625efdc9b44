# GPU box: k_all_contig tile order A/B (contiguous ranges vs grid-stride sweep) on the batched and single launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03ts}
mkdir -p $OUT
for v in "" _ts; do
  RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64$v.jsonl 2>$OUT/f64$v.err || exit 1
  RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_handoff.py > $OUT/handoff$v.jsonl 2>$OUT/handoff$v.err || exit 1
done
for v in "" _ts; do
  RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64${v}_2.jsonl 2>>$OUT/f64$v.err || exit 1
done
