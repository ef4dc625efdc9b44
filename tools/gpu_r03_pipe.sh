# GPU box: software-pipelined sum loops A/B (k_all_contig), batched 8 x 64 MiB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03pipe}
mkdir -p $OUT
for rep in 1 2; do
  for v in "" _p1 _p2; do
    RDX_LIB_PATH=reductionist-rs_amd/librdx$v.so timeout -k 10 200 python -u tools/probe_f64.py > $OUT/f64${v}_$rep.jsonl 2>>$OUT/f64.err || exit 1
  done
done
