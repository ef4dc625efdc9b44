# Round 5: randomised parity stress on the closing build (axis kernels' new load schedule, deep rows,
# staged CBOR untouched here): two seeds of tools/stress_parity.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05stress}
mkdir -p $OUT
for seed in 77 505; do
  timeout -k 10 500 python3 -u tools/stress_parity.py --cases 2000 --seed $seed >> $OUT/stress.jsonl 2>> $OUT/stress.err || exit 1
done
