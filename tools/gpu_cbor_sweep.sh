# k_cbor on the GPU box: the device-encoder tests, then the cbor leg per workgroups-per-CU setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RDX_TAG:-cbor}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_cbor.py -x -q --timeout 100 --timeout-method thread > $OUT/t.log 2>&1 || exit 1
for b in 0; do
  RDX_CBOR_BLOCKS_PER_CU=$b timeout -k 10 200 python3 tools/probe_cbor.py >> $OUT/sweep.jsonl 2>> $OUT/err.log || exit 1
done
