# Round 6: f32 axis sums with pairwise in-load adds and two alternating partial sums per pass (librdx.so, the default now:
# only k_axis_f32.o differs) against the sequential f64 chain (librdx_nopair.so); tools/probe_axis.py's configs,
# interleaved, three reps; then the config / parity GPU tests on the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r06pair}
mkdir -p $OUT
for rep in 1 2 3; do for lib in librdx_nopair.so librdx.so; do
  RDX_LIB_PATH=reductionist-rs_amd/$lib timeout -k 10 120 python3 -u tools/probe_axis.py 2>> $OUT/axis.err | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> $OUT/axis.jsonl || exit 1
done; done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_pair.log 2>&1 || exit 1
