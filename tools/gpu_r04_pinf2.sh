# GPU box (round 4): pinflate tests, then the lone-stream probe + per-workgroup profile for the product
# library and each variant library named in RDX_VARIANTS, then the find-kernel probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r04pinf2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pinflate.py > $OUT/pytest_pinf.txt 2>&1
rc=$?
tail -3 $OUT/pytest_pinf.txt
[ $rc -eq 0 ] || { tail -40 $OUT/pytest_pinf.txt; exit $rc; }
for lib in librdx ${RDX_VARIANTS:-}; do
  [ -f reductionist-rs_amd/$lib.so ] || continue
  echo "== $lib"
  RDX_LIB_PATH=$PWD/reductionist-rs_amd/$lib.so timeout -k 10 300 python -u tools/probe_pinflate.py 10 > $OUT/probe_$lib.jsonl 2>$OUT/probe_$lib.err || { tail -20 $OUT/probe_$lib.err; exit 1; }
  cat $OUT/probe_$lib.jsonl
  RDX_LIB_PATH=$PWD/reductionist-rs_amd/$lib.so RDX_PINF_PROF=1 timeout -k 10 300 python -u tools/probe_pinflate.py 1 > /dev/null 2>$OUT/wgprof_$lib.txt || { tail -20 $OUT/wgprof_$lib.txt; exit 1; }
  grep pinf_prof $OUT/wgprof_$lib.txt | head -12
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/probe_pinflate.py 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/pinf_trace.py $OUT/prof/run_kernel_trace.csv 4
