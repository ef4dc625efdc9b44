# Round 5: A/B of k_pinflate.hip — round 4's source (librdx_pold.so, same runtime) against this round's.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r05p3}
mkdir -p $OUT
RDX_LIB_PATH=$PWD/reductionist-rs_amd/librdx_pold.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/old -o run --output-format csv -- python3 tools/probe_pinflate.py 5 > $OUT/old.jsonl 2> $OUT/old.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/new -o run --output-format csv -- python3 tools/probe_pinflate.py 5 > $OUT/new.jsonl 2> $OUT/new.err
