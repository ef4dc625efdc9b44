# GPU box: blosc2 decode probe incl. zstd (kernel trace) — k_blosc2_zstd vs the LZ codecs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${RDX_TAG:-r03zstd}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/probe_blosc2.py 256 zstd,lz4_lib,lz4 > $OUT/probe.jsonl 2> $OUT/trace.log
