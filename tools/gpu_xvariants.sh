set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/x1
for v in base xNOMISS xNOFIN xBOTH; do
  if [ $v = base ]; then L=$PWD/reductionist-rs_amd/librdx.so; else L=$PWD/reductionist-rs_amd/librdx_$v.so; fi
  RDX_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/x1/$v -o run --output-format csv -- python3 tools/probe_small.py > gpurun_out/x1/$v.log 2>&1 || exit 1
done
