# A/B variants of k_pinflate: k_pinflate.o and rdx_runtime.o (the only objects that include rdx_pinflate.h)
# rebuilt with extra defines, linked with the product's other objects into librdx_pv_<name>.so.
# Usage (on the CPU host, after `make -C reductionist-rs_amd`): tools/build_pinf_variant.sh <name> "<defines>"
set -euo pipefail
cd "$(dirname "$0")/../reductionist-rs_amd"
name=$1
defs=${2:-}
B=build_pv_$name
mkdir -p $B
FLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 $defs"
rm -f $B/k_pinflate.o $B/rdx_runtime.o librdx_pv_$name.so
/opt/rocm/bin/hipcc $FLAGS -c csrc/k_pinflate.hip -o $B/k_pinflate.o & p1=$!
/opt/rocm/bin/hipcc $FLAGS -c csrc/rdx_runtime.cpp -o $B/rdx_runtime.o & p2=$!
wait $p1
wait $p2
objs=$(ls build/*.o | grep -v -e '/k_pinflate.o$' -e '/rdx_runtime.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o librdx_pv_$name.so $objs $B/k_pinflate.o $B/rdx_runtime.o
echo "built reductionist-rs_amd/librdx_pv_$name.so ($defs)"
