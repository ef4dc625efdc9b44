# tools/probe_aql: the kernels as a bare gfx950 code object (unbundled), the host program against HIP + HSA.
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --genco --offload-arch=gfx950 -O3 probe_aql_kernels.hip -o probe_aql_kernels.bundle
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=probe_aql_kernels.bundle \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=probe_aql_kernels.co
rm -f probe_aql_kernels.bundle
/opt/rocm/bin/hipcc -O2 -std=c++17 probe_aql.cpp -o probe_aql -I/opt/rocm/include -L/opt/rocm/lib -lhsa-runtime64 \
    -Wl,-rpath,/opt/rocm/lib
