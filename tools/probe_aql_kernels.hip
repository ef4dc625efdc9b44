// Kernels of tools/probe_aql.cpp, built as a bare gfx950 code object (hipcc --genco) so the probe can load
// them through the HSA loader and dispatch them by writing AQL packets itself.
#include <hip/hip_runtime.h>
#include <stdint.h>

// nothing: the launch floor
extern "C" __global__ void k_empty(uint64_t *slot, uint64_t tag) {}

// one lane writes `tag` to a host-visible word (system scope): what the engine's host slots do
extern "C" __global__ void k_slot(uint64_t *slot, uint64_t tag) {
    if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(slot, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
