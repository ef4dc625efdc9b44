// Launch entry points of the gfx950 kernels (k_all.hip, k_axis.hip, k_map.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "rdx_kdesc.h"

namespace rdx {

hipError_t launch_all_contig(uint32_t dtype, uint32_t op, const KAllContig &a, uint32_t n_chunks, hipStream_t s);
hipError_t launch_all_strided(uint32_t dtype, uint32_t op, const KAllStrided &a, uint32_t n_chunks, hipStream_t s);
hipError_t launch_axis(uint32_t dtype, uint32_t op, const KAxis &a, int cus, hipStream_t s);
hipError_t launch_map(uint32_t dtype, const KMap &a, int cus, hipStream_t s);
hipError_t launch_unshuffle(const uint8_t *in, uint8_t *out, uint64_t len, uint64_t es, int cus, hipStream_t s);

}  // namespace rdx
