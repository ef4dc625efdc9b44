// Runtime dtype -> per-dtype kernel translation unit (k_all.hip / k_axis.hip built once per dtype).
#include "../../include/rdx.h"
#include "rdx_kernels.hpp"

namespace rdx {

#define RDX_DTYPE_SWITCH(fn, ...)                                        \
    switch (dtype) {                                                     \
        case RDX_DTYPE_INT32: return fn##_i32(__VA_ARGS__);              \
        case RDX_DTYPE_INT64: return fn##_i64(__VA_ARGS__);              \
        case RDX_DTYPE_UINT32: return fn##_u32(__VA_ARGS__);             \
        case RDX_DTYPE_UINT64: return fn##_u64(__VA_ARGS__);             \
        case RDX_DTYPE_FLOAT32: return fn##_f32(__VA_ARGS__);            \
        case RDX_DTYPE_FLOAT64: return fn##_f64(__VA_ARGS__);            \
    }                                                                    \
    return hipErrorInvalidValue;

hipError_t launch_all_contig(uint32_t dtype, uint32_t op, const KAllContig &a, uint32_t n_chunks, hipStream_t s) {
    RDX_DTYPE_SWITCH(launch_all_contig, op, a, n_chunks, s)
}

hipError_t launch_all_strided(uint32_t dtype, uint32_t op, const KAllStrided &a, uint32_t n_chunks, hipStream_t s) {
    RDX_DTYPE_SWITCH(launch_all_strided, op, a, n_chunks, s)
}

hipError_t launch_axis(uint32_t dtype, uint32_t op, const KAxis &a, int cus, hipStream_t s) {
    RDX_DTYPE_SWITCH(launch_axis, op, a, cus, s)
}

}  // namespace rdx
