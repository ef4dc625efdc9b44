// Heterogeneous request batch: ONE launch over many independent all-axes requests that each carry
// their own dtype, operation, hyperslab view, byte order, fused shuffle, missing predicate and outputs
// (the request-level concurrency of src/app.rs:147-152, where every request is its own
// operation<T>() call, folded into one grid).  Block -> request through a block map uploaded with the
// request table; each request's blocks run the strided all-axes loop of k_all.hip (runtime rank,
// generic missing predicate) on their slice of the request's flattened view and finish with the
// request's own deterministic cross-workgroup fold (finalize_all).  The dtype / op / access path switch
// is uniform per block, so every wave executes exactly one body.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

constexpr int kMultiDims = 4;   // canonical dims kept in registers; deeper views read the table per vector

template <typename T, int OP, bool FUSED, int VW>
__device__ __forceinline__ void multi_body(const KMultiItem *__restrict__ it, uint32_t b) {
    constexpr int kU = VW > 1 ? 4 : 8;
    const KAllStrided &a = it->a;
    const uint32_t bpc = a.blocks_per_chunk;
    const uint8_t *base = a.src.base;
    const bool bswap = a.src.bswap;
    const KView &v = a.view;
    const int nd = v.ndim;
    uint32_t cnt[kMultiDims];
    uint64_t mag[kMultiDims];
    int64_t vs[kMultiDims], rs[kMultiDims];
#pragma unroll
    for (int k = 0; k < kMultiDims; ++k) {
        cnt[k] = k < nd ? v.count[k] : 1;
        mag[k] = k < nd ? v.div[k].magic : 0;
        vs[k] = k < nd ? v.vstride[k] : 0;
        rs[k] = k < nd ? v.rstride[k] : 0;
    }
    const bool deep = nd > kMultiDims;
    Red<T, OP> r;
    r.init();
    const uint64_t nv = v.n / VW;
    const uint64_t per = ((nv + bpc - 1) / bpc + kBlock - 1) / kBlock * kBlock;
    const uint64_t g_begin = (uint64_t)b * per;
    const uint64_t g_end = g_begin + per < nv ? g_begin + per : nv;
    for (uint64_t g0 = g_begin + threadIdx.x; g0 < g_end; g0 += (uint64_t)kBlock * kU) {
        int64_t off[kU], rk[kU];
        bool ok[kU];
        T x[kU][VW];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            uint64_t g = g0 + (uint64_t)u * kBlock;
            ok[u] = g < g_end;
            if (!ok[u]) g = g0;  // clamped into the range: the load issues unconditionally
            uint32_t q = (uint32_t)(g * VW);
            int64_t o = v.base_off, rr = v.r0;
            if (!deep) {
#pragma unroll
                for (int k = 0; k < kMultiDims; ++k) {
                    const uint32_t qn = udiv(q, mag[k]);
                    const uint32_t idx = q - qn * cnt[k];
                    o += (int64_t)idx * vs[k];
                    rr += (int64_t)idx * rs[k];
                    q = qn;
                }
            } else {
                for (int k = 0; k < nd; ++k) {
                    const uint32_t qn = udiv(q, v.div[k].magic);
                    const uint32_t idx = q - qn * v.count[k];
                    o += (int64_t)idx * v.vstride[k];
                    rr += (int64_t)idx * v.rstride[k];
                    q = qn;
                }
            }
            off[u] = o;
            rk[u] = rr;
        }
        Raw<T, FUSED, VW> raw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_load(raw[u], base, a.src.plane, (uint64_t)off[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_cvt(raw[u], bswap, x[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (!ok[u]) continue;
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                if (!included_mk<T, MK_ANY>(a.miss, x[u][j], a.filter_semantics)) continue;
                if constexpr (OP == OP_COUNT) r.cnt += 1;
                else r.add(x[u][j], [&]() { return rk[u] + (int64_t)j * rs[0]; });
            }
        }
    }
    finalize_all<T, OP>(r, a.out, 0, bpc, b);
}

template <typename T, int OP>
__device__ __forceinline__ void multi_paths(const KMultiItem *__restrict__ it, uint32_t b) {
    constexpr int VWV = 16 / (int)sizeof(T);
    if (it->a.src.fused) multi_body<T, OP, true, 1>(it, b);
    else if (it->a.vec > 1) multi_body<T, OP, false, VWV>(it, b);
    else multi_body<T, OP, false, 1>(it, b);
}

template <typename T>
__device__ __forceinline__ void multi_ops(const KMultiItem *__restrict__ it, uint32_t b) {
    switch (it->op) {
        case OP_COUNT: multi_paths<T, OP_COUNT>(it, b); break;
        case OP_MAX: multi_paths<T, OP_MAX>(it, b); break;
        case OP_MIN: multi_paths<T, OP_MIN>(it, b); break;
        default: multi_paths<T, OP_SUM>(it, b); break;
    }
}

__global__ __launch_bounds__(kBlock) void k_multi(const KMulti m) {
    const uint32_t item = m.blk2item[blockIdx.x];
    const KMultiItem *__restrict__ it = m.items + item;
    const uint32_t b = blockIdx.x - it->block0;
    switch (it->dtype) {
        case RDX_DTYPE_INT32: multi_ops<int32_t>(it, b); break;
        case RDX_DTYPE_INT64: multi_ops<int64_t>(it, b); break;
        case RDX_DTYPE_UINT32: multi_ops<uint32_t>(it, b); break;
        case RDX_DTYPE_UINT64: multi_ops<uint64_t>(it, b); break;
        case RDX_DTYPE_FLOAT32: multi_ops<float>(it, b); break;
        default: multi_ops<double>(it, b); break;
    }
}

}  // namespace

hipError_t launch_multi(const KMulti &m, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_multi, dim3(blocks), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

}  // namespace rdx
