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

constexpr int kMultiDims = 4;   // canonical dims of a k_multi view (deeper views run as their own launch)

// Per-workgroup copy of a request's missing_values list (compared per element from LDS).
struct MultiShared {
    uint64_t list[kInlineMissing];
};

// The missing predicate of one request (missing.rs:114-122 / operations.rs:25-33): the comparison
// forms branch-free on two scalars, a missing_values list (<= 16, reference order) from LDS, so the
// request's descriptor never has to live in scalar registers whole (a 16-entry list there spilled the
// kernel's SGPRs into its inner loop).
template <typename T>
struct MultiMiss {
    T a, hi;
    bool eq_on, lo_on, hi_on, filt;
    uint32_t n_list;
    const uint64_t *list;   // LDS
    __device__ __forceinline__ bool included(T x) const {
        bool missing = (eq_on & (x == a)) | (lo_on & (x < a)) | (hi_on & (x > hi));
        for (uint32_t i = 0; i < n_list; ++i) missing |= x == from_bits64<T>(list[i]);
        bool inc = !missing;
        if constexpr (std::is_floating_point_v<T>) inc = inc & !(filt & (lo_on | hi_on) & (x != x));
        return inc;
    }
};

template <typename T, int OP, bool FUSED, int VW>
__device__ __forceinline__ void multi_body(const KMultiItem *__restrict__ it, uint32_t b, MultiShared *sd) {
    constexpr int kU = 4;   // loads in flight per lane per step (8 for the lighter bodies measured slower)
    const KAllStrided &a = it->a;
    const uint32_t bpc = a.blocks_per_chunk;
    const uint8_t *base = a.src.base;
    const uint64_t plane = a.src.plane;
    const bool bswap = a.src.bswap;
    const KView &v = a.view;
    MultiMiss<T> mm;
    {
        const uint32_t k = a.miss.kind;
        mm.a = from_bits64<T>(a.miss.v0);
        mm.hi = k == RDX_MISSING_VALID_MAX ? mm.a : from_bits64<T>(a.miss.v1);
        mm.eq_on = k == RDX_MISSING_VALUE;
        mm.lo_on = k == RDX_MISSING_VALID_MIN || k == RDX_MISSING_VALID_RANGE;
        mm.hi_on = k == RDX_MISSING_VALID_MAX || k == RDX_MISSING_VALID_RANGE;
        mm.filt = a.filter_semantics != 0;
        mm.n_list = k == RDX_MISSING_VALUES ? a.miss.n : 0;   // <= kInlineMissing (longer lists run alone)
        if (threadIdx.x < mm.n_list) sd->list[threadIdx.x] = a.miss.inl[threadIdx.x];
        mm.list = sd->list;
        __syncthreads();
    }
    // The view's dims: uniform loads of the request table (scalar registers); the host pads every
    // view to kMultiDims dims with count 1 / stride 0 (rdx_execute_multi_device).
    uint32_t cnt[kMultiDims];
    uint64_t mag[kMultiDims];
    int64_t vs[kMultiDims], rs[kMultiDims];
#pragma unroll
    for (int k = 0; k < kMultiDims; ++k) {
        cnt[k] = v.count[k];
        mag[k] = v.div[k].magic;
        vs[k] = v.vstride[k];
        rs[k] = v.rstride[k];
    }
    const int64_t base_off = v.base_off, r0 = v.r0;
    const int nd = v.ndim;   // dims >= nd are padding (count 1): skipped by a uniform branch
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
            int64_t o = base_off, rr = r0;
#pragma unroll
            for (int k = 0; k < kMultiDims; ++k) {
                if (k > 0 && k >= nd) break;
                const uint32_t qn = k + 1 < nd ? udiv(q, mag[k]) : 0u;   // the last dim needs no division
                const uint32_t idx = q - qn * cnt[k];
                o += (int64_t)idx * vs[k];
                if constexpr (Red<T, OP>::kRank) rr += (int64_t)idx * rs[k];
                q = qn;
            }
            off[u] = o;
            rk[u] = rr;
        }
        Raw<T, FUSED, VW> raw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_load(raw[u], base, plane, (uint64_t)off[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_cvt(raw[u], bswap, x[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (!ok[u]) continue;
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                if (!mm.included(x[u][j])) continue;
                if constexpr (OP == OP_COUNT) r.cnt += 1;
                else r.add(x[u][j], [&]() { return rk[u] + (int64_t)j * rs[0]; });
            }
        }
    }
    finalize_all<T, OP>(r, a.out, 0, bpc, b);
}

template <typename T, int OP>
__device__ __forceinline__ void multi_paths(const KMultiItem *__restrict__ it, uint32_t b, MultiShared *sl) {
    constexpr int VWV = 16 / (int)sizeof(T);
    if (it->a.vec > 1) multi_body<T, OP, false, VWV>(it, b, sl);
    else multi_body<T, OP, false, 1>(it, b, sl);
}

template <typename T>
__device__ __forceinline__ void multi_ops(const KMultiItem *__restrict__ it, uint32_t b, MultiShared *sl) {
    switch (it->op) {
        case OP_COUNT: multi_paths<T, OP_COUNT>(it, b, sl); break;
        case OP_MAX: multi_paths<T, OP_MAX>(it, b, sl); break;
        case OP_MIN: multi_paths<T, OP_MIN>(it, b, sl); break;
        default: multi_paths<T, OP_SUM>(it, b, sl); break;
    }
}

#ifndef RDX_MULTI_WAVES
#define RDX_MULTI_WAVES 5   // >= 5 waves per SIMD: <= 102 VGPRs (the heaviest body needs 95)
#endif
__global__ __launch_bounds__(kBlock, RDX_MULTI_WAVES) void k_multi(const KMulti m) {
    __shared__ MultiShared s_req;
    const uint32_t item = m.blk2item[blockIdx.x];
    const KMultiItem *__restrict__ it = m.items + item;
    const uint32_t b = blockIdx.x - it->block0;
    switch (it->dtype) {
        case RDX_DTYPE_INT32: multi_ops<int32_t>(it, b, &s_req); break;
        case RDX_DTYPE_INT64: multi_ops<int64_t>(it, b, &s_req); break;
        case RDX_DTYPE_UINT32: multi_ops<uint32_t>(it, b, &s_req); break;
        case RDX_DTYPE_UINT64: multi_ops<uint64_t>(it, b, &s_req); break;
        case RDX_DTYPE_FLOAT32: multi_ops<float>(it, b, &s_req); break;
        default: multi_ops<double>(it, b, &s_req); break;
    }
}

}  // namespace

hipError_t launch_multi(const KMulti &m, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_multi, dim3(blocks), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

}  // namespace rdx
