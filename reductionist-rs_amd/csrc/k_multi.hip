// Heterogeneous request batch: ONE launch over many independent all-axes requests that each carry
// their own dtype, operation, hyperslab view, byte order, missing predicate and outputs
// (the request-level concurrency of src/app.rs:147-152, where every request is its own
// operation<T>() call, folded into one grid).  The request descriptors travel in the kernel arguments
// (KMultiArgs, < 4 KiB); block -> request by a uniform binary search over their first blocks.  Each
// request's blocks run the strided all-axes loop of k_all.hip (runtime rank, generic missing predicate)
// on their slice of the request's flattened view and finish with the request's own deterministic
// cross-workgroup fold (finalize_all).  The dtype / op / access path switch is uniform per block, so
// every wave executes exactly one body.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

// The missing predicate of one request (missing.rs:114-122 / operations.rs:25-33) as branch-free
// comparisons on two scalars: MISSING_VALUE / MISSING_VALUES of <= 2 entries are equalities,
// VALID_MIN / VALID_MAX / VALID_RANGE bounds (longer lists run as their own launches).
template <typename T>
struct MultiMiss {
    T a, b;
    bool eq0, eq1, lo, hi, filt;
    __device__ __forceinline__ bool included(T x) const {
        const bool missing = (eq0 & (x == a)) | (eq1 & (x == b)) | (lo & (x < a)) | (hi & (x > b));
        bool inc = !missing;
        if constexpr (std::is_floating_point_v<T>) inc = inc & !(filt & (lo | hi) & (x != x));
        return inc;
    }
};

template <typename T, int OP, int VW>
__device__ __forceinline__ void multi_body(const KMultiArgs &m, const KMultiReq &q, uint32_t item, uint32_t b) {
    constexpr int kU = 4;   // loads in flight per lane per step (8 for the lighter bodies measured slower)
    const uint32_t bpc = q.bpc;
    const uint8_t *base = q.base;
    const bool bswap = q.flags & kMultiBswap;
    MultiMiss<T> mm;
    mm.a = from_bits64<T>(q.v0);
    mm.b = from_bits64<T>(q.v1);
    mm.eq0 = q.flags & kMultiEq0;
    mm.eq1 = q.flags & kMultiEq1;
    mm.lo = q.flags & kMultiLo;
    mm.hi = q.flags & kMultiHi;
    mm.filt = q.flags & kMultiFilt;
    // the view's dims: uniform loads of the kernel arguments (scalar registers)
    uint32_t cnt[kMultiDims - 1];
    uint64_t mag[kMultiDims - 1];
    int32_t vs[kMultiDims], rs[kMultiDims];   // 32-bit: one SGPR each
#pragma unroll
    for (int k = 0; k < kMultiDims; ++k) {
        if (k < kMultiDims - 1) {
            cnt[k] = q.count[k];
            mag[k] = q.magic[k];
        }
        vs[k] = q.vstride[k];
        rs[k] = q.rstride[k];
    }
    const int64_t base_off = q.base_off, r0 = q.r0;
    const int nd = q.ndim;   // 1..kMultiDims
    Red<T, OP> r;
    r.init();
    const uint32_t nv = q.n / VW;
    const uint32_t per = ((nv + bpc - 1) / bpc + kBlock - 1) / kBlock * kBlock;
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
            uint32_t qi = (uint32_t)(g * VW);
            int64_t o = base_off, rr = r0;
#pragma unroll
            for (int k = 0; k < kMultiDims; ++k) {
                if (k > 0 && k >= nd) break;
                constexpr int kLast = kMultiDims - 2;          // dims 0..kLast carry extents / magics
                const int kd = k < kLast ? k : kLast;          // (compile-time: k is unrolled)
                const bool inner = k + 1 < nd;                 // the outermost dim needs no division
                const uint32_t qn = inner ? udiv(qi, mag[kd]) : 0u;
                const uint32_t idx = inner ? qi - qn * cnt[kd] : qi;
                o += (int64_t)(int32_t)idx * vs[k];   // idx < n < 2^31: v_mad_i64_i32
                if constexpr (Red<T, OP>::kRank) rr += (int64_t)(int32_t)idx * rs[k];
                qi = qn;
            }
            off[u] = o;
            rk[u] = rr;
        }
        Raw<T, false, VW> raw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_load(raw[u], base, 0, (uint64_t)off[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_pin(raw[u]);   // (no load sunk into its ok[u] branch)
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_cvt(raw[u], bswap, x[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (!ok[u]) continue;
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                if (!mm.included(x[u][j])) continue;
                if constexpr (OP == OP_COUNT) r.cnt += 1;
                else r.add(x[u][j], [&]() { return rk[u] + (int64_t)(j * rs[0]); });
            }
        }
    }
    KOut out{};
    out.body = q.body;
    out.counts = q.counts;
    out.status = q.status;
    out.partials = m.partials + (uint64_t)q.block0 * kRecordU64;
    out.tickets = m.tickets + (uint64_t)item * kTicketWords;
    out.epoch = m.epoch;
    out.fold_last = (m.flags & kMultiFoldLast) ? ((m.flags & kMultiAtomicFold) ? 2u : 1u) : 0u;
    out.host_slots = (m.flags & kMultiHostSlots) != 0;
    finalize_all<T, OP>(r, out, 0, bpc, b);
}

template <typename T, int OP>
__device__ __forceinline__ void multi_paths(const KMultiArgs &m, const KMultiReq &q, uint32_t item, uint32_t b) {
    constexpr int VWV = 16 / (int)sizeof(T);
    if (q.vec > 1) multi_body<T, OP, VWV>(m, q, item, b);
    else multi_body<T, OP, 1>(m, q, item, b);
}

template <typename T>
__device__ __forceinline__ void multi_ops(const KMultiArgs &m, const KMultiReq &q, uint32_t item, uint32_t b) {
    switch (q.op) {
        case OP_COUNT: multi_paths<T, OP_COUNT>(m, q, item, b); break;
        case OP_MAX: multi_paths<T, OP_MAX>(m, q, item, b); break;
        case OP_MIN: multi_paths<T, OP_MIN>(m, q, item, b); break;
        default: multi_paths<T, OP_SUM>(m, q, item, b); break;
    }
}

#ifndef RDX_MULTI_WAVES
#define RDX_MULTI_WAVES 5   // >= 5 waves per SIMD: <= 102 VGPRs
#endif
__global__ __launch_bounds__(kBlock, RDX_MULTI_WAVES) void k_multi([[maybe_unused]] const KMultiArgs args) {
    // The arguments are read in place from the kernel-argument segment (the only parameter, offset 0):
    // indexing the by-value parameter with a runtime request index would copy all of it to scratch.
    const KMultiArgs &m = *(const KMultiArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    // block -> request: the last request whose first block is <= blockIdx.x (uniform binary search over
    // the block0 column of the arguments)
    uint32_t lo = 0, hi = m.n_items - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (m.req[mid].block0 <= blockIdx.x) lo = mid;
        else hi = mid - 1;
    }
    const KMultiReq &q = m.req[lo];
    const uint32_t b = blockIdx.x - q.block0;
    switch (q.dtype) {
        case RDX_DTYPE_INT32: multi_ops<int32_t>(m, q, lo, b); break;
        case RDX_DTYPE_INT64: multi_ops<int64_t>(m, q, lo, b); break;
        case RDX_DTYPE_UINT32: multi_ops<uint32_t>(m, q, lo, b); break;
        case RDX_DTYPE_UINT64: multi_ops<uint64_t>(m, q, lo, b); break;
        case RDX_DTYPE_FLOAT32: multi_ops<float>(m, q, lo, b); break;
        default: multi_ops<double>(m, q, lo, b); break;
    }
}

}  // namespace

hipError_t launch_multi(const KMultiArgs &m, uint32_t blocks, hipStream_t s) {
    if (m.n_items == 0 || m.n_items > (uint32_t)kMultiMaxItems) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_multi, dim3(blocks), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

}  // namespace rdx
