// Element-wise kernels and the generic unshuffle.
//
//  k_map       — Select (src/operations.rs:487-526: every selected element in C order, or F order
//                when the unsliced array is not standard layout, plus the non-missing count with
//                missing_filter semantics) and reductions over axis=() (operations.rs:58-67,
//                188-210: value + 0/1 count per element).
//  k_unshuffle — src/filters/shuffle.rs:20-85 for any element_size into a scratch buffer: a workgroup
//                stages a tile of TI elements x es byte-planes in LDS (coalesced plane reads),
//                then writes TI*es contiguous output bytes.  Used for filter chains and for
//                element_size != sizeof(dtype); the common es == sizeof(dtype) case is fused into
//                the reduction kernels instead.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

// VW > 1: contiguous, VW-aligned inner runs in BOTH the input view and the output (output order is
// the traversal order), so each lane moves VW elements with one 16-byte load and one 16-byte store.
// KIND (a.kind) and MK (missing-predicate form) are compile-time, so the element loop carries no
// runtime switches.
// Offsets: a lane's kU vectors lie kBlock vectors apart in output order; the first is decomposed
// into (inner index, outer offset) with one magic division per dim, the others are the same row
// moved along the inner dim (vstride[0]) while they stay inside it — only a vector that crosses a
// row end is decomposed in full.  Select's long rows (C5: 32768-element runs) thus cost one
// decomposition per kU vectors instead of kU full ones (the map was ALU-bound on them).
template <typename T, bool FUSED, int VW, int KIND, int MK>
__global__ __launch_bounds__(kBlock) void k_map(const KMap a) {
    constexpr int kU = 4;
    const KView &v = a.view;
    const bool bswap = a.src.bswap;
    int64_t cnt = 0;
    const uint64_t nv = v.n / VW;
    // each workgroup streams one contiguous stretch of the output (and of each input row)
    const uint64_t per = ((nv + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
    const uint64_t g_begin = (uint64_t)blockIdx.x * per;
    const uint64_t g_end = g_begin + per < nv ? g_begin + per : nv;
    const uint64_t stride = kBlock;
    const uint32_t count0 = v.count[0];
    const uint64_t magic0 = v.div[0].magic;
    const int64_t vs0 = v.vstride[0];
    auto outer = [&](uint32_t q) -> int64_t {   // offset of outer index q (dims 1..ndim-1)
        int64_t o = v.base_off;
        for (int k = 1; k < v.ndim; ++k) {
            const uint32_t qn = udiv(q, v.div[k].magic);
            o += (int64_t)(q - qn * v.count[k]) * v.vstride[k];
            q = qn;
        }
        return o;
    };
    // nothing here can fail, except the hand-off of Select's count: there the folding workgroup alone writes
    // the status (finalize_count), so a detected fault is never overwritten by this store
    constexpr bool kCountHandoff = KIND == 0 && MK != MK_NONE;
    if (!kCountHandoff && blockIdx.x == 0 && threadIdx.x == 0 && a.out.status) *a.out.status = 0;
    for (uint64_t g0 = g_begin + threadIdx.x; g0 < g_end; g0 += stride * kU) {
        int64_t off[kU];
        bool ok[kU];
        T x[kU][VW];
        {
            const uint32_t q = (uint32_t)(g0 * VW);
            const uint32_t q1 = udiv(q, magic0);
            const uint32_t i0 = q - q1 * count0;
            const int64_t ob = outer(q1);
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                uint64_t g = g0 + (uint64_t)u * stride;
                ok[u] = g < g_end;
                if (!ok[u]) g = g0;  // clamped into the range: the load issues unconditionally
                const uint64_t iu = (uint64_t)i0 + (g - g0) * VW;
                if (iu < count0) {
                    off[u] = ob + (int64_t)iu * vs0;
                } else {
                    const uint32_t qq = (uint32_t)(g * VW), qq1 = udiv(qq, magic0);
                    off[u] = outer(qq1) + (int64_t)(qq - qq1 * count0) * vs0;
                }
            }
        }
        Raw<T, FUSED, VW> raw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_load(raw[u], a.src.base, a.src.plane, (uint64_t)off[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_pin(raw[u]);   // (no load sunk into its ok[u] branch)
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_cvt(raw[u], bswap, x[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (!ok[u]) continue;
            const uint64_t g = (g0 + (uint64_t)u * stride) * VW;
            int64_t c[VW];
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                if constexpr (KIND == 0) c[j] = included_mk<T, MK>(a.miss, x[u][j], true) ? 1 : 0;
                else c[j] = included_mk<T, MK>(a.miss, x[u][j], false) ? 1 : 0;
            }
            if constexpr (KIND == 0 && MK != MK_NONE) {
#pragma unroll
                for (int j = 0; j < VW; ++j) cnt += c[j];
            }
            if constexpr (KIND != 2) {  // values
                if constexpr (VW == 1) {
                    gst<T>(reinterpret_cast<T *>(a.out.body) + g, x[u][0]);
                } else {
                    uint4 w;
                    __builtin_memcpy(&w, x[u], 16);
                    gst<uint4>(reinterpret_cast<T *>(a.out.body) + g, w);
                }
            }
            if constexpr (KIND != 0) {  // per-element counts (and the body itself for Count)
#pragma unroll
                for (int j = 0; j < VW; j += 2) {
                    if constexpr (VW == 1) {
                        gst<int64_t>(a.out.counts + g, c[0]);
                        if constexpr (KIND == 2) gst<int64_t>(reinterpret_cast<int64_t *>(a.out.body) + g, c[0]);
                    } else {
                        uint4 w;
                        __builtin_memcpy(&w, &c[j], 16);
                        gst<uint4>(a.out.counts + g + j, w);
                        if constexpr (KIND == 2) gst<uint4>(reinterpret_cast<int64_t *>(a.out.body) + g + j, w);
                    }
                }
            }
        }
    }
    if constexpr (KIND == 0) {
        if constexpr (MK != MK_NONE) finalize_count(cnt, a.out.counts, a.out.status, a.out.partials, a.out.tickets, a.out.epoch,
                                                 gridDim.x, blockIdx.x);
        else if (blockIdx.x == 0 && threadIdx.x == 0) a.out.counts[0] = (int64_t)v.n;  // sliced.len()
    }
}

// out[i*es + k] = in[k*N + i]
__global__ __launch_bounds__(kBlock) void k_unshuffle(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                      uint64_t n, uint32_t es, uint32_t ti) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    for (uint64_t i0 = (uint64_t)blockIdx.x * ti; i0 < n; i0 += (uint64_t)gridDim.x * ti) {
        const uint32_t cnt = (uint32_t)((n - i0) < ti ? (n - i0) : ti);
        for (uint32_t k = 0; k < es; ++k)
            for (uint32_t i = threadIdx.x; i < cnt; i += kBlock) tile[i * es + k] = gld<uint8_t>(in + (uint64_t)k * n + i0 + i);
        __syncthreads();
        const uint64_t obase = i0 * es;
        const uint32_t bytes = cnt * es;
        if ((((uintptr_t)out + obase) & 3) == 0) {
            const uint32_t words = bytes / 4;
            for (uint32_t w = threadIdx.x; w < words; w += kBlock)
                gst<uint32_t>(reinterpret_cast<uint32_t *>(out + obase) + w, reinterpret_cast<const uint32_t *>(tile)[w]);
            for (uint32_t q = words * 4 + threadIdx.x; q < bytes; q += kBlock) out[obase + q] = tile[q];
        } else {
            for (uint32_t q = threadIdx.x; q < bytes; q += kBlock) out[obase + q] = tile[q];
        }
        __syncthreads();
    }
}

// element sizes too large for an LDS tile: direct byte gather
__global__ __launch_bounds__(kBlock) void k_unshuffle_big(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                          uint64_t n, uint64_t es) {
    const uint64_t total = n * es;
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i = j / es, k = j - i * es;
        gst<uint8_t>(out + j, gld<uint8_t>(in + k * n + i));
    }
}

template <typename T, bool FUSED, int VW, int KIND>
void launch_map_mk(const KMap &a, dim3 grid, hipStream_t s) {
    const dim3 block(kBlock);
    switch (miss_kind_of(a.miss.kind)) {
        case MK_NONE: hipLaunchKernelGGL((k_map<T, FUSED, VW, KIND, MK_NONE>), grid, block, 0, s, a); break;
        case MK_CMP: hipLaunchKernelGGL((k_map<T, FUSED, VW, KIND, MK_CMP>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((k_map<T, FUSED, VW, KIND, MK_ANY>), grid, block, 0, s, a); break;
    }
}

template <typename T, bool FUSED, int VW>
void launch_map_kind(const KMap &a, dim3 grid, hipStream_t s) {
    if (a.kind == 0) launch_map_mk<T, FUSED, VW, 0>(a, grid, s);
    else if (a.kind == 1) launch_map_mk<T, FUSED, VW, 1>(a, grid, s);
    else launch_map_mk<T, FUSED, VW, 2>(a, grid, s);
}

template <typename T>
hipError_t launch_map_t(const KMap &a, int cus, hipStream_t s) {
    constexpr int VW = 16 / sizeof(T);
    const uint64_t vw = a.vec > 1 ? VW : 1;
    uint64_t blocks = (a.view.n / vw + kBlock * 4 - 1) / (kBlock * 4);
    const uint64_t cap = (uint64_t)cus * 8;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    const dim3 grid((uint32_t)blocks);
    if (a.src.fused) launch_map_kind<T, true, 1>(a, grid, s);
    else if (a.vec > 1) launch_map_kind<T, false, VW>(a, grid, s);
    else launch_map_kind<T, false, 1>(a, grid, s);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_map(uint32_t dtype, const KMap &a, int cus, hipStream_t s) {
    switch (dtype) {
        case RDX_DTYPE_INT32: return launch_map_t<int32_t>(a, cus, s);
        case RDX_DTYPE_INT64: return launch_map_t<int64_t>(a, cus, s);
        case RDX_DTYPE_UINT32: return launch_map_t<uint32_t>(a, cus, s);
        case RDX_DTYPE_UINT64: return launch_map_t<uint64_t>(a, cus, s);
        case RDX_DTYPE_FLOAT32: return launch_map_t<float>(a, cus, s);
        case RDX_DTYPE_FLOAT64: return launch_map_t<double>(a, cus, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_unshuffle(const uint8_t *in, uint8_t *out, uint64_t len, uint64_t es, int cus, hipStream_t s) {
    const uint64_t n = len / es;
    if (n == 0) return hipSuccess;
    if (es > 16384) {
        uint64_t blocks = (len + kBlock - 1) / kBlock;
        if (blocks > (uint64_t)cus * 16) blocks = (uint64_t)cus * 16;
        hipLaunchKernelGGL(k_unshuffle_big, dim3((uint32_t)blocks), dim3(kBlock), 0, s, in, out, n, es);
        return hipGetLastError();
    }
    uint32_t ti = (uint32_t)(16384 / es);
    if (ti > 4096) ti = 4096;
    if (ti == 0) ti = 1;
    uint64_t blocks = (n + ti - 1) / ti;
    if (blocks > (uint64_t)cus * 8) blocks = (uint64_t)cus * 8;
    const size_t lds = (size_t)ti * es;
    hipLaunchKernelGGL(k_unshuffle, dim3((uint32_t)blocks), dim3(kBlock), lds, s, in, out, n, (uint32_t)es, ti);
    return hipGetLastError();
}

}  // namespace rdx
