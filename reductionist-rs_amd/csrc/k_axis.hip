// Reductions over a subset of axes: count_array_multi_axis / max_ / min_ / sum_array_multi_axis
// (src/operations.rs:51-100, 213-268, 361-416, 532-583).  Output o (C order over the kept dims)
// folds every element of its reduced sub-array.  The values are order independent except the f32/f64
// sum (tolerance) and the ±0 tie of float min/max, which is resolved by the rank of the
// zero in the reference's fold order: F order over the reduced axes in request order (fold_axis
// over the first axis, then over the partials along the next, operations.rs:229-258).
//
//  k_axis_rows<VW> — the innermost memory dim is reduced: a group of `group` lanes per (output,
//                    slice) (the whole wave for long rows, 64/group outputs per wave for short ones);
//                    each lane loads VW consecutive elements (16 B when VW > 1), 4 loads in flight,
//                    butterfly within the group.
//  k_axis_cols<VW> — otherwise: a workgroup owns a tile of W lanes x VW consecutive outputs along
//                    the innermost kept dim (W = 64, or fewer when there are few outputs, and then
//                    64/W rows per wave access); its lanes split the slice's reduced rows (8-16 loads
//                    in flight per lane) and combine by shuffles and LDS.
//  When the reduced range is split into slices (few outputs), every slice publishes a partial and
//  the last slice to arrive for an output (rows) or tile (cols) folds them: one launch, no
//  second kernel.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

template <typename T, int OP>
__device__ __forceinline__ void write_result(const KOut &out, uint64_t o, const Red<T, OP> &r) {
    if constexpr (OP == OP_COUNT) reinterpret_cast<int64_t *>(out.body)[o] = r.cnt;
    else reinterpret_cast<T *>(out.body)[o] = r.value();
    out.counts[o] = r.cnt;
    if constexpr (Red<T, OP>::kRank) {
        if (r.nan && out.status)
            __hip_atomic_fetch_or(out.status, (uint32_t)RDX_E_NAN_UNORDERED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ int64_t kept_offset(const KView &kv, uint32_t t, int64_t &out_index) {
    int64_t off = kv.base_off, oi = 0;
    uint32_t q = t;
    for (int k = 0; k < kv.ndim; ++k) {
        const uint32_t qn = udiv(q, kv.div[k].magic);
        const uint32_t idx = q - qn * kv.count[k];
        off += (int64_t)idx * kv.vstride[k];
        oi += (int64_t)idx * kv.rstride[k];
        q = qn;
    }
    out_index = oi;
    return off;
}

template <bool RANK>
__device__ __forceinline__ int64_t red_offset(const KView &rv, uint32_t r, int64_t &rank) {
    int64_t off = 0, rk = rv.r0;
    uint32_t q = r;
    for (int k = 0; k < rv.ndim; ++k) {
        const uint32_t qn = udiv(q, rv.div[k].magic);
        const uint32_t idx = q - qn * rv.count[k];
        off += (int64_t)idx * rv.vstride[k];
        if (RANK) rk += (int64_t)idx * rv.rstride[k];
        q = qn;
    }
    rank = rk;
    return off;
}

// The reduced view's first two dims in registers, read from the kernel arguments once per lane
// (not per load: a cold launch otherwise waits on one scalar-cache miss per dim per load, as the
// strided all-axes kernel measured); deeper views fall back to the generic loop.
struct RedRegs {
    int32_t nd;
    uint32_t c0;
    uint64_t m0;
    int64_t v0, v1, s0, s1, r0;
    __device__ __forceinline__ void load(const KView &rv) {
        nd = rv.ndim;
        c0 = rv.count[0];
        m0 = rv.div[0].magic;
        v0 = rv.vstride[0];
        s0 = rv.rstride[0];
        v1 = rv.ndim > 1 ? rv.vstride[1] : 0;
        s1 = rv.ndim > 1 ? rv.rstride[1] : 0;
        r0 = rv.r0;
    }
};

// GEN: the reduced view has more than 2 dims (generic per-dim loop); chosen at launch, so the
// per-load offset code carries no rank branch.
template <bool RANK, bool GEN>
__device__ __forceinline__ int64_t red_offset(const RedRegs &g, const KView &rv, uint32_t r, int64_t &rank) {
    if constexpr (!GEN) {  // idx1 = r / count0 (< count1 for r in range), idx0 = r % count0
        const uint32_t q = g.nd == 2 ? udiv(r, g.m0) : 0u;
        const uint32_t idx0 = r - q * g.c0;
        if (RANK) rank = g.r0 + (int64_t)idx0 * g.s0 + (int64_t)q * g.s1;
        return (int64_t)idx0 * g.v0 + (int64_t)q * g.v1;
    } else {
        return red_offset<RANK>(rv, r, rank);
    }
}

template <typename T, int OP, int MK>
__device__ __forceinline__ void fold_in(Red<T, OP> &r, const KMissing &miss, T x, int64_t rank) {
    if (!included_mk<T, MK>(miss, x, false)) return;
    if constexpr (OP == OP_COUNT) r.cnt += 1;
    else r.add(x, [&]() { return rank; });
}

// Without a missing predicate every element is counted: the loops add the value only and count the
// elements once per load (one 64-bit add per load instead of one per element and output).
template <typename T, int OP, int MK>
__device__ __forceinline__ void fold_value(Red<T, OP> &r, const KMissing &miss, T x, int64_t rank) {
    if constexpr (MK == MK_NONE) {
        if constexpr (OP != OP_COUNT) r.add_value(x, [&]() { return rank; });
    } else {
        fold_in<T, OP, MK>(r, miss, x, rank);
    }
}

template <typename T, int OP, bool FUSED, int VW, bool GEN, int MK, int KU>
__global__ __launch_bounds__(kBlock) void k_axis_rows(const KAxis a) {
    constexpr bool RANK = Red<T, OP>::kRank;
    constexpr int kU = KU;   // loads in flight per lane (4; 16 for long rows, launch_axis_k)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t L = a.group, G = 64 / L;        // lanes per item, items per wave pass
    const uint32_t l = lane & (L - 1), g = lane / L;
    const uint64_t nw = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t items = a.n_out * a.slices;
    RedRegs rg;
    rg.load(a.red);
    const uint64_t nrv = a.n_red / VW;  // reduced vectors per output
    // only float min/max can report an error (NaN); the host clears the status word for those
    if (!RANK && blockIdx.x == 0 && threadIdx.x == 0 && a.out.status) *a.out.status = 0;
    for (uint64_t w0 = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w0 * G < items; w0 += nw) {
        const uint64_t it = w0 * G + g;
        const bool valid = it < items;
        const uint64_t o = valid ? it / a.slices : 0, s = valid ? it - o * a.slices : 0;
        int64_t oi = 0, koff = 0;
        if (valid) koff = kept_offset(a.kept, (uint32_t)o, oi);
        const uint64_t r_lo = s * nrv / a.slices, r_hi = valid ? (s + 1) * nrv / a.slices : 0;
        Red<T, OP> r;
        r.init();
        for (uint64_t r0 = r_lo + l; r0 < r_hi; r0 += (uint64_t)L * kU) {
            int64_t off[kU], rk[kU];
            if (!GEN && rg.nd <= 1) {
                // one reduced dim: a lane's loads are L vectors apart, so the offsets (and ranks) are a base plus
                // multiples of one step: adds, not the general decomposition's 64-bit multiplies per load
                int64_t rk0;
                const int64_t o0 = koff + red_offset<RANK, GEN>(rg, a.red, (uint32_t)(r0 * VW), rk0);
                const int64_t od = (int64_t)L * VW * rg.v0, kd = (int64_t)L * VW * rg.s0;
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const bool in = r0 + (uint64_t)u * L < r_hi;   // clamped: every load issues, the value is dropped below
                    off[u] = in ? o0 + u * od : o0;
                    rk[u] = in ? rk0 + u * kd : rk0;
                }
            } else {
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    uint64_t rv = r0 + (uint64_t)u * L;
                    if (rv >= r_hi) rv = r0;  // clamped: every load issues, the value is dropped below
                    off[u] = koff + red_offset<RANK, GEN>(rg, a.red, (uint32_t)(rv * VW), rk[u]);
                }
            }
            Raw<T, FUSED, VW> raw[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) raw_load(raw[u], a.src.base, a.src.plane, (uint64_t)off[u]);
#pragma unroll
            for (int u = 0; u < kU; ++u) raw_pin(raw[u]);
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                if (r0 + (uint64_t)u * L >= r_hi) continue;
                T x[VW];
                raw_cvt(raw[u], a.src.bswap, x);
#pragma unroll
                for (int j = 0; j < VW; ++j) fold_value<T, OP, MK>(r, a.miss, x[j], rk[u] + (int64_t)j * rg.s0);
                if constexpr (MK == MK_NONE) r.cnt += VW;
            }
        }
        group_reduce(r, L);
        if (a.slices == 1) {
            if (valid && l == 0) write_result(a.out, (uint64_t)oi, r);
            continue;
        }
        // sliced (group == 64, one item per wave): publish, and the last slice to arrive folds them
        constexpr int kR = granules<T, OP>();
        uint32_t last = 0;
        if (lane == 0) {
            publish<T, OP>(a.out.partials + it * kR, r, a.out.epoch);
            uint32_t *tk = a.out.tickets + o * kTicketStride;   // one L2 line per counter: same-line atomics serialise
            last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.slices - 1;
            if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!__shfl(last, 0, 64)) continue;
        Red<T, OP> acc;
        acc.init();
        uint32_t fault = 0;
        for (uint32_t q = lane; q < a.slices; q += 64) {
            Red<T, OP> p;
            collect<T, OP>(a.out.partials + (o * a.slices + q) * kR, p, a.out.epoch, fault);
            acc.merge(p);
        }
        if (__builtin_amdgcn_ballot_w64(fault) && lane == 0 && a.out.status)
            __hip_atomic_fetch_or(a.out.status, (uint32_t)RDX_E_DEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_reduce(acc);
        if (lane == 0) write_result(a.out, (uint64_t)oi, acc);
    }
}

// Merge the states of lanes that hold the same columns (lane bits >= W, i.e. other rows) and then
// the 4 waves through LDS, in wave order; the workgroup total for column c ends in wave 0, lane c.
template <typename T, int OP, int VW>
__device__ __forceinline__ void cols_combine(Red<T, OP> (&r)[VW], uint64_t *lds, uint32_t W) {
    constexpr int kWaves = kBlock / 64;
    constexpr int kW = packed_words<T, OP>();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t m = W; m < 64; m <<= 1) {
#pragma unroll
        for (int j = 0; j < VW; ++j) xor_merge(r[j], (int)m);
    }
    if (wave > 0 && lane < W) {
#pragma unroll
        for (int j = 0; j < VW; ++j) store_packed<T, OP>(lds + (((wave - 1) * 64 + lane) * VW + j) * kW, r[j]);
    }
    __syncthreads();
    if (wave == 0 && lane < W) {
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            for (int w = 0; w < kWaves - 1; ++w) {
                Red<T, OP> o;
                load_packed<T, OP>(lds + ((w * 64 + lane) * VW + j) * kW, o);
                r[j].merge(o);
            }
        }
    }
}

template <typename T, int OP, bool FUSED, int VW, bool GEN, int MK>
__global__ __launch_bounds__(kBlock) void k_axis_cols(const KAxis a) {
    constexpr bool RANK = Red<T, OP>::kRank;
#ifndef RDX_AXIS_COLS_U16
#define RDX_AXIS_COLS_U16 16
#endif
#ifndef RDX_AXIS_COLS_U8
#define RDX_AXIS_COLS_U8 16
#endif
    constexpr int kU = VW * sizeof(T) >= 16 ? RDX_AXIS_COLS_U16 : RDX_AXIS_COLS_U8;   // loads in flight per lane
    constexpr int kWaves = kBlock / 64;
    constexpr int kW = packed_words<T, OP>();
    __shared__ uint64_t lds[(kWaves - 1) * 64 * VW * kW];
    __shared__ uint32_t s_last, s_fault;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t W = a.group, R = 64 / W;              // lanes per row of the tile, rows per wave access
    const uint32_t c = lane & (W - 1), rsub = lane / W;
    const uint64_t nkv = a.n_out / VW;                   // kept vectors
    const uint64_t kv = (uint64_t)blockIdx.x * W + c;
    const uint64_t s = blockIdx.y;
    if (!RANK && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && a.out.status) *a.out.status = 0;
    const bool active = kv < nkv;
    RedRegs rg;
    rg.load(a.red);
    int64_t oi = 0, koff = 0;
    if (active) koff = kept_offset(a.kept, (uint32_t)(kv * VW), oi);
    const uint64_t r_lo = s * a.n_red / a.slices, r_hi = (s + 1) * a.n_red / a.slices;
    Red<T, OP> r[VW];
#pragma unroll
    for (int j = 0; j < VW; ++j) r[j].init();
    int64_t rows = 0;   // (MK_NONE: the elements each output of this lane folded)
    if (active) {
        const uint64_t step = (uint64_t)kWaves * R;      // rows between a lane's consecutive loads
        for (uint64_t r0 = r_lo + wave * R + rsub; r0 < r_hi; r0 += step * kU) {
            int64_t off[kU], rk[kU];
            if (!GEN && rg.nd <= 1) {
                // one reduced dim ([R, C] axis 0): a lane's rows are `step` apart, so the offsets (and ranks) are a
                // base plus multiples of one step (the general decomposition's 64-bit multiplies per load held
                // the loads back: ~200 dependent instructions before the first one issued)
                int64_t rk0;
                const int64_t o0 = koff + red_offset<RANK, GEN>(rg, a.red, (uint32_t)r0, rk0);
                const int64_t od = (int64_t)step * rg.v0, kd = (int64_t)step * rg.s0;
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const bool in = r0 + (uint64_t)u * step < r_hi;   // clamped: every load issues, the value is dropped below
                    off[u] = in ? o0 + u * od : o0;
                    rk[u] = in ? rk0 + u * kd : rk0;
                }
            } else {
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    uint64_t rr = r0 + (uint64_t)u * step;
                    if (rr >= r_hi) rr = r0;  // clamped: every load issues, the value is dropped below
                    off[u] = koff + red_offset<RANK, GEN>(rg, a.red, (uint32_t)rr, rk[u]);
                }
            }
            Raw<T, FUSED, VW> raw[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) raw_load(raw[u], a.src.base, a.src.plane, (uint64_t)off[u]);
#pragma unroll
            for (int u = 0; u < kU; ++u) raw_pin(raw[u]);
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                if (r0 + (uint64_t)u * step >= r_hi) continue;
                T x[VW];
                raw_cvt(raw[u], a.src.bswap, x);
#pragma unroll
                for (int j = 0; j < VW; ++j) fold_value<T, OP, MK>(r[j], a.miss, x[j], rk[u]);
                if constexpr (MK == MK_NONE) ++rows;
            }
        }
    }
    if constexpr (MK == MK_NONE) {
#pragma unroll
        for (int j = 0; j < VW; ++j) r[j].cnt = rows;
    }
    cols_combine<T, OP, VW>(r, lds, W);
#if RDX_PROBES
    if (a.probe == 2) return;
#endif
    if (a.slices == 1) {
        if (wave == 0 && lane < W && active) {
#pragma unroll
            for (int j = 0; j < VW; ++j) write_result(a.out, (uint64_t)(oi + (int64_t)j * a.kept.rstride[0]), r[j]);
        }
        return;
    }
    // Sliced: publish this slice's records and count arrivals per tile; the workgroup of the last
    // slice to arrive folds all slices: its 256/W lane groups take contiguous slice ranges, then the
    // same lane + LDS combine.  In-kernel fold: records word-major per tile ([word][slice][c][j]), so
    // each word of a wave's records is one coalesced store / load ([4096,4096] f32 axis 0: 20.5 ->
    // 19.3 us).  Fold launch: record-major ([slice][c][j][word]) — k_axis_cols_fold reads a lane's
    // slice records one after another, one line per record.
    const uint64_t tile_rec = (uint64_t)W * VW;
    const uint64_t wstride = (uint64_t)a.slices * tile_rec;     // granules of one kind per tile
    if (a.fold_sep) {   // k_axis_cols_fold reads the records after this launch: plain stores
        uint64_t *P = a.out.partials + (uint64_t)blockIdx.x * wstride * kW;
        if (wave == 0 && lane < W) {
#pragma unroll
            for (int j = 0; j < VW; ++j) store_packed<T, OP>(P + ((uint64_t)s * tile_rec + c * VW + j) * kW, r[j]);
        }
        return;
    }
    uint64_t *P = a.out.partials + (uint64_t)blockIdx.x * wstride * granules<T, OP>();
    if (wave == 0 && lane < W) {
#pragma unroll
        for (int j = 0; j < VW; ++j) publish<T, OP>(P + (uint64_t)s * tile_rec + c * VW + j, r[j], a.out.epoch, wstride);
    }
    __syncthreads();   // every record of this slice issued before thread 0 counts the arrival
    if (threadIdx.x == 0) {
        uint32_t *tk = a.out.tickets + blockIdx.x * kTicketStride;
        const bool last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.slices - 1;
        if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last;
        s_fault = 0;
    }
    __syncthreads();
    if (!s_last) return;
#if RDX_PROBES
    if (a.probe == 1) return;
#endif
    const uint32_t G = kBlock / W, grp = threadIdx.x / W;    // parallel slice streams
    const uint32_t q_lo = (uint32_t)((uint64_t)grp * a.slices / G), q_hi = (uint32_t)((uint64_t)(grp + 1) * a.slices / G);
#pragma unroll
    for (int j = 0; j < VW; ++j) r[j].init();
    uint32_t fault = 0;
    if (active) {
        constexpr int kQ = 4;  // slices' records in flight per lane
        for (uint32_t q0 = q_lo; q0 < q_hi; q0 += kQ) {
            Red<T, OP> p[kQ][VW];
#pragma unroll
            for (int u = 0; u < kQ; ++u) {
#pragma unroll
                for (int j = 0; j < VW; ++j) {
                    if (q0 + u < q_hi) collect<T, OP>(P + (uint64_t)(q0 + u) * tile_rec + c * VW + j, p[u][j], a.out.epoch, fault, wstride);
                    else p[u][j].init();
                }
            }
#pragma unroll
            for (int u = 0; u < kQ; ++u) {
#pragma unroll
                for (int j = 0; j < VW; ++j) r[j].merge(p[u][j]);
            }
        }
    }
    if (fault) s_fault = 1;
    cols_combine<T, OP, VW>(r, lds, W);
    if (wave == 0 && lane < W && active) {
#pragma unroll
        for (int j = 0; j < VW; ++j) write_result(a.out, (uint64_t)(oi + (int64_t)j * a.kept.rstride[0]), r[j]);
    }
    if (threadIdx.x == 0 && s_fault && a.out.status)
        __hip_atomic_fetch_or(a.out.status, (uint32_t)RDX_E_DEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The fold of sliced column reductions as its own launch (fold_sep), parallel across outputs instead of
// one workgroup per tile: a wave per output (WG = false; its lanes take contiguous slice ranges, the
// wave butterfly merges them) or, for few outputs with many slices, a workgroup per output (WG = true,
// 256 slice ranges, block combine), so a tall narrow reduction folds in one or two round trips.
template <typename T, int OP, int VW, bool WG>
__global__ __launch_bounds__(kBlock) void k_axis_cols_fold(const KAxis a) {
    constexpr int kW = packed_words<T, OP>();
    constexpr uint32_t kLanes = WG ? kBlock : 64;
    const uint32_t lane = WG ? threadIdx.x : threadIdx.x & 63;
    const uint32_t W = a.group;
    const uint64_t tile_rec = (uint64_t)W * VW;
    const uint64_t nkv = a.n_out / VW;
    const uint64_t q = WG ? (uint64_t)blockIdx.x : (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t x = q / tile_rec, cj = q - x * tile_rec;                        // tile, c * VW + j
    const uint64_t kv = x * W + cj / VW;
    const uint32_t j = (uint32_t)(cj % VW);
    if (kv >= nkv) return;   // uniform over the wave (WG: over the workgroup)
    const uint64_t *P = a.out.partials + x * a.slices * tile_rec * kW + cj * kW;   // record-major (k_axis_cols)
    const uint32_t s_lo = (uint32_t)((uint64_t)lane * a.slices / kLanes);
    const uint32_t s_hi = (uint32_t)((uint64_t)(lane + 1) * a.slices / kLanes);
    Red<T, OP> r;
    r.init();
    for (uint32_t s0 = s_lo; s0 < s_hi; s0 += 4) {
        Red<T, OP> p[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            if (s0 + u < s_hi) load_packed<T, OP>(P + (uint64_t)(s0 + u) * tile_rec * kW, p[u]);
            else p[u].init();
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) r.merge(p[u]);
    }
    if constexpr (WG) block_reduce(r);
    else wave_reduce(r);
    if (lane == 0) {
        int64_t oi;
        kept_offset(a.kept, (uint32_t)(kv * VW), oi);
        write_result(a.out, (uint64_t)(oi + (int64_t)j * a.kept.rstride[0]), r);
    }
}

template <typename T, int OP, int VW, bool GEN, int MK>
void launch_axis_k(const KAxis &a, int cus, hipStream_t st) {
    const dim3 block(kBlock);
    if (a.mode == 0) {
        const uint64_t waves = (a.n_out * a.slices + 64 / a.group - 1) / (64 / a.group);
        uint64_t blocks = (waves + kBlock / 64 - 1) / (kBlock / 64);
        const uint64_t cap = (uint64_t)cus * 16;
        if (blocks > cap) blocks = cap;
        if (blocks == 0) blocks = 1;
        // rows whose slice gives every lane of its group 16 or more vectors (e.g. [4096, 4096] f32 axis 1: 1024
        // vectors per 64-lane row) keep 16 loads in flight per lane; shorter ones 4 (a load past the row's
        // end still issues, clamped, and would only cost)
#ifndef RDX_AXIS_ROWS_DEEP
#define RDX_AXIS_ROWS_DEEP 1
#endif
        const bool deep = RDX_AXIS_ROWS_DEEP && !a.src.fused && a.n_red / VW / a.slices >= 16ull * a.group;
        if (a.src.fused) hipLaunchKernelGGL((k_axis_rows<T, OP, true, 1, GEN, MK, 4>), dim3((uint32_t)blocks), block, 0, st, a);
        else if (deep) hipLaunchKernelGGL((k_axis_rows<T, OP, false, VW, GEN, MK, 16>), dim3((uint32_t)blocks), block, 0, st, a);
        else hipLaunchKernelGGL((k_axis_rows<T, OP, false, VW, GEN, MK, 4>), dim3((uint32_t)blocks), block, 0, st, a);
    } else {
        const dim3 grid((uint32_t)((a.n_out / VW + a.group - 1) / a.group), a.slices);
        if (a.src.fused) hipLaunchKernelGGL((k_axis_cols<T, OP, true, 1, GEN, MK>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((k_axis_cols<T, OP, false, VW, GEN, MK>), grid, block, 0, st, a);
        if (a.slices > 1 && a.fold_sep && a.probe == 0) {   // (probe is 0 unless built with RDX_PROBES)
            const uint64_t cols = (uint64_t)grid.x * a.group * (a.src.fused ? 1 : VW);   // record columns
            const bool wg = cols * 4 <= (uint64_t)cus * 4 && a.slices >= 256;   // few outputs, long folds
            const dim3 fgrid((uint32_t)(wg ? cols : (cols + kBlock / 64 - 1) / (kBlock / 64)));
            if (a.src.fused) {
                if (wg) hipLaunchKernelGGL((k_axis_cols_fold<T, OP, 1, true>), fgrid, block, 0, st, a);
                else hipLaunchKernelGGL((k_axis_cols_fold<T, OP, 1, false>), fgrid, block, 0, st, a);
            } else {
                if (wg) hipLaunchKernelGGL((k_axis_cols_fold<T, OP, VW, true>), fgrid, block, 0, st, a);
                else hipLaunchKernelGGL((k_axis_cols_fold<T, OP, VW, false>), fgrid, block, 0, st, a);
            }
        }
    }
}

template <typename T, int OP, int VW>
void launch_axis_vw(const KAxis &a, int cus, hipStream_t st) {
    const bool gen = a.red.ndim > 2;
    switch (miss_kind_of(a.miss.kind) * 2 + (gen ? 1 : 0)) {
        case MK_NONE * 2: launch_axis_k<T, OP, VW, false, MK_NONE>(a, cus, st); break;
        case MK_NONE * 2 + 1: launch_axis_k<T, OP, VW, true, MK_NONE>(a, cus, st); break;
        case MK_CMP * 2: launch_axis_k<T, OP, VW, false, MK_CMP>(a, cus, st); break;
        case MK_CMP * 2 + 1: launch_axis_k<T, OP, VW, true, MK_CMP>(a, cus, st); break;
        case MK_ANY * 2: launch_axis_k<T, OP, VW, false, MK_ANY>(a, cus, st); break;
        default: launch_axis_k<T, OP, VW, true, MK_ANY>(a, cus, st); break;
    }
}

template <typename T, int OP>
hipError_t launch_axis_t(const KAxis &a, int cus, hipStream_t st) {
    if (a.src.fused || a.vec <= 1) launch_axis_vw<T, OP, 1>(a, cus, st);
    else if (a.vec == 2) launch_axis_vw<T, OP, 2>(a, cus, st);
    else if constexpr (sizeof(T) == 4) launch_axis_vw<T, OP, 4>(a, cus, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

template <typename T>
hipError_t launch_axis_op(uint32_t op, const KAxis &a, int cus, hipStream_t s) {
    switch (op) {
        case OP_COUNT: return launch_axis_t<T, OP_COUNT>(a, cus, s);
        case OP_MAX: return launch_axis_t<T, OP_MAX>(a, cus, s);
        case OP_MIN: return launch_axis_t<T, OP_MIN>(a, cus, s);
        case OP_SUM: return launch_axis_t<T, OP_SUM>(a, cus, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace

// One dtype per translation unit (see k_all.hip); the dtype switch lives in k_dispatch.cpp.
hipError_t RDX_KFN(launch_axis)(uint32_t op, const KAxis &a, int cus, hipStream_t s) {
    return launch_axis_op<RDX_T>(op, a, cus, s);
}

}  // namespace rdx
