// Reductions over ALL axes (axis unset: src/operations.rs:139-148, :303-318, :457-473, :622-632).
//
//  k_all_contig  — the selection is one ascending contiguous run of the chunk (whole chunk, or any
//                  hyperslab that canonicalises to one run).  HBM-bound streaming:
//                    * every lane reads 16 B per byte-plane (fused unshuffle, 4 or 8 planes) or
//                      4 x 16 B of plain data per tile: each wave instruction reads 1 KiB contiguous;
//                    * the byte transpose of the unshuffle and the byte-order swap happen in
//                      registers with v_perm_b32 (two stages of 4 perms per 4 elements) — no LDS
//                      round trip is needed because each lane already holds every plane of its
//                      elements;
//                    * per-lane accumulation, a 64-lane butterfly, a 4-wave LDS combine, and one
//                      partial per workgroup folded by the last-arriving workgroup (no 2nd launch).
//  k_all_strided — any other hyperslab: per-element index decomposition with magic division.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) {
    return __builtin_amdgcn_perm(a, b, sel);
}

// 4x4 byte transpose: d[k] holds byte k of elements 0..3 (one dword per byte-plane).  Output w[m] is
// element m assembled little-endian (selA/selB = 0x05040100/0x07060302) or byte-reversed
// (0x00010405/0x02030607, the non-native byte order of array.rs:147-154).
__device__ __forceinline__ void transpose4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t selA,
                                           uint32_t selB, uint32_t w[4]) {
    const uint32_t t01lo = perm(d1, d0, 0x05010400u), t01hi = perm(d1, d0, 0x07030602u);
    const uint32_t t23lo = perm(d3, d2, 0x05010400u), t23hi = perm(d3, d2, 0x07030602u);
    w[0] = perm(t23lo, t01lo, selA);
    w[1] = perm(t23lo, t01lo, selB);
    w[2] = perm(t23hi, t01hi, selA);
    w[3] = perm(t23hi, t01hi, selB);
}

__device__ __forceinline__ uint32_t comp(const uint4 &v, int j) {
    return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// Chunk `chunk`'s base: the argument's own table (read in place from the kernel-argument segment — the
// kernels' only parameter, at offset 0 — so a runtime index does not copy the argument to scratch), the
// device pointer array, or the single chunk.
template <class A>
__device__ __forceinline__ const uint8_t *chunk_ptr(const A &a, uint32_t chunk) {
    if (a.src.table) return (*(const A *)__builtin_amdgcn_kernarg_segment_ptr()).tbl.p[chunk];
    return chunk_base(a.src, chunk);
}

template <typename T, int OP, int MK>
__device__ __forceinline__ void consume(Red<T, OP> &r, T x, const KAllContig &a, uint64_t e) {
    auto rank = [&]() -> int64_t { return a.r0 + (int64_t)(e - a.off) * a.rs; };
    if constexpr (MK != MK_NONE) {
        if (!included_mk<T, MK>(a.miss, x, a.filter_semantics)) return;
    }
    if constexpr (OP == OP_COUNT) r.cnt += 1;
    else r.add(x, rank);
}

// N elements at consecutive indices e0.. .  Float min/max without a missing predicate fold the value
// order-free (v_max/v_min: a NaN operand only sets the error flag, a zero's sign is decided later
// from the ±0 ranks) and compute fold-order ranks only when the group holds a zero, instead of
// evaluating a 64-bit rank per element (f32 min over 8 x 64 MiB: 127 -> 86 us, tools/probe_f64.py).
template <typename T, int OP, int MK, int N>
__device__ __forceinline__ void consume_group(Red<T, OP> &r, const T (&x)[N], const KAllContig &a, uint64_t e0) {
    if constexpr (Red<T, OP>::kRank && MK == MK_NONE) {
        bool nn = false, z = false;
#pragma unroll
        for (int m = 0; m < N; ++m) {
            nn |= x[m] != x[m];
            z |= x[m] == T(0);
            if constexpr (OP == OP_MAX) r.v = __builtin_fmax(r.v, x[m]);
            else r.v = __builtin_fmin(r.v, x[m]);
        }
        r.nan |= nn;
        r.cnt += N;
        if (__builtin_expect(z, 0)) {
#pragma unroll
            for (int m = 0; m < N; ++m) {
                if (x[m] == T(0)) {
                    const int64_t rk = a.r0 + (int64_t)(e0 + m - a.off) * a.rs;
                    if (__builtin_signbit(x[m])) r.zn = OP == OP_MAX ? max(r.zn, rk) : min(r.zn, rk);
                    else r.zp = OP == OP_MAX ? max(r.zp, rk) : min(r.zp, rk);
                }
            }
        }
    } else {
#pragma unroll
        for (int m = 0; m < N; ++m) consume<T, OP, MK>(r, x[m], a, e0 + m);
    }
}

// f64 sums without a missing predicate: groups of a lane's consecutive elements are added pairwise and the
// group's sum enters the compensated (Neumaier) accumulator once.  Integer-valued data stays exact; the
// order of additions already differs from the reference's sequential sum (lanes, then a tree), so no new
// class of deviation: a NaN or an inf anywhere gives the same NaN / inf.
#ifndef RDX_F64_GROUP_SUM
#define RDX_F64_GROUP_SUM 1
#endif
template <typename T, int OP, int MK>
constexpr bool kGroupSum = RDX_F64_GROUP_SUM && OP == OP_SUM && std::is_same_v<T, double> && MK == MK_NONE;

// One tile step for one lane: the 16-byte granules this lane owns in tile `t`.
//   fused   : element granule [e, e+16) with e = t*4096 + lane*16, one 16 B load per plane
//   plain   : 4 granules of 16 B at byte offsets t*16384 + m*4096 + lane*16
template <typename T, bool FUSED>
struct Tile {
    static constexpr int kPlanes = FUSED ? (int)sizeof(T) : 4;
    uint4 p[kPlanes];
};

template <typename T, bool FUSED>
__device__ __forceinline__ uint64_t tile_elems() {
    return FUSED ? (uint64_t)kBlock * 16 : (uint64_t)kBlock * 64 / sizeof(T);
}

// FULL: every lane's granules are inside [va, vb) -> unconditional loads, so all UNR tiles' loads
// issue back to back; the single partial tile of a range goes through the checked variant.
template <typename T, bool FUSED, bool FULL>
__device__ __forceinline__ void load_tile(Tile<T, FUSED> &tl, const uint8_t *base, uint64_t plane, uint64_t t0,
                                          uint64_t vb) {
    if constexpr (FUSED) {
        const uint64_t e = t0 + threadIdx.x * 16;
        if (FULL || e + 16 <= vb) {
#pragma unroll
            for (int k = 0; k < (int)sizeof(T); ++k) tl.p[k] = gld_stream<uint4>(base + (uint64_t)k * plane + e);
        }
    } else {
        const uint8_t *b = base + t0 * sizeof(T);
        const uint64_t lim = (vb - t0) * sizeof(T);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint64_t o = (uint64_t)m * kBlock * 16 + threadIdx.x * 16;
            if (FULL || o + 16 <= lim) tl.p[m] = gld_stream<uint4>(b + o);
        }
    }
}

// UNR full tiles' loads; RDX_PLANE_MAJOR: byte-shuffled 8-byte elements issue plane by plane across the
// tiles (planes 0-3 of every tile, then 4-7) instead of tile by tile
#ifndef RDX_PLANE_MAJOR
#define RDX_PLANE_MAJOR 0
#endif
template <typename T, bool FUSED, int UNR>
__device__ __forceinline__ void load_tiles(Tile<T, FUSED> (&x)[UNR], const uint8_t *base, uint64_t plane,
                                           const uint64_t (&t0)[UNR], uint64_t vb) {
    if constexpr (RDX_PLANE_MAJOR && FUSED && sizeof(T) == 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int u = 0; u < UNR; ++u)
                x[u].p[k] = gld_stream<uint4>(base + (uint64_t)k * plane + t0[u] + threadIdx.x * 16);
    } else {
#pragma unroll
        for (int u = 0; u < UNR; ++u) load_tile<T, FUSED, true>(x[u], base, plane, t0[u], vb);
    }
}

// Byte-shuffled 8-byte elements, split in time (RDX_F8_SPLIT=1, measured, off): planes 0-3 of the UNR
// tiles, a wait until they have all landed, then planes 4-7, so a lane keeps four plane streams busy at a
// time instead of eight.  The stand-alone probe's integer sums liked it (tools/probe_f64lds.hip: 85.3 ->
// 79.3 us for 8 x 64 MiB) but inside this kernel it lost to the pipelined form: f64 84.8 / 82.4 vs 82.4 /
// 82.8 us, i64 86.8 / 87.1 vs 80.7 / 81.0 (profiles/r05_f64_split.jsonl).
#ifndef RDX_F8_SPLIT
#define RDX_F8_SPLIT 0
#endif
template <typename T, int OP, bool FUSED>
constexpr bool kSplit8 = RDX_F8_SPLIT && FUSED && sizeof(T) == 8 && !Red<T, OP>::kRank;

template <typename T, bool FUSED, int UNR>
__device__ __forceinline__ void load_tiles_split(Tile<T, FUSED> (&x)[UNR], const uint8_t *base, uint64_t plane,
                                                 const uint64_t (&t0)[UNR]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) x[u].p[k] = gld_stream<uint4>(base + (uint64_t)k * plane + t0[u] + threadIdx.x * 16);
    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int k = 4; k < 8; ++k) x[u].p[k] = gld_stream<uint4>(base + (uint64_t)k * plane + t0[u] + threadIdx.x * 16);
}

template <typename T, int OP, bool FUSED, int MK, bool FULL>
__device__ __forceinline__ void consume_tile(Red<T, OP> &r, const Tile<T, FUSED> &tl, const KAllContig &a, uint64_t t0,
                                             uint64_t vb, uint32_t selA, uint32_t selB) {
    using U = typename UIntOf<T>::type;
    const bool bswap = a.src.bswap;
    if constexpr (FUSED) {
        const uint64_t e = t0 + threadIdx.x * 16;
        if (!FULL && e + 16 > vb) return;
        if constexpr (OP == OP_COUNT && MK == MK_NONE) {
            r.cnt += 16;
            return;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t lo[4];
            if constexpr (sizeof(T) == 4) {
                transpose4(comp(tl.p[0], j), comp(tl.p[1], j), comp(tl.p[2], j), comp(tl.p[3], j), selA, selB, lo);
                if constexpr (OP == OP_SUM && std::is_same_v<T, float> && MK == MK_NONE) {
                    // pairwise f64 partial of 4 elements (ILP), then one dependent add
                    const double s01 = (double)__builtin_bit_cast(float, lo[0]) + (double)__builtin_bit_cast(float, lo[1]);
                    const double s23 = (double)__builtin_bit_cast(float, lo[2]) + (double)__builtin_bit_cast(float, lo[3]);
                    r.s += s01 + s23;
                    r.cnt += 4;
                } else {
                    T xs[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) xs[m] = from_u<T>((U)lo[m]);
                    consume_group<T, OP, MK, 4>(r, xs, a, e + j * 4);
                }
            } else {
                // 8-byte elements: low dwords from planes 0-3, high from 4-7 (swapped + reversed
                // for the non-native byte order).
                uint32_t hi[4];
                const int A = bswap ? 4 : 0, B = bswap ? 0 : 4;
                transpose4(comp(tl.p[A + 0], j), comp(tl.p[A + 1], j), comp(tl.p[A + 2], j), comp(tl.p[A + 3], j),
                           selA, selB, lo);
                transpose4(comp(tl.p[B + 0], j), comp(tl.p[B + 1], j), comp(tl.p[B + 2], j), comp(tl.p[B + 3], j),
                           selA, selB, hi);
                T xs[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) xs[m] = from_u<T>((U)(((uint64_t)hi[m] << 32) | lo[m]));
                if constexpr (kGroupSum<T, OP, MK>) {
                    // the 4 elements summed pairwise with their rounding errors kept, then one
                    // compensated add (a quarter of the per-element Neumaier steps, the same accuracy)
                    Red<T, OP>::add4(r.s, r.c, (double)xs[0], (double)xs[1], (double)xs[2], (double)xs[3]);
                    r.cnt += 4;
                } else {
                    consume_group<T, OP, MK, 4>(r, xs, a, e + j * 4);
                }
            }
        }
    } else if constexpr (kGroupSum<T, OP, MK>) {
        // plain f64 sums: two granules (4 elements) per compensated step, as the fused form (a step per
        // granule cost 10 % on 8 x 64 MiB: 77 -> 86 us against an i64 sum of the same bytes)
        const uint64_t lim = (vb - t0) * sizeof(T);
#pragma unroll
        for (int m = 0; m < 4; m += 2) {
            const uint64_t o0 = (uint64_t)m * kBlock * 16 + threadIdx.x * 16, o1 = o0 + (uint64_t)kBlock * 16;
            const bool v0 = FULL || o0 + 16 <= lim, v1 = FULL || o1 + 16 <= lim;   // (v1 implies v0)
            uint64_t w[4] = {((uint64_t)tl.p[m].y << 32) | tl.p[m].x, ((uint64_t)tl.p[m].w << 32) | tl.p[m].z,
                             ((uint64_t)tl.p[m + 1].y << 32) | tl.p[m + 1].x, ((uint64_t)tl.p[m + 1].w << 32) | tl.p[m + 1].z};
            double xs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) xs[q] = __builtin_bit_cast(double, bswap ? bswap_u(w[q]) : w[q]);
            if (v1) {
                Red<T, OP>::add4(r.s, r.c, xs[0], xs[1], xs[2], xs[3]);
                r.cnt += 4;
            } else if (v0) {
                Red<T, OP>::add2(r.s, r.c, xs[0], xs[1]);
                r.cnt += 2;
            }
        }
    } else {
        const uint64_t lim = (vb - t0) * sizeof(T);
        constexpr int kPer = 16 / sizeof(T);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint64_t o = (uint64_t)m * kBlock * 16 + threadIdx.x * 16;
            if (!FULL && o + 16 > lim) continue;
            const uint64_t e = t0 + o / sizeof(T);
            if constexpr (OP == OP_COUNT && MK == MK_NONE) {
                r.cnt += kPer;
                continue;
            }
            if constexpr (sizeof(T) == 4) {
                uint32_t w[4] = {tl.p[m].x, tl.p[m].y, tl.p[m].z, tl.p[m].w};
                if constexpr (OP == OP_SUM && std::is_same_v<T, float> && MK == MK_NONE) {
                    float f[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) f[q] = __builtin_bit_cast(float, bswap ? bswap_u(w[q]) : w[q]);
                    r.s += ((double)f[0] + (double)f[1]) + ((double)f[2] + (double)f[3]);
                    r.cnt += 4;
                } else {
                    T xs[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) xs[q] = from_u<T>((U)(bswap ? bswap_u(w[q]) : w[q]));
                    consume_group<T, OP, MK, 4>(r, xs, a, e);
                }
            } else {
                uint64_t w[2] = {((uint64_t)tl.p[m].y << 32) | tl.p[m].x, ((uint64_t)tl.p[m].w << 32) | tl.p[m].z};
                T xs[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) xs[q] = from_u<T>((U)(bswap ? bswap_u(w[q]) : w[q]));
                if constexpr (kGroupSum<T, OP, MK>) {
                    Red<T, OP>::add2(r.s, r.c, (double)xs[0], (double)xs[1]);
                    r.cnt += 2;
                } else {
                    consume_group<T, OP, MK, 2>(r, xs, a, e);
                }
            }
        }
    }
}

// Which loops are software pipelined (next tiles' loads issued before the current ones are folded).
#ifndef RDX_PIPE_SUM
#define RDX_PIPE_SUM 2   // byte-shuffled 8-byte sums (f64 8 x 64 MiB: 85.0 -> 83.4 us; every sum (1): f32 slower)
#endif
template <typename T, int OP, bool FUSED>
constexpr bool kPipelined = !kSplit8<T, OP, FUSED> &&
                            (Red<T, OP>::kRank || (OP == OP_SUM && (RDX_PIPE_SUM == 1 || (RDX_PIPE_SUM == 2 && FUSED && sizeof(T) == 8))));

template <typename T, int OP, bool FUSED, int MK, int UNR>
__global__ __launch_bounds__(kBlock) void k_all_contig(const KAllContig a) {
    RDX_STAMP(0);
    const uint32_t bpc = a.blocks_per_chunk;
    const uint32_t chunk = blockIdx.x / bpc, b = blockIdx.x - chunk * bpc;
    const uint8_t *base = chunk_ptr(a, chunk);
    const bool bswap = a.src.bswap;
    const uint32_t selA = bswap ? 0x00010405u : 0x05040100u;
    const uint32_t selB = bswap ? 0x02030607u : 0x07060302u;

    Red<T, OP> r;
    r.init();
    const uint64_t lo = a.off, hi = a.off + a.n;
    // 16-byte granules: G elements per granule
    constexpr uint64_t G = FUSED ? 16 : 16 / sizeof(T);
    const bool vec_ok = ((uintptr_t)base % 16 == 0) && (!FUSED || a.src.plane % 16 == 0);
    uint64_t va = hi, vb = hi;
    if (vec_ok) {
        va = (lo + G - 1) / G * G;
        vb = hi / G * G;
        if (va >= vb) va = vb = hi;
    }
    // scalar head and tail (< G elements each), owned by workgroup 0 of the chunk
    if (b == 0) {
        for (uint64_t e = lo + threadIdx.x; e < va; e += kBlock)
            consume<T, OP, MK>(r, load_elem<T, FUSED>(base, a.src.plane, bswap, e), a, e);
        for (uint64_t e = vb + threadIdx.x; e < hi; e += kBlock)
            consume<T, OP, MK>(r, load_elem<T, FUSED>(base, a.src.plane, bswap, e), a, e);
    }
    // vector body: full tiles split into contiguous per-workgroup ranges, UNR tiles in flight per
    // lane; the one partial tile (if any) goes to workgroup 0 with the scalar head/tail.  (A dynamic
    // hand-out of the last tiles to the workgroups that finish first was measured slower: the claim
    // round trips cost more than the imbalance, profiles/r02_pool_ab.jsonl.)
    const uint64_t te = tile_elems<T, FUSED>();
    const uint64_t nfull = (vb - va) / te;
#if RDX_TILE_STRIDE
    // tiles b, b + bpc, b + 2 bpc, ...: the chunk's workgroups sweep it together, a window of bpc tiles
    // wide (few DRAM pages / translations live at once) instead of bpc separate streams
    const uint64_t kstride = bpc, k0 = b;
    const uint64_t nk = b < nfull ? (nfull - b + bpc - 1) / bpc : 0;
#else
    const uint64_t per = (nfull + bpc - 1) / bpc;
    const uint64_t t_begin = (uint64_t)b * per;
    const uint64_t t_end = t_begin + per < nfull ? t_begin + per : nfull;
    const uint64_t kstride = 1, k0 = t_begin;
    const uint64_t nk = t_end > t_begin ? t_end - t_begin : 0;
#endif
#if RDX_TILE_ROT
    // each workgroup starts its range at a different point and wraps (decorrelates the DRAM channels the
    // workgroups of a chunk stream from at one time)
    const uint64_t rot = nk ? ((uint64_t)b * 0x9E3779B1u) % nk : 0;
    auto tile = [&](uint64_t k) {
        uint64_t kk = k + rot;
        kk -= kk >= nk ? nk : 0;
        return va + (k0 + kk * kstride) * te;
    };
#else
    auto tile = [&](uint64_t k) { return va + (k0 + k * kstride) * te; };   // first element of the k-th tile
#endif
    uint64_t k = 0;
    // Float min/max (the heaviest per-element fold) are software pipelined: the next UNR tiles'
    // loads are issued before the current UNR tiles are consumed (two register sets, alternating),
    // so a lane's fold work overlaps its next round trip (f32 min over 8 x 64 MiB 86 -> 80 us).  Sums
    // keep the plain loop: pipelined they measured 1-3 % slower (78.6 -> 80.7 us, tools/gpu_pipe.sh).
    if constexpr (kPipelined<T, OP, FUSED>) {
    if (k + UNR <= nk) {
        Tile<T, FUSED> x[UNR], y[UNR];
        auto tiles_at = [&](uint64_t k0_, uint64_t (&t)[UNR]) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) t[u] = tile(k0_ + u);
        };
        {
            uint64_t t[UNR];
            tiles_at(k, t);
            load_tiles<T, FUSED, UNR>(x, base, a.src.plane, t, vb);
        }
        while (true) {
            const bool m1 = k + 2 * UNR <= nk;
            if (m1) {
                uint64_t t[UNR];
                tiles_at(k + UNR, t);
                load_tiles<T, FUSED, UNR>(y, base, a.src.plane, t, vb);
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) consume_tile<T, OP, FUSED, MK, true>(r, x[u], a, tile(k + u), vb, selA, selB);
            k += UNR;
            if (!m1) break;
            const bool m2 = k + 2 * UNR <= nk;
            if (m2) {
                uint64_t t[UNR];
                tiles_at(k + UNR, t);
                load_tiles<T, FUSED, UNR>(x, base, a.src.plane, t, vb);
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) consume_tile<T, OP, FUSED, MK, true>(r, y[u], a, tile(k + u), vb, selA, selB);
            k += UNR;
            if (!m2) break;
        }
    }
    } else if constexpr (kSplit8<T, OP, FUSED>) {
    for (; k + UNR <= nk; k += UNR) {
        Tile<T, FUSED> x[UNR];
        uint64_t t[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) t[u] = tile(k + u);
        load_tiles_split<T, FUSED, UNR>(x, base, a.src.plane, t);
#pragma unroll
        for (int u = 0; u < UNR; ++u) consume_tile<T, OP, FUSED, MK, true>(r, x[u], a, t[u], vb, selA, selB);
    }
    } else {
    for (; k + UNR <= nk; k += UNR) {
        Tile<T, FUSED> x[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) load_tile<T, FUSED, true>(x[u], base, a.src.plane, tile(k + u), vb);
#pragma unroll
        for (int u = 0; u < UNR; ++u) consume_tile<T, OP, FUSED, MK, true>(r, x[u], a, tile(k + u), vb, selA, selB);
    }
    }
    for (; k < nk; ++k) {
        Tile<T, FUSED> x0;
        load_tile<T, FUSED, true>(x0, base, a.src.plane, tile(k), vb);
        consume_tile<T, OP, FUSED, MK, true>(r, x0, a, tile(k), vb, selA, selB);
    }
    if (b == 0 && va + nfull * te < vb) {
        Tile<T, FUSED> x0;
        load_tile<T, FUSED, false>(x0, base, a.src.plane, va + nfull * te, vb);
        consume_tile<T, OP, FUSED, MK, false>(r, x0, a, va + nfull * te, vb, selA, selB);
    }
    RDX_STAMP(1);
    finalize_all<T, OP>(r, a.out, chunk, bpc, b);
}

// ---- strided views ---------------------------------------------------------------------------------
// VW > 1: the innermost canonical dim is contiguous (stride 1), its count and every other stride are
// multiples of VW and the origin is VW-aligned, so each lane loads VW consecutive elements with one
// 16-byte global_load.  U vectors per lane are in flight at once; the host sizes the grid so a
// lane normally needs a single round trip.
// ND > 0: the view has exactly ND canonical dims, known at compile time.  The dims' counts, magic
// divisors and strides are then read from the kernel arguments once, up front (all scalar loads
// issued together), instead of inside the per-vector decomposition loop, where every dim of every
// vector waited for its own scalar-cache miss on a cold launch (~5 us of an 11 us C3 launch).
// ND == 0: any ndim (<= kMaxKDims), read in the loop.
template <int ND>
struct DimRegs {
    static constexpr int N = ND > 0 ? ND : 1;
    uint32_t count[N];
    uint64_t magic[N];
    int64_t vstride[N], rstride[N];
    __device__ __forceinline__ void load(const KView &v) {
        if constexpr (ND > 0) {
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                count[k] = v.count[k];
                magic[k] = v.div[k].magic;
                vstride[k] = v.vstride[k];
                rstride[k] = v.rstride[k];
            }
        }
    }
};

// element offset and fold rank of flattened index q (innermost-first digits)
template <int ND, bool RANK>
__device__ __forceinline__ void decompose(const KView &v, const DimRegs<ND> &d, uint32_t q, int64_t &o, int64_t &rr) {
    o = v.base_off;
    rr = v.r0;
    if constexpr (ND > 0) {
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            const uint32_t qn = udiv(q, d.magic[k]);
            const uint32_t idx = q - qn * d.count[k];
            o += (int64_t)idx * d.vstride[k];
            if constexpr (RANK) rr += (int64_t)idx * d.rstride[k];
            q = qn;
        }
    } else {
        for (int k = 0; k < v.ndim; ++k) {
            const uint32_t qn = udiv(q, v.div[k].magic);
            const uint32_t idx = q - qn * v.count[k];
            o += (int64_t)idx * v.vstride[k];
            if constexpr (RANK) rr += (int64_t)idx * v.rstride[k];
            q = qn;
        }
    }
}

template <typename T, int OP, bool FUSED, int VW, int ND, int MK>
__global__ __launch_bounds__(kBlock) void k_all_strided(const KAllStrided a) {
    RDX_STAMP(0);
    constexpr int kU = VW > 1 ? 4 : 8;
    const uint32_t bpc = a.blocks_per_chunk;
    const uint32_t chunk = blockIdx.x / bpc, b = blockIdx.x - chunk * bpc;
    const uint8_t *base = chunk_ptr(a, chunk);
    const bool bswap = a.src.bswap;
    const KView &v = a.view;
    DimRegs<ND> d;
    d.load(v);
    const int64_t rs0 = ND > 0 ? d.rstride[0] : v.rstride[0];
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
            decompose<ND, Red<T, OP>::kRank>(v, d, (uint32_t)(g * VW), off[u], rk[u]);
        }
        Raw<T, FUSED, VW> raw[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_load(raw[u], base, a.src.plane, (uint64_t)off[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_pin(raw[u]);   // (no load sunk into its ok[u] branch)
#pragma unroll
        for (int u = 0; u < kU; ++u) raw_cvt(raw[u], bswap, x[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (!ok[u]) continue;
#pragma unroll
            for (int j = 0; j < VW; ++j) {
                if (!included_mk<T, MK>(a.miss, x[u][j], a.filter_semantics)) continue;
                if constexpr (OP == OP_COUNT) r.cnt += 1;
                else r.add(x[u][j], [&]() { return rk[u] + (int64_t)j * rs0; });
            }
        }
    }
    RDX_STAMP(1);
    finalize_all<T, OP>(r, a.out, chunk, bpc, b);
}

template <typename T, int OP, int UNR>
void launch_contig_u(const KAllContig &a, dim3 grid, hipStream_t s) {
    const dim3 block(kBlock);
    const int mk = miss_kind_of(a.miss.kind);
#define RDX_CONTIG(F, M) hipLaunchKernelGGL((k_all_contig<T, OP, F, M, UNR>), grid, block, 0, s, a)
    if (a.src.fused) {
        if (mk == MK_NONE) RDX_CONTIG(true, MK_NONE);
        else if (mk == MK_CMP) RDX_CONTIG(true, MK_CMP);
        else RDX_CONTIG(true, MK_ANY);
    } else {
        if (mk == MK_NONE) RDX_CONTIG(false, MK_NONE);
        else if (mk == MK_CMP) RDX_CONTIG(false, MK_CMP);
        else RDX_CONTIG(false, MK_ANY);
    }
#undef RDX_CONTIG
}

#ifndef RDX_UNR_F8
#define RDX_UNR_F8 2   // tiles in flight per lane for byte-shuffled 8-byte elements (8 plane loads per tile)
#endif

template <typename T, int OP>
hipError_t launch_contig_t(const KAllContig &a, uint32_t n_chunks, hipStream_t s) {
    const dim3 grid(a.blocks_per_chunk * n_chunks);
    // 2 tiles in flight per lane at one workgroup per CU: 4 tiles, or 2/4/6/8 workgroups per CU,
    // measured slower with non-temporal loads (tools/gpu_bpcu.sh, gpurun_out/bpcu*).
    if (sizeof(T) == 8 && a.src.fused) launch_contig_u<T, OP, RDX_UNR_F8>(a, grid, s);
    else launch_contig_u<T, OP, 2>(a, grid, s);
    return hipGetLastError();
}

template <typename T, int OP, bool FUSED, int VW, int MK>
void launch_strided_nd(const KAllStrided &a, uint32_t n_chunks, hipStream_t s) {
    const dim3 grid(a.blocks_per_chunk * n_chunks), block(kBlock);
    switch (a.view.ndim) {   // canonical views of up to 4 dims cover the 1-4-D arrays of the API
        case 1: hipLaunchKernelGGL((k_all_strided<T, OP, FUSED, VW, 1, MK>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_all_strided<T, OP, FUSED, VW, 2, MK>), grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL((k_all_strided<T, OP, FUSED, VW, 3, MK>), grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL((k_all_strided<T, OP, FUSED, VW, 4, MK>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((k_all_strided<T, OP, FUSED, VW, 0, MK>), grid, block, 0, s, a); break;
    }
}

template <typename T, int OP, bool FUSED, int VW>
void launch_strided_mk(const KAllStrided &a, uint32_t n_chunks, hipStream_t s) {
    switch (miss_kind_of(a.miss.kind)) {
        case MK_NONE: launch_strided_nd<T, OP, FUSED, VW, MK_NONE>(a, n_chunks, s); break;
        case MK_CMP: launch_strided_nd<T, OP, FUSED, VW, MK_CMP>(a, n_chunks, s); break;
        default: launch_strided_nd<T, OP, FUSED, VW, MK_ANY>(a, n_chunks, s); break;
    }
}

template <typename T, int OP>
hipError_t launch_strided_t(const KAllStrided &a, uint32_t n_chunks, hipStream_t s) {
    constexpr int VW = 16 / sizeof(T);
    if (a.src.fused) launch_strided_mk<T, OP, true, 1>(a, n_chunks, s);
    else if (a.vec > 1) launch_strided_mk<T, OP, false, VW>(a, n_chunks, s);
    else launch_strided_mk<T, OP, false, 1>(a, n_chunks, s);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_contig_op(uint32_t op, const KAllContig &a, uint32_t n, hipStream_t s) {
    switch (op) {
        case OP_COUNT: return launch_contig_t<T, OP_COUNT>(a, n, s);
        case OP_MAX: return launch_contig_t<T, OP_MAX>(a, n, s);
        case OP_MIN: return launch_contig_t<T, OP_MIN>(a, n, s);
        case OP_SUM: return launch_contig_t<T, OP_SUM>(a, n, s);
    }
    return hipErrorInvalidValue;
}

template <typename T>
hipError_t launch_strided_op(uint32_t op, const KAllStrided &a, uint32_t n, hipStream_t s) {
    switch (op) {
        case OP_COUNT: return launch_strided_t<T, OP_COUNT>(a, n, s);
        case OP_MAX: return launch_strided_t<T, OP_MAX>(a, n, s);
        case OP_MIN: return launch_strided_t<T, OP_MIN>(a, n, s);
        case OP_SUM: return launch_strided_t<T, OP_SUM>(a, n, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace

// One dtype per translation unit (the Makefile builds this file once per RDX_T, in parallel); the
// dtype switch lives in k_dispatch.cpp.
hipError_t RDX_KFN(launch_all_contig)(uint32_t op, const KAllContig &a, uint32_t n_chunks, hipStream_t s) {
    return launch_contig_op<RDX_T>(op, a, n_chunks, s);
}

hipError_t RDX_KFN(launch_all_strided)(uint32_t op, const KAllStrided &a, uint32_t n_chunks, hipStream_t s) {
    return launch_strided_op<RDX_T>(op, a, n_chunks, s);
}

#if RDX_PROBES
}  // namespace rdx
// probe builds: the phase timeline of the last all-axes launch of this dtype (rdx_device.hpp RDX_STAMP)
extern "C" int RDX_KFN(rdx_probe_read)(uint64_t *host, uint32_t n) {
    if (n > 8 * 8192) n = 8 * 8192;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rdx::g_rdx_probe), n * sizeof(uint64_t)) == hipSuccess ? 0 : 1;
}
namespace rdx {
#endif

}  // namespace rdx
