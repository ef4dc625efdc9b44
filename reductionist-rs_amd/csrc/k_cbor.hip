// Response serialisation on the device (include/rdx.h rdx_cbor_encode_device): the CBOR body of
// serde_cbor::to_vec(&CBORResponse::new(&response)) (src/app.rs:33-40, src/models.rs:355-416) written
// from device-resident outputs, so a large count vector (axis reductions with many outputs, axis = [])
// is packed where it was computed and only the packed bytes cross PCIe.
//
// The host-known segments (map head, keys, dtype, shape, the array / byte-string heads: rdx_cbor.hpp)
// travel in the kernel arguments; the body and a count_as_bytes payload are copied by the same launch
// (every workgroup a share, 16-byte loads, dword-aligned 16-byte stores) when the alignments allow.  What needs the device is the count ARRAY: every i64 becomes a CBOR
// integer of 1, 2, 3, 5 or 9 bytes, so each count's output offset is an exclusive prefix sum of the
// encoded lengths.  Reduce, scan, encode (three launches, no cross-workgroup waiting): k_cbor_agg sums the
// encoded lengths of each tile of 2048 counts, k_cbor_scan turns the tile sums into exclusive offsets (one
// workgroup), and k_cbor (workgroup t: tile t) scans its lengths in registers and LDS, encodes the tile
// into LDS and writes it out contiguously at its offset.  The last tile writes the trailing segments after
// the array and the total length.  (A one-pass decoupled look-back over tagged tile records measured 172
// us for 32 Mi counts: each tile's walk back to an inclusive prefix, not bytes, bounded it; a 256-wide
// look-back window, and resident workgroups with the next tile prefetched, measured slower still.)
//
// Roofline: HBM.  Algorithmic bytes per launch = 8 B read + 1-9 B written per count.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

constexpr int kCborPer = 8;                       // counts per thread (four 16-byte loads)
constexpr int kCborTile = kBlock * kCborPer;      // counts per tile

__device__ __forceinline__ uint32_t int_len(int64_t v) {
    const uint64_t u = v < 0 ? ~(uint64_t)v : (uint64_t)v;   // -1 - v for negatives
    return u < 24 ? 1u : u <= 0xffu ? 2u : u <= 0xffffu ? 3u : u <= 0xffffffffull ? 5u : 9u;
}

__device__ __forceinline__ uint32_t put_int(uint8_t *p, int64_t v) {   // p in LDS
    const uint8_t major = v < 0 ? 0x20 : 0x00;
    const uint64_t u = v < 0 ? ~(uint64_t)v : (uint64_t)v;
    if (u < 24) {
        p[0] = (uint8_t)(major | u);
        return 1;
    }
    const int n = u <= 0xffu ? 1 : u <= 0xffffu ? 2 : u <= 0xffffffffull ? 4 : 8;
    p[0] = (uint8_t)(major | (n == 1 ? 24 : n == 2 ? 25 : n == 4 ? 26 : 27));
    for (int i = 0; i < n; ++i) p[1 + i] = (uint8_t)(u >> (8 * (n - 1 - i)));
    return 1u + (uint32_t)n;
}

// Stores through the GLOBAL address space (a generic store is a flat store, which also counts against
// lgkmcnt, so LDS reads issued after it would wait for it).
__device__ __forceinline__ void gst8(uint8_t *p, uint8_t v) { *(__attribute__((address_space(1))) uint8_t *)p = v; }
__device__ __forceinline__ void gst32(uint8_t *p, uint32_t v) { *(__attribute__((address_space(1))) uint32_t *)p = v; }

__device__ void put_tail(const KCbor &m, uint64_t clen) {   // D and F after the count array
    uint8_t *d = m.out + m.c_off + clen;
    for (uint32_t i = threadIdx.x; i < m.d_len; i += kBlock) gst8(d + i, m.tail[i]);
    uint8_t *f = d + m.d_len + m.raw_len;
    for (uint32_t i = threadIdx.x; i < m.f_len; i += kBlock) gst8(f + i, m.tail[m.d_len + i]);
}

// This workgroup's share of a device-to-device copy (the body; the count_as_bytes payload): src 16-byte
// aligned, dst 4-byte aligned (the host checks both; else it copies with hipMemcpyAsync), 16-byte loads
// and dword-aligned 16-byte stores, the < 16 byte tail by workgroup 0.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ void copy_share(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const uint64_t units = n / 16;
    const uint64_t per = (units + gridDim.x - 1) / gridDim.x;
    const uint64_t u0 = (uint64_t)blockIdx.x * per, u1 = u0 + per < units ? u0 + per : units;
    for (uint64_t u = u0 + threadIdx.x; u < u1; u += kBlock) {
        const uint4 v = gld_stream<uint4>(src + 16 * u);
        u32x4_a4 w = {v.x, v.y, v.z, v.w};
        *(__attribute__((address_space(1))) u32x4_a4 *)(dst + 16 * u) = w;
    }
    if (blockIdx.x == 0)
        for (uint64_t i = units * 16 + threadIdx.x; i < n; i += kBlock) gst8(dst + i, gld<uint8_t>(src + i));
}

// this thread's 8 counts of tile `tile` (zeros past the end)
__device__ __forceinline__ void load_counts(const KCbor &m, uint64_t i0, int64_t (&v)[kCborPer]) {
    if (m.vec && i0 + kCborPer <= m.n) {
#pragma unroll
        for (int k = 0; k < kCborPer / 2; ++k) {
            const uint4 q = gld_stream<uint4>(m.counts + i0 + 2 * k);
            v[2 * k] = (int64_t)(((uint64_t)q.y << 32) | q.x);
            v[2 * k + 1] = (int64_t)(((uint64_t)q.w << 32) | q.z);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kCborPer; ++k) v[k] = i0 + k < m.n ? gld<int64_t>(m.counts + i0 + k) : 0;
    }
}

// 1. tile t's encoded length -> records[t]: one wavefront per tile, all of a lane's loads in flight at once
// (16 x 16 B); wavefronts loop over tiles (a workgroup per tile, 16 KiB each, ran at 3.9 TB/s)
constexpr int kAggQ = kCborTile / 2 / 64;   // 16-byte loads per lane and tile
__global__ __launch_bounds__(kBlock) void k_cbor_agg(const KCbor args) {
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t t = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); t < m.n_tiles; t += nw) {
        const uint64_t e0 = t * kCborTile;
        uint64_t sum = 0;
        if (m.vec && e0 + kCborTile <= m.n) {
            uint4 q[kAggQ];
#pragma unroll
            for (int k = 0; k < kAggQ; ++k) q[k] = gld_stream<uint4>(m.counts + e0 + 2 * (lane + 64 * k));
#pragma unroll
            for (int k = 0; k < kAggQ; ++k)
                sum += int_len((int64_t)(((uint64_t)q[k].y << 32) | q[k].x)) + int_len((int64_t)(((uint64_t)q[k].w << 32) | q[k].z));
        } else {
            for (uint64_t e = e0 + lane; e < m.n && e < e0 + kCborTile; e += 64) sum += int_len(gld<int64_t>(m.counts + e));
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) sum += (uint64_t)__shfl_xor((long long)sum, d, 64);
        if (lane == 0) m.records[t] = sum;
    }
}

// 2. exclusive offsets of the tiles, in place: one workgroup of 1024, passes of 16384 tiles read and written
// coalesced through LDS (128 KiB; thread-contiguous runs of 16 for the scan): one load round trip per pass
constexpr uint32_t kScanThreads = 1024, kScanPer = 16;
__global__ __launch_bounds__(kScanThreads) void k_cbor_scan(const KCbor args) {
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ uint64_t buf[kScanThreads * kScanPer];
    __shared__ uint64_t wsum[kScanThreads / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < m.n_tiles; b0 += (uint64_t)kScanThreads * kScanPer) {
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; ++k) {
            const uint64_t j = b0 + k * kScanThreads + t;
            buf[k * kScanThreads + t] = j < m.n_tiles ? m.records[j] : 0;
        }
        __syncthreads();
        uint64_t v[kScanPer], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; ++k) {
            v[k] = buf[kScanPer * t + k];
            sum += v[k];
        }
        uint64_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = (uint64_t)__shfl_up((long long)x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint64_t base = carry, tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < kScanThreads / 64; ++w) {
            base += w < wave ? wsum[w] : 0;
            tot += wsum[w];
        }
        uint64_t run = base + x - sum;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; ++k) {
            buf[kScanPer * t + k] = run;
            run += v[k];
        }
        carry += tot;
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; ++k) {
            const uint64_t j = b0 + k * kScanThreads + t;
            if (j < m.n_tiles) m.records[j] = buf[k * kScanThreads + t];
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kBlock) void k_cbor([[maybe_unused]] const KCbor args) {
    // read in place from the kernel-argument segment (the only parameter): no scratch copy of the
    // fixed byte arrays
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ uint32_t stage32[(kCborTile * 9 + 8) / 4];   // the encoded tile, at dst's alignment mod 4
    uint8_t *const stage = reinterpret_cast<uint8_t *>(stage32);
    __shared__ uint32_t wsum[kBlock / 64];
    __shared__ uint64_t s_excl;
    if (blockIdx.x == 0) {   // A at 0, B after the body
        for (uint32_t i = threadIdx.x; i < m.a_len; i += kBlock) gst8(m.out + i, m.fixed[i]);
        for (uint32_t i = threadIdx.x; i < m.b_len; i += kBlock) gst8(m.out + m.b_off + i, m.fixed[m.a_len + i]);
        if (m.n_tiles == 0) {   // no count array: D and F right after B
            put_tail(m, 0);
            if (threadIdx.x == 0) gst<uint64_t>(m.out_len, m.c_off + m.d_len + m.raw_len + m.f_len);
        }
    }
    const uint32_t tile = blockIdx.x;   // tiles in workgroup order; copy-only workgroups past n_tiles
    if (tile < m.n_tiles) {
        if (threadIdx.x == 0) s_excl = m.records[tile];   // k_cbor_scan's offset of the tile (issued first)
        const uint64_t i0 = (uint64_t)tile * kCborTile + (uint64_t)threadIdx.x * kCborPer;
        int64_t v[kCborPer];
        load_counts(m, i0, v);
        uint32_t len = 0;
#pragma unroll
        for (int k = 0; k < kCborPer; ++k) len += i0 + k < m.n ? int_len(v[k]) : 0u;
        // block exclusive scan of the per-thread lengths
        const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint32_t x = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t base = 0, agg = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) {
            base += w < (int)wave ? wsum[w] : 0u;
            agg += wsum[w];
        }
        const uint32_t off = base + x - len;
        // encode the tile into LDS at the thread's offset, shifted by dst's misalignment so that LDS dwords
        // line up with the destination's; then whole dwords out (bytes at the two ends)
        const uint64_t excl = s_excl;
        uint8_t *dst = m.out + m.c_off + excl;
        const uint32_t sh = (uint32_t)((uintptr_t)dst & 3);
        uint32_t o = sh + off;
#pragma unroll
        for (int k = 0; k < kCborPer; ++k)
            if (i0 + k < m.n) o += put_int(stage + o, v[k]);
        __syncthreads();
        const uint32_t end = sh + agg;                    // stage bytes [sh, end) -> dst[0, agg)
        const uint32_t w0 = (sh + 3) / 4, w1 = end / 4;   // whole dwords [w0, w1)
        uint8_t *const dst0 = dst - sh;                   // dword aligned
        if (w0 < w1) {
            for (uint32_t w = w0 + threadIdx.x; w < w1; w += kBlock) gst32(dst0 + 4 * w, stage32[w]);
            if (threadIdx.x < 4 * w0 - sh) gst8(dst + threadIdx.x, stage[sh + threadIdx.x]);
            if (threadIdx.x < end - 4 * w1) gst8(dst0 + 4 * w1 + threadIdx.x, stage[4 * w1 + threadIdx.x]);
        } else {
            for (uint32_t i = threadIdx.x; i < agg; i += kBlock) gst8(dst + i, stage[sh + i]);
        }
        if (tile == m.n_tiles - 1) {
            put_tail(m, excl + agg);
            if (threadIdx.x == 0) gst<uint64_t>(m.out_len, m.c_off + excl + agg + m.d_len + m.raw_len + m.f_len);
        }
    }
    // this workgroup's share of the body / count_as_bytes copies
    if (m.copy_body) copy_share(m.out + m.a_len, m.body, m.body_len);
    if (m.copy_raw) copy_share(m.out + m.c_off + m.d_len, reinterpret_cast<const uint8_t *>(m.counts), m.raw_len);
}

// ---- the staged form (round 5): pack -> scan -> place -----------------------------------------------------
// The count array is read ONCE.  k_cbor_pack: workgroup g owns the contiguous tiles [g T, g T + T) and its
// waves take them in turn; a tile's 32 counts per lane are loaded as agg loads them (all 16 loads in
// flight) and encoded straight into the tile's staging slot in global memory, round by round (per load
// round a wave-wide exclusive scan of the lanes' lengths; a round whose 128 counts all take one byte — the
// counts of axis = [] responses — is one 16-bit store per lane, no scan).  The workgroup then scans its
// tiles' lengths (records[t] = local offset << 32 | length) and publishes its total as a tagged granule;
// the last workgroup to arrive scans the G totals into group offsets (records[n_tiles + 1 + g]) and the
// grand total (records[n_tiles]).  k_cbor_place: one wavefront per tile copies the staged bytes to their
// offset (dword stores built with v_alignbyte from 16-byte loads), the segments and the trailer as k_cbor
// does.  Bytes moved: counts (8 B per count) once + the encoded bytes three times (staged write, read, final
// write), against counts twice + encoded once for agg / scan / encode: less for every count array whose
// counts take under ~3.5 bytes on average.  (Records: profiles/r05_cbor_staged.jsonl.)
constexpr uint32_t kStageWave = (uint32_t)kCborTile * 9 + 16;   // a tile's worst case, 16-byte multiple
static_assert(kStageWave % 16 == 0, "staging slots stay 16-byte aligned");
constexpr uint32_t kPackMaxT = 1024;   // tiles per workgroup (host: n_tiles <= 2048 * 1024, i.e. < 2^32 counts)
constexpr uint32_t kPackMaxG = 2048;   // workgroups

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t lane, uint32_t &total) {
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
    }
    total = __shfl(inc, 63, 64);
    return inc - x;
}

__device__ __forceinline__ uint32_t put_int_global(uint8_t *p, int64_t v) {
    const uint8_t major = v < 0 ? 0x20 : 0x00;
    const uint64_t u = v < 0 ? ~(uint64_t)v : (uint64_t)v;
    if (u < 24) {
        gst8(p, (uint8_t)(major | u));
        return 1;
    }
    const int n = u <= 0xffu ? 1 : u <= 0xffffu ? 2 : u <= 0xffffffffull ? 4 : 8;
    gst8(p, (uint8_t)(major | (n == 1 ? 24 : n == 2 ? 25 : n == 4 ? 26 : 27)));
    for (int i = 0; i < n; ++i) gst8(p + 1 + i, (uint8_t)(u >> (8 * (n - 1 - i))));
    return 1u + (uint32_t)n;
}

__global__ __launch_bounds__(kBlock) void k_cbor_pack(const KCbor args) {
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ uint32_t s_len[kPackMaxT];
    __shared__ uint64_t s_tot[kBlock / 64];
    __shared__ uint32_t s_last, s_fault;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t T = m.tpg, g = blockIdx.x;
    const uint64_t t0 = (uint64_t)g * T;
    const uint32_t nt = (uint32_t)(t0 < m.n_tiles ? std::min<uint64_t>(T, m.n_tiles - t0) : 0);
    // a wave's tiles i, i + 4, ...: load, then encode.  (RDX_CBOR_PACK_PIPE=1 issues the next tile's loads
    // before the current one is encoded, two register sets in turn: 216 VGPRs, two waves per SIMD instead of
    // three, and pack 61.9 -> 73.7 us for 32 Mi counts, profiles/r05_cbor_staged.jsonl: off)
    auto load = [&](uint32_t i, uint4 (&q)[kAggQ]) {
        const uint64_t e0 = (t0 + i) * kCborTile;
        if (m.vec && e0 + kCborTile <= m.n) {
#pragma unroll
            for (int k = 0; k < kAggQ; ++k) q[k] = gld_stream<uint4>(m.counts + e0 + 2 * (lane + 64 * k));
        } else {
#pragma unroll
            for (int k = 0; k < kAggQ; ++k) {
                const uint64_t e = e0 + 2 * (lane + 64 * k);
                const uint64_t a = e < m.n ? (uint64_t)gld<int64_t>(m.counts + e) : 0, b = e + 1 < m.n ? (uint64_t)gld<int64_t>(m.counts + e + 1) : 0;
                q[k] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
            }
        }
    };
    auto encode = [&](uint32_t i, const uint4 (&q)[kAggQ]) {
        const uint64_t t = t0 + i, e0 = t * kCborTile;
        const bool full = m.vec && e0 + kCborTile <= m.n;
        uint8_t *const dst = m.stage + t * kStageWave;
        uint32_t base = 0;
#pragma unroll
        for (int k = 0; k < kAggQ; ++k) {
            const uint64_t e = e0 + 2 * (lane + 64 * k);
            const int64_t v0 = (int64_t)(((uint64_t)q[k].y << 32) | q[k].x), v1 = (int64_t)(((uint64_t)q[k].w << 32) | q[k].z);
            const bool in0 = full || e < m.n, in1 = full || e + 1 < m.n;
            const bool small = (!in0 || (uint64_t)v0 < 24) && (!in1 || (uint64_t)v1 < 24) && in0 == in1;
            if (__builtin_amdgcn_ballot_w64(!small) == 0 && (full || e0 + 128 * (k + 1) <= m.n)) {
                if (base & 1) {   // (wave-uniform) an odd start: two byte stores instead of an unaligned one
                    gst8(dst + base + 2 * lane, (uint8_t)v0);
                    gst8(dst + base + 2 * lane + 1, (uint8_t)v1);
                } else {
                    *(__attribute__((address_space(1))) uint16_t *)(dst + base + 2 * lane) = (uint16_t)((uint32_t)v0 | (uint32_t)v1 << 8);
                }
                base += 128;
                continue;
            }
            const uint32_t l0 = in0 ? int_len(v0) : 0u, l1 = in1 ? int_len(v1) : 0u;
            uint32_t tot;
            const uint32_t off = base + wave_excl_scan(l0 + l1, lane, tot);
            if (l0) put_int_global(dst + off, v0);
            if (l1) put_int_global(dst + off + l0, v1);
            base += tot;
        }
        if (lane == 0) s_len[i] = base;
    };
#ifndef RDX_CBOR_PACK_PIPE
#define RDX_CBOR_PACK_PIPE 0
#endif
    if (RDX_CBOR_PACK_PIPE) {
        uint4 x[kAggQ], y[kAggQ];
        uint32_t i = wave;
        if (i < nt) load(i, x);
        while (i < nt) {
            const uint32_t i1 = i + kBlock / 64;
            if (i1 < nt) load(i1, y);
            encode(i, x);
            if (i1 >= nt) break;
            const uint32_t i2 = i1 + kBlock / 64;
            if (i2 < nt) load(i2, x);
            encode(i1, y);
            i = i2;
        }
    } else {
        for (uint32_t i = wave; i < nt; i += kBlock / 64) {
            uint4 q[kAggQ];
            load(i, q);
            encode(i, q);
        }
    }
    __syncthreads();
    // this workgroup's tiles: local exclusive offsets (wave 0, 64 tiles per step) and the group total
    if (wave == 0) {
        uint64_t run = 0;
        for (uint32_t i0 = 0; i0 < nt; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint32_t len = i < nt ? s_len[i] : 0u;
            uint32_t tot;
            const uint32_t ex = wave_excl_scan(len, lane, tot);
            if (i < nt) m.records[t0 + i] = (run + ex) << 32 | len;
            run += tot;
        }
        if (lane == 0) {
            put_granule(m.tagged + g, run, m.epoch);
            s_last = arrive_last(m.arrive, gridDim.x, g);
            s_fault = 0;
        }
    }
    __syncthreads();
    if (!s_last) return;
    // the last workgroup: group offsets (thread-contiguous runs of kPer totals, tagged granules polled)
    constexpr uint32_t kPer = kPackMaxG / kBlock;
    const uint32_t G = gridDim.x;
    uint64_t v[kPer], sum = 0;
    uint32_t fault = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t j = threadIdx.x * kPer + k;
        uint64_t x = 0;
        if (j < G) {
            x = __hip_atomic_load(m.tagged + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_expect((uint32_t)(x >> 48) != m.epoch, 0)) {
                if (!fault) x = poll_granule(m.tagged + j, m.epoch);   // (one spin budget per lane)
                fault |= (uint32_t)(x >> 48) != m.epoch;
            }
        }
        v[k] = x & kPayload;
        sum += v[k];
    }
    uint64_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = (uint64_t)__shfl_up((long long)x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_tot[wave] = x;
    if (fault) s_fault = 1;   // (benign race: every writer stores 1)
    __syncthreads();
    // a group total that never arrived (a device fault) leaves stale payloads behind: every group offset and
    // the total are then 0, so k_cbor_place writes only inside the output bound (tiles overlap; the status
    // word carries RDX_E_DEVICE and the response is discarded)
    const bool bad = s_fault != 0;
    uint64_t pre = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBlock / 64; ++w) {
        pre += w < wave ? s_tot[w] : 0;
        all += s_tot[w];
    }
    uint64_t run = pre + x - sum;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t j = threadIdx.x * kPer + k;
        if (j < G) m.records[m.n_tiles + 1 + j] = bad ? 0 : run;
        run += v[k];
    }
    if (threadIdx.x == 0) {
        m.records[m.n_tiles] = bad ? 0 : all;
        __hip_atomic_store(m.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // the top counter
    }
    if (fault && m.status) __hip_atomic_fetch_or(m.status, (uint32_t)RDX_E_DEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the staged tile t -> out + c_off + offset: lane i writes destination dwords 4i..4i+3 (relative to the
// dword-aligned base below dst) built from the staged dwords 4i-1..4i+3 (v_alignbyte), bytes at the ends
__global__ __launch_bounds__(kBlock) void k_cbor_place(const KCbor args) {
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (blockIdx.x == 0) {   // A at 0, B after the body
        for (uint32_t i = threadIdx.x; i < m.a_len; i += kBlock) gst8(m.out + i, m.fixed[i]);
        for (uint32_t i = threadIdx.x; i < m.b_len; i += kBlock) gst8(m.out + m.b_off + i, m.fixed[m.a_len + i]);
        if (m.n_tiles == 0) {
            put_tail(m, 0);
            if (threadIdx.x == 0) gst<uint64_t>(m.out_len, m.c_off + m.d_len + m.raw_len + m.f_len);
        }
    }
    const uint64_t nw = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t t = (uint64_t)blockIdx.x * (kBlock / 64) + wave; t < m.n_tiles; t += nw) {
        const uint64_t r = m.records[t];
        const uint64_t off = m.records[m.n_tiles + 1 + t / m.tpg] + (r >> 32), len = r & 0xffffffffu;
        const uint8_t *src = m.stage + t * kStageWave;
        uint8_t *dst = m.out + m.c_off + off;
        const uint32_t sh = (uint32_t)((uintptr_t)dst & 3);
        uint8_t *const dst0 = dst - sh;
        // destination dword w (0 <= w < nd) holds tile bytes [4w - sh, 4w - sh + 4)
        const uint64_t nd = (sh + len + 3) / 4;
        uint32_t carry = 0;   // staged dword 4i - 1 (the previous lane's last, or the previous pass's)
        for (uint64_t i0 = 0; 4 * i0 < nd; i0 += 64) {
            const uint64_t i = i0 + lane;
            uint4 x = make_uint4(0, 0, 0, 0);
            if (16 * i < len + 16) x = gld<uint4>(reinterpret_cast<const uint4 *>(src + 16 * i));   // (slot holds >= len + 16)
            uint32_t prev = __shfl_up(x.w, 1, 64);
            if (lane == 0) prev = carry;
            carry = __shfl(x.w, 63, 64);
            const uint32_t s4 = sh ? 4 - sh : 0;
            uint32_t d[4];
            if (sh) {
                d[0] = __builtin_amdgcn_alignbyte(x.x, prev, s4);
                d[1] = __builtin_amdgcn_alignbyte(x.y, x.x, s4);
                d[2] = __builtin_amdgcn_alignbyte(x.z, x.y, s4);
                d[3] = __builtin_amdgcn_alignbyte(x.w, x.z, s4);
            } else {
                d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t w = 4 * i + k;
                const int64_t b = (int64_t)(4 * w) - (int64_t)sh;   // first tile byte of this dword
                if (b >= 0 && (uint64_t)b + 4 <= len) {
                    gst32(dst0 + 4 * w, d[k]);
                } else if (b + 4 > 0 && b < (int64_t)len) {   // a partial dword: its tile bytes only
                    for (int j = 0; j < 4; ++j) {
                        const int64_t bj = b + j;
                        if (bj >= 0 && bj < (int64_t)len) gst8(dst0 + 4 * w + j, (uint8_t)(d[k] >> (8 * j)));
                    }
                }
            }
        }
        if (t == m.n_tiles - 1 && lane == 0) gst<uint64_t>(m.out_len, m.c_off + off + len + m.d_len + m.raw_len + m.f_len);
    }
    if (m.n_tiles && blockIdx.x == gridDim.x - 1) put_tail(m, m.records[m.n_tiles]);
    if (m.copy_body) copy_share(m.out + m.a_len, m.body, m.body_len);
    if (m.copy_raw) copy_share(m.out + m.c_off + m.d_len, reinterpret_cast<const uint8_t *>(m.counts), m.raw_len);
}

}  // namespace

hipError_t launch_cbor(const KCbor &m, uint32_t blocks, hipStream_t s) {
    if (blocks < m.n_tiles || blocks == 0) return hipErrorInvalidValue;
    if (m.staged) {   // pack -> place (the scan inside pack's last workgroup)
        if (m.tpg == 0 || m.tpg > kPackMaxT || (uint64_t)m.tpg * kPackMaxG < m.n_tiles) return hipErrorInvalidValue;
        const uint32_t groups = (m.n_tiles + m.tpg - 1) / m.tpg;
        if (m.n_tiles) hipLaunchKernelGGL(k_cbor_pack, dim3(groups), dim3(kBlock), 0, s, m);
        const uint32_t pgrid = std::max<uint32_t>({1, std::min<uint32_t>((m.n_tiles + 3) / 4, 2048), blocks / 4});
        hipLaunchKernelGGL(k_cbor_place, dim3(pgrid), dim3(kBlock), 0, s, m);
        return hipGetLastError();
    }
    if (m.n_tiles) {
        hipLaunchKernelGGL(k_cbor_agg, dim3(std::min<uint32_t>((m.n_tiles + 3) / 4, 2048)), dim3(kBlock), 0, s, m);
        hipLaunchKernelGGL(k_cbor_scan, dim3(1), dim3(kScanThreads), 0, s, m);
    }
    hipLaunchKernelGGL(k_cbor, dim3(blocks), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

uint64_t cbor_stage_bytes(uint64_t n_tiles) { return n_tiles * kStageWave; }
uint32_t cbor_pack_tpg(uint64_t n_tiles) {   // tiles per k_cbor_pack workgroup: >= 4 (a tile per wave), <= 2048 groups
    const uint64_t t = std::max<uint64_t>(4, (n_tiles + kPackMaxG - 1) / kPackMaxG);
    return t <= kPackMaxT ? (uint32_t)t : 0u;   // 0: too many tiles for the staged form
}

}  // namespace rdx
