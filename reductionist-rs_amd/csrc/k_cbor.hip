// Response serialisation on the device (include/rdx.h rdx_cbor_encode_device): the CBOR body of
// serde_cbor::to_vec(&CBORResponse::new(&response)) (src/app.rs:33-40, src/models.rs:355-416) written
// from device-resident outputs, so a large count vector (axis reductions with many outputs, axis = [])
// is packed where it was computed and only the packed bytes cross PCIe.
//
// The host-known segments (map head, keys, dtype, shape, the array / byte-string heads: rdx_cbor.hpp)
// travel in the kernel arguments; the body and a count_as_bytes payload are copied by the same launch
// (every workgroup a share, 16-byte loads, dword-aligned 16-byte stores) when the alignments allow.  What needs the device is the count ARRAY: every i64 becomes a CBOR
// integer of 1, 2, 3, 5 or 9 bytes, so each count's output offset is an exclusive prefix sum of the
// encoded lengths.  One pass (read each count once, write each byte once): workgroup t takes tile t of
// 2048 counts, scans its lengths in registers and LDS,
// finds its tile's offset by a decoupled look-back over its predecessors' records (tagged granules,
// rdx_device.hpp: {flag 2 b | value 46 b} + launch tag; flag A = tile aggregate, P = inclusive prefix;
// one wave reads 64 predecessors per round trip),
// encodes the tile into LDS and writes it out contiguously.  The last tile writes the trailing
// segments after the array and the total length.
//
// Roofline: HBM.  Algorithmic bytes per launch = 8 B read + 1-9 B written per count.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

constexpr int kCborPer = 8;                       // counts per thread (four 16-byte loads)
constexpr int kCborTile = kBlock * kCborPer;      // counts per tile
constexpr uint64_t kFlagA = 1ull << 46, kFlagP = 2ull << 46, kVal = (1ull << 46) - 1;

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

// Aggregate (total encoded length) of tile t computed from its counts by one wave: the look-back's
// fallback for a predecessor that has not published yet (e.g. not yet scheduled), so no tile ever
// depends on another workgroup's progress.
__device__ uint64_t tile_aggregate_wave(const KCbor &m, uint64_t t, uint32_t lane) {
    uint64_t sum = 0;
    const uint64_t e0 = t * kCborTile, e1 = e0 + kCborTile < m.n ? e0 + kCborTile : m.n;
    for (uint64_t e = e0 + lane; e < e1; e += 64) sum += int_len(gld<int64_t>(m.counts + e));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    return sum;
}

// polls of a predecessor's record before computing its aggregate instead (probe builds: none, so the
// fallback runs for every predecessor not yet published: tests run the suite on that build too)
#if RDX_PROBES
constexpr uint32_t kLookbackPolls = 0;
#else
constexpr uint32_t kLookbackPolls = 32;
#endif

__global__ __launch_bounds__(kBlock) void k_cbor([[maybe_unused]] const KCbor args) {
    // read in place from the kernel-argument segment (the only parameter): no scratch copy of the
    // fixed byte arrays
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ uint8_t stage[kCborTile * 9];
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
        const uint64_t i0 = (uint64_t)tile * kCborTile + (uint64_t)threadIdx.x * kCborPer;
        int64_t v[kCborPer];
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
        // the tile's offset in the array: decoupled look-back, one wave reading 64 predecessors' records
        // per round trip (lane j: tile p - j); the nearest inclusive prefix (P) ends the walk; a
        // predecessor that has not published within kLookbackPolls polls has its aggregate computed here
        if (wave == 0) {
            if (lane == 0) put_granule(m.records + tile, (tile == 0 ? kFlagP : kFlagA) | agg, m.epoch);
            uint64_t excl = 0;
            for (int64_t p = (int64_t)tile - 1; p >= 0; p -= 64) {
                const int64_t idx = p - (int64_t)lane;
                uint64_t g = kFlagP | ((uint64_t)m.epoch << 48);   // before tile 0: an empty inclusive prefix
                if (idx >= 0) {
                    g = __hip_atomic_load(m.records + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    for (uint32_t i = 0; (uint32_t)(g >> 48) != m.epoch && i < kLookbackPolls; ++i) {
                        __builtin_amdgcn_s_sleep(2);
                        g = __hip_atomic_load(m.records + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                const bool ready = (uint32_t)(g >> 48) == m.epoch;
                const uint64_t pmask = __ballot(ready && (g & kFlagP));
                const uint32_t first = pmask ? (uint32_t)__builtin_ctzll(pmask) : 64u;   // nearest P
                uint64_t val = ready ? (g & kVal) : 0;
                uint64_t need = __ballot(!ready && lane < first);
                while (need) {   // late predecessors: their aggregates from their counts
                    const uint32_t j = (uint32_t)__builtin_ctzll(need);
                    need &= need - 1;
                    const uint64_t a = tile_aggregate_wave(m, (uint64_t)(p - j), lane);
                    if (lane == j) val = a;
                }
                if (lane > first) val = 0;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) val += __shfl_xor(val, d, 64);
                excl += val;
                if (pmask) break;
            }
            if (lane == 0) {
                if (tile) put_granule(m.records + tile, kFlagP | ((excl + agg) & kVal), m.epoch);
                s_excl = excl;
            }
        }
        // encode the tile into LDS at the thread's offset, then copy it out contiguously (dword stores
        // between a byte head and tail)
        uint32_t o = off;
#pragma unroll
        for (int k = 0; k < kCborPer; ++k)
            if (i0 + k < m.n) o += put_int(stage + o, v[k]);
        __syncthreads();
        const uint64_t excl = s_excl;
        uint8_t *dst = m.out + m.c_off + excl;
        const uint32_t mis = (uint32_t)((4 - ((uintptr_t)dst & 3)) & 3);
        const uint32_t head = mis < agg ? mis : agg;
        const uint32_t words = (agg - head) / 4;
        if (threadIdx.x < head) gst8(dst + threadIdx.x, stage[threadIdx.x]);
        for (uint32_t w = threadIdx.x; w < words; w += kBlock) {
            const uint32_t s0 = head + 4 * w;
            const uint32_t word = (uint32_t)stage[s0] | ((uint32_t)stage[s0 + 1] << 8) |
                                  ((uint32_t)stage[s0 + 2] << 16) | ((uint32_t)stage[s0 + 3] << 24);
            gst32(dst + s0, word);
        }
        for (uint32_t i = head + 4 * words + threadIdx.x; i < agg; i += kBlock) gst8(dst + i, stage[i]);
        if (tile == m.n_tiles - 1) {
            put_tail(m, excl + agg);
            if (threadIdx.x == 0) gst<uint64_t>(m.out_len, m.c_off + excl + agg + m.d_len + m.raw_len + m.f_len);
        }
    }
    // this workgroup's share of the body / count_as_bytes copies
    if (m.copy_body) copy_share(m.out + m.a_len, m.body, m.body_len);
    if (m.copy_raw) copy_share(m.out + m.c_off + m.d_len, reinterpret_cast<const uint8_t *>(m.counts), m.raw_len);
}

}  // namespace

hipError_t launch_cbor(const KCbor &m, uint32_t blocks, hipStream_t s) {
    if (blocks < m.n_tiles || blocks == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_cbor, dim3(blocks), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

}  // namespace rdx
