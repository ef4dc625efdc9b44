// Response serialisation on the device (include/rdx.h rdx_cbor_encode_device): the CBOR body of
// serde_cbor::to_vec(&CBORResponse::new(&response)) (src/app.rs:33-40, src/models.rs:355-416) written
// from device-resident outputs, so a large count vector (axis reductions with many outputs, axis = [])
// is packed where it was computed and only the packed bytes cross PCIe.
//
// The host-known segments (map head, keys, dtype, shape, the array / byte-string heads: rdx_cbor.hpp)
// travel in the kernel arguments; the body and a count_as_bytes payload are copied by the same launch
// (every workgroup a share, 16-byte loads, dword-aligned 16-byte stores) when the alignments allow.  What needs the device is the count ARRAY: every i64 becomes a CBOR
// integer of 1, 2, 3, 5 or 9 bytes, so each count's output offset is an exclusive prefix sum of the
// encoded lengths.  One pass (read each count once, write each byte once): workgroup w takes tiles w,
// w + grid, ... of 2048 counts (the next tile's loads in flight while the current one finishes), scans
// a tile's lengths in registers and LDS,
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

constexpr int kCborPer = 16;                      // counts per thread (eight 16-byte loads)
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

__device__ void put_tail(const KCbor &m, uint64_t clen) {   // D and F after the count array
    uint8_t *d = m.out + m.c_off + clen;
    for (uint32_t i = threadIdx.x; i < m.d_len; i += kBlock) d[i] = m.tail[i];
    uint8_t *f = d + m.d_len + m.raw_len;
    for (uint32_t i = threadIdx.x; i < m.f_len; i += kBlock) f[i] = m.tail[m.d_len + i];
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
        for (uint64_t i = units * 16 + threadIdx.x; i < n; i += kBlock) dst[i] = src[i];
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

// This thread's kCborPer counts of tile t.
__device__ __forceinline__ void load_counts(const KCbor &m, uint64_t t, int64_t (&v)[kCborPer]) {
    const uint64_t i0 = t * kCborTile + (uint64_t)threadIdx.x * kCborPer;
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

__global__ __launch_bounds__(kBlock) void k_cbor([[maybe_unused]] const KCbor args) {
    // read in place from the kernel-argument segment (the only parameter): no scratch copy of the
    // fixed byte arrays
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ uint8_t stage[kCborTile * 9];
    __shared__ uint32_t wsum[kBlock / 64];
    __shared__ uint64_t s_excl;
    struct Win {
        uint64_t sum;
        uint32_t taken;
        bool stop, hit_p;
    };
    __shared__ Win s_win[kBlock / 64];
    if (blockIdx.x == 0) {   // A at 0, B after the body
        for (uint32_t i = threadIdx.x; i < m.a_len; i += kBlock) m.out[i] = m.fixed[i];
        for (uint32_t i = threadIdx.x; i < m.b_len; i += kBlock) m.out[m.b_off + i] = m.fixed[m.a_len + i];
        if (m.n_tiles == 0) {   // no count array: D and F right after B
            put_tail(m, 0);
            if (threadIdx.x == 0) *m.out_len = m.c_off + m.d_len + m.raw_len + m.f_len;
        }
    }
    // tiles blockIdx.x, + gridDim.x, ...: the next tile's counts are loaded while this one is scanned,
    // looked back and written out
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t v[kCborPer];
    if (blockIdx.x < m.n_tiles) load_counts(m, blockIdx.x, v);
    for (uint32_t tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
        const uint64_t i0 = (uint64_t)tile * kCborTile + (uint64_t)threadIdx.x * kCborPer;
        uint32_t len = 0;
#pragma unroll
        for (int k = 0; k < kCborPer; ++k) len += i0 + k < m.n ? int_len(v[k]) : 0u;
        // block exclusive scan of the per-thread lengths
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
        // the tile's offset in the array: decoupled look-back, the workgroup reading 256 predecessors'
        // records per round trip (thread j: tile p - j; a window of W covers W / 64 steps of the walk a
        // single wave would make, and with every resident workgroup on its own tile the walk back to
        // the last inclusive prefix is what bounds the kernel); the ready aggregates (A) nearest the
        // tile are taken as they come, the nearest inclusive prefix (P) ends the walk; a predecessor
        // that has not published within kLookbackPolls polls has its aggregate computed here, so no
        // tile waits on another workgroup's progress
        if (threadIdx.x == 0) put_granule(m.records + tile, (tile == 0 ? kFlagP : kFlagA) | agg, m.epoch);
        {
            uint64_t excl = 0;
            uint32_t polls = 0;
            int64_t p = (int64_t)tile - 1;
            while (p >= 0) {   // (p, excl, polls: uniform, from LDS through readfirstlane)
                // thread j: tile p - j
                const int64_t idx = p - (int64_t)threadIdx.x;
                uint64_t g = kFlagP | ((uint64_t)m.epoch << 48);   // before tile 0: an empty inclusive prefix
                if (idx >= 0) g = __hip_atomic_load(m.records + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool ready = (uint32_t)(g >> 48) == m.epoch;
                const uint64_t late = __ballot(!ready);
                const uint64_t pmask = __ballot(ready && (g & kFlagP));
                const uint32_t k = late ? (uint32_t)__builtin_ctzll(late) : 64u;        // ready prefix
                const uint32_t first = pmask ? (uint32_t)__builtin_ctzll(pmask) : 64u;  // nearest P
                const uint32_t upto = first < k ? first + 1 : k;                        // lanes to take
                uint64_t val = lane < upto ? (g & kVal) : 0;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) val += __shfl_xor(val, d, 64);
                if (lane == 0) {
                    s_win[wave].sum = val;
                    s_win[wave].taken = upto;
                    s_win[wave].stop = first < k || k < 64;   // a P, or a late tile, inside this wave's 64
                    s_win[wave].hit_p = first < k;
                }
                __syncthreads();
                // waves in order: take each wave's part until one stops the window
                uint64_t add = 0;
                uint32_t taken = 0;
                bool done = false, stopped = false;
#pragma unroll
                for (int w = 0; w < kBlock / 64; ++w) {
                    if (stopped) break;
                    add += s_win[w].sum;
                    taken += s_win[w].taken;
                    stopped = s_win[w].stop;
                    done = s_win[w].hit_p;
                }
                __syncthreads();   // s_win is rewritten next round
                excl += add;
                // wave-uniform to the compiler too (the loop holds barriers)
                if (__builtin_amdgcn_readfirstlane((uint32_t)done)) break;
                if (__builtin_amdgcn_readfirstlane(taken) > 0) {
                    p -= taken;
                    polls = 0;
                    continue;
                }
                // tile p has not published: poll it a while, then compute its aggregate here (wave 0)
                if (++polls <= kLookbackPolls) {
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
                if (wave == 0) {
                    const uint64_t a = tile_aggregate_wave(m, (uint64_t)p, lane);
                    if (lane == 0) s_excl = a;
                }
                __syncthreads();
                excl += __builtin_amdgcn_readfirstlane((uint32_t)s_excl) | ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(s_excl >> 32)) << 32);
                __syncthreads();
                p -= 1;
                polls = 0;
            }
            if (threadIdx.x == 0) {
                if (tile) put_granule(m.records + tile, kFlagP | ((excl + agg) & kVal), m.epoch);
                s_excl = excl;
            }
        }
        // the next tile's loads go out now, under the encode and the copy
        int64_t vn[kCborPer];
        const uint32_t next = tile + gridDim.x;
        if (next < m.n_tiles) load_counts(m, next, vn);
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
        if (threadIdx.x < head) dst[threadIdx.x] = stage[threadIdx.x];
        for (uint32_t w = threadIdx.x; w < words; w += kBlock) {
            const uint32_t s0 = head + 4 * w;
            const uint32_t word = (uint32_t)stage[s0] | ((uint32_t)stage[s0 + 1] << 8) |
                                  ((uint32_t)stage[s0 + 2] << 16) | ((uint32_t)stage[s0 + 3] << 24);
            *reinterpret_cast<uint32_t *>(dst + s0) = word;
        }
        for (uint32_t i = head + 4 * words + threadIdx.x; i < agg; i += kBlock) dst[i] = stage[i];
        if (tile == m.n_tiles - 1) {
            put_tail(m, excl + agg);
            if (threadIdx.x == 0) *m.out_len = m.c_off + excl + agg + m.d_len + m.raw_len + m.f_len;
        }
        __syncthreads();   // stage, wsum and s_excl are rewritten by the next tile
#pragma unroll
        for (int k = 0; k < kCborPer; ++k) v[k] = vn[k];
    }
    // this workgroup's share of the body / count_as_bytes copies
    if (m.copy_body) copy_share(m.out + m.a_len, m.body, m.body_len);
    if (m.copy_raw) copy_share(m.out + m.c_off + m.d_len, reinterpret_cast<const uint8_t *>(m.counts), m.raw_len);
}

}  // namespace

// Workgroups of k_cbor resident per CU (its grid never exceeds what the chip holds at once: a tile's
// predecessors then belong to running workgroups).
int cbor_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_cbor, kBlock, 0) != hipSuccess || n < 1) n = 1;
    return n;
}

hipError_t launch_cbor(const KCbor &m, uint32_t blocks, hipStream_t s) {
    if (blocks == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_cbor, dim3(blocks), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

}  // namespace rdx
