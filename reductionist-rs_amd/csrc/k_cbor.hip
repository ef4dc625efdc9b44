// Response serialisation on the device (include/rdx.h rdx_cbor_encode_device): the CBOR body of
// serde_cbor::to_vec(&CBORResponse::new(&response)) (src/app.rs:33-40, src/models.rs:355-416) written
// from device-resident outputs, so a large count vector (axis reductions with many outputs, axis = [])
// is packed where it was computed and only the packed bytes cross PCIe.
//
// The host-known segments (map head, keys, dtype, shape, the array / byte-string heads: rdx_cbor.hpp)
// travel in the kernel arguments; the body and a count_as_bytes copy are device-to-device copies the
// host enqueues beside this kernel.  What needs the device is the count ARRAY: every i64 becomes a CBOR
// integer of 1, 2, 3, 5 or 9 bytes, so each count's output offset is an exclusive prefix sum of the
// encoded lengths.  One pass (read each count once, write each byte once): a workgroup takes the next
// tile of 2048 counts (tile order = start order, from a counter), scans its lengths in registers and LDS,
// finds its tile's offset by a decoupled look-back over its predecessors' records (tagged granules,
// rdx_device.hpp: {flag 2 b | value 46 b} + launch tag; flag A = tile aggregate, P = inclusive prefix),
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

__device__ void put_tail(const KCbor &m, uint64_t clen) {   // D and F after the count array
    uint8_t *d = m.out + m.c_off + clen;
    for (uint32_t i = threadIdx.x; i < m.d_len; i += kBlock) d[i] = m.tail[i];
    uint8_t *f = d + m.d_len + m.raw_len;
    for (uint32_t i = threadIdx.x; i < m.f_len; i += kBlock) f[i] = m.tail[m.d_len + i];
}

__global__ __launch_bounds__(kBlock) void k_cbor([[maybe_unused]] const KCbor args) {
    // read in place from the kernel-argument segment (the only parameter): no scratch copy of the
    // fixed byte arrays
    const KCbor &m = *(const KCbor *)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ uint8_t stage[kCborTile * 9];
    __shared__ uint32_t wsum[kBlock / 64];
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_tile, s_fault;
    if (blockIdx.x == 0) {   // A at 0, B after the body
        for (uint32_t i = threadIdx.x; i < m.a_len; i += kBlock) m.out[i] = m.fixed[i];
        for (uint32_t i = threadIdx.x; i < m.b_len; i += kBlock) m.out[m.b_off + i] = m.fixed[m.a_len + i];
    }
    if (m.n_tiles == 0) {   // no count array: D and F right after B
        if (blockIdx.x == 0) {
            put_tail(m, 0);
            if (threadIdx.x == 0) *m.out_len = m.c_off + m.d_len + m.raw_len + m.f_len;
        }
        return;
    }
    if (threadIdx.x == 0) {
        s_tile = __hip_atomic_fetch_add(m.tile_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_fault = 0;
    }
    __syncthreads();
    const uint32_t tile = s_tile;
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
    // the tile's offset in the array: decoupled look-back over the predecessors' records
    if (threadIdx.x == 0) {
        uint64_t excl = 0;
        uint32_t fault = 0;
        if (tile == 0) {
            put_granule(m.records, kFlagP | agg, m.epoch);
        } else {
            put_granule(m.records + tile, kFlagA | agg, m.epoch);
            for (uint32_t p = tile - 1;; --p) {
                uint64_t g = __hip_atomic_load(m.records + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(g >> 48) != m.epoch) {
                    g = poll_granule(m.records + p, m.epoch);
                    if ((uint32_t)(g >> 48) != m.epoch) {
                        fault = 1;
                        break;
                    }
                }
                excl += g & kVal;
                if ((g & kFlagP) || p == 0) break;
            }
            put_granule(m.records + tile, kFlagP | ((excl + agg) & kVal), m.epoch);
        }
        s_excl = excl;
        s_fault = fault;
    }
    // encode the tile into LDS at the thread's offset, then copy it out contiguously
    uint32_t o = off;
#pragma unroll
    for (int k = 0; k < kCborPer; ++k)
        if (i0 + k < m.n) o += put_int(stage + o, v[k]);
    __syncthreads();
    const uint64_t excl = s_excl;
    uint8_t *dst = m.out + m.c_off + excl;
    for (uint32_t i = threadIdx.x; i < agg; i += kBlock) dst[i] = stage[i];
    if (s_fault && threadIdx.x == 0 && m.status)
        __hip_atomic_store(m.status, (uint32_t)RDX_E_DEVICE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tile == m.n_tiles - 1) {   // every tile has taken its number: the counter can be reset
        put_tail(m, excl + agg);
        if (threadIdx.x == 0) {
            *m.out_len = m.c_off + excl + agg + m.d_len + m.raw_len + m.f_len;
            __hip_atomic_store(m.tile_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

hipError_t launch_cbor(const KCbor &m, hipStream_t s) {
    hipLaunchKernelGGL(k_cbor, dim3(m.n_tiles ? m.n_tiles : 1), dim3(kBlock), 0, s, m);
    return hipGetLastError();
}

}  // namespace rdx
