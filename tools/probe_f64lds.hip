// Byte-shuffled 8-byte elements (8 byte planes per chunk): does streaming four planes at a time help?
// 8 chunks x 64 MiB HBM-resident, one launch over all of them (the bench's f64 leg), integer sums of the
// assembled elements (the arithmetic is negligible: what is measured is the access pattern).
//   direct   : every lane loads its 16-byte granule of all 8 planes per tile (k_all_contig's form), UNR tiles
//   split    : planes 0-3 of R tiles into registers, wait, then planes 4-7 of the same tiles
//   lds      : planes 0-3 of R tiles through LDS (R x 16 KiB), barrier, then planes 4-7 streamed
//   plain    : the same bytes unshuffled (the floor)
// HIP events over 20 launches after 5 warm-up ones; one JSON line per variant.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_f64lds tools/probe_f64lds.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kB = 256;
constexpr uint64_t kChunk = 64ull << 20, kPlane = kChunk / 8, kTileE = kB * 16;   // elements per tile

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld(const uint8_t *p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint64_t fold(const uint4 (&g)[8]) {
    // sum of the 16 elements the granules hold, byte k of element m = byte m of plane k's granule
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t d[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = j == 0 ? g[k].x : j == 1 ? g[k].y : j == 2 ? g[k].z : g[k].w;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint64_t v = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) v |= (uint64_t)((d[k] >> (8 * m)) & 0xFF) << (8 * k);
            s += v;
        }
    }
    return s;
}

template <int UNR>
__global__ __launch_bounds__(kB) void k_direct(const uint8_t *buf, uint32_t bpc, uint64_t *out) {
    const uint32_t c = blockIdx.x / bpc, b = blockIdx.x % bpc;
    const uint8_t *base = buf + (uint64_t)c * kChunk;
    const uint64_t per = kPlane / bpc, e0 = b * per, e1 = e0 + per;
    uint64_t s = 0;
    for (uint64_t t = e0; t < e1; t += UNR * kTileE) {
        uint4 g[UNR][8];
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) g[u][k] = ld(base + k * kPlane + t + u * kTileE + threadIdx.x * 16);
#pragma unroll
        for (int u = 0; u < UNR; ++u) s += fold(g[u]);
    }
    out[blockIdx.x * kB + threadIdx.x] = s;
}

template <int R>
__global__ __launch_bounds__(kB) void k_split(const uint8_t *buf, uint32_t bpc, uint64_t *out) {
    const uint32_t c = blockIdx.x / bpc, b = blockIdx.x % bpc;
    const uint8_t *base = buf + (uint64_t)c * kChunk;
    const uint64_t per = kPlane / bpc, e0 = b * per, e1 = e0 + per;
    uint64_t s = 0;
    for (uint64_t t = e0; t < e1; t += R * kTileE) {
        uint4 g[R][8];
#pragma unroll
        for (int u = 0; u < R; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) g[u][k] = ld(base + k * kPlane + t + u * kTileE + threadIdx.x * 16);
        __builtin_amdgcn_s_waitcnt(0);   // all of planes 0-3 landed before planes 4-7 are asked for
#pragma unroll
        for (int u = 0; u < R; ++u)
#pragma unroll
            for (int k = 4; k < 8; ++k) g[u][k] = ld(base + k * kPlane + t + u * kTileE + threadIdx.x * 16);
#pragma unroll
        for (int u = 0; u < R; ++u) s += fold(g[u]);
    }
    out[blockIdx.x * kB + threadIdx.x] = s;
}

// planes 0-3 of R tiles -> LDS (wave w of 4 streams plane w: each wave instruction reads 1 KiB of ONE
// plane), barrier, then every lane streams planes 4-7 of its granules and takes 0-3 from LDS.
template <int R>
__global__ __launch_bounds__(kB) void k_lds(const uint8_t *buf, uint32_t bpc, uint64_t *out) {
    extern __shared__ uint4 sh[];   // [4][R * kB] granules
    const uint32_t c = blockIdx.x / bpc, b = blockIdx.x % bpc;
    const uint8_t *base = buf + (uint64_t)c * kChunk;
    const uint64_t per = kPlane / bpc, e0 = b * per, e1 = e0 + per;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    uint64_t s = 0;
    for (uint64_t t = e0; t < e1; t += R * kTileE) {
        // wave w: plane w's R*kTileE bytes, 1 KiB per instruction
        uint4 a[R * 4];
#pragma unroll
        for (int i = 0; i < R * 4; ++i) a[i] = ld(base + wave * kPlane + t + (uint64_t)i * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < R * 4; ++i) sh[wave * R * kB + i * 64 + lane] = a[i];
        __syncthreads();
        uint4 g[R][8];
#pragma unroll
        for (int u = 0; u < R; ++u)
#pragma unroll
            for (int k = 4; k < 8; ++k) g[u][k] = ld(base + k * kPlane + t + u * kTileE + threadIdx.x * 16);
#pragma unroll
        for (int u = 0; u < R; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) g[u][k] = sh[k * R * kB + u * kB + threadIdx.x];
#pragma unroll
        for (int u = 0; u < R; ++u) s += fold(g[u]);
        __syncthreads();
    }
    out[blockIdx.x * kB + threadIdx.x] = s;
}

template <int UNR>
__global__ __launch_bounds__(kB) void k_plain(const uint8_t *buf, uint32_t bpc, uint64_t *out) {
    const uint32_t c = blockIdx.x / bpc, b = blockIdx.x % bpc;
    const uint8_t *base = buf + (uint64_t)c * kChunk;
    const uint64_t per = kChunk / bpc, o0 = b * per, o1 = o0 + per;
    uint64_t s = 0;
    for (uint64_t o = o0; o < o1; o += UNR * kB * 16) {
        uint4 g[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) g[u] = ld(base + o + u * kB * 16 + threadIdx.x * 16);
#pragma unroll
        for (int u = 0; u < UNR; ++u) s += ((uint64_t)g[u].y << 32 | g[u].x) + ((uint64_t)g[u].w << 32 | g[u].z);
    }
    out[blockIdx.x * kB + threadIdx.x] = s;
}

__global__ void k_fill(uint32_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u + 0x9E3779B9u;
        x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13;
        p[i] = x;
    }
}

template <class K>
static void run(const char *name, int param, K kern, uint32_t bpc, size_t lds, const uint8_t *buf, uint64_t *out) {
    const uint32_t grid = 8 * bpc;
    if (lds > 65536) CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int i = 0; i < 5; ++i) kern<<<grid, kB, lds>>>(buf, bpc, out);
    CK(hipGetLastError());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) kern<<<grid, kB, lds>>>(buf, bpc, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 20;
    printf("{\"probe\": \"f64_planes\", \"variant\": \"%s\", \"param\": %d, \"bpc\": %u, \"lds_bytes\": %zu, \"us\": %.2f, \"frac\": %.4f}\n",
           name, param, bpc, lds, us, 8.0 * kChunk / us / 1e3 / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    uint8_t *buf;
    uint64_t *out;
    CK(hipMalloc(&buf, 8 * kChunk));
    CK(hipMalloc(&out, 8ull * 64 * kB * sizeof(uint64_t)));
    k_fill<<<4096, 256>>>((uint32_t *)buf, 8 * kChunk / 4);
    CK(hipDeviceSynchronize());
    for (uint32_t bpc : {32u, 64u}) {
        run("plain", 4, k_plain<4>, bpc, 0, buf, out);
        run("direct", 1, k_direct<1>, bpc, 0, buf, out);
        run("direct", 2, k_direct<2>, bpc, 0, buf, out);
        run("split", 1, k_split<1>, bpc, 0, buf, out);
        run("split", 2, k_split<2>, bpc, 0, buf, out);
        run("lds", 1, k_lds<1>, bpc, 4 * 1 * kB * 16, buf, out);
        run("lds", 2, k_lds<2>, bpc, 4 * 2 * kB * 16, buf, out);
        run("lds", 4, k_lds<4>, bpc, 4 * 4 * kB * 16, buf, out);
        run("lds", 8, k_lds<8>, bpc, 4 * 8 * kB * 16, buf, out);
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
