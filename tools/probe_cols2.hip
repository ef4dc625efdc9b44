// Column reductions without slices (tuning probe, not product code): sum over axis 0 of a [4096, 4096] f32
// matrix (64 MiB, 6 rotating copies > Infinity Cache) where ONE workgroup owns a strip of columns over ALL
// rows, so no per-slice records are written: THREADS lanes, STRIP bytes of every row (16 B per lane), U
// loads in flight per lane, then an LDS fold of the row groups and one store per column.  XCD: adjacent
// strips share 128-byte lines when STRIP < 128; with xcd = 1 the strips of one XCD (blockIdx % 8) are a
// contiguous range, so a line's two halves are read through the same L2.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_cols2 tools/probe_cols2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t kRows = 4096, kRowBytes = 4096 * 4;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int STRIP, int U, int THREADS>
__global__ __launch_bounds__(THREADS) void k_full(const uint8_t *m, uint32_t xcd, float *out) {
    constexpr int kLanesPerRow = STRIP / 16, kGroups = THREADS / kLanesPerRow;   // row groups
    constexpr int kCols = STRIP / 4;
    __shared__ double red[kGroups][kCols + 1];
    const uint32_t nstrips = kRowBytes / STRIP;
    uint32_t strip = blockIdx.x;
    if (xcd) {   // XCD x = blockIdx % 8 takes strips [x * n / 8, (x + 1) * n / 8)
        const uint32_t x = blockIdx.x % 8, i = blockIdx.x / 8;
        strip = x * (nstrips / 8) + i;
    }
    const uint32_t c = threadIdx.x % kLanesPerRow, g = threadIdx.x / kLanesPerRow;
    const uint8_t *base = m + (uint64_t)strip * STRIP + c * 16;
    double acc[4] = {0, 0, 0, 0};
    for (uint32_t r0 = g; r0 < kRows; r0 += kGroups * U) {
        u32x4_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t r = r0 + u * kGroups;
            if (r >= kRows) r = r0;
            typedef const __attribute__((address_space(1))) u32x4_t GV;
            v[u] = __builtin_nontemporal_load((GV *)(base + (uint64_t)r * kRowBytes));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (r0 + u * kGroups < kRows)
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] += (double)__builtin_bit_cast(float, v[u][k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[g][c * 4 + k] = acc[k];
    __syncthreads();
    // fold the row groups: column j by THREADS / kCols threads, then one of them adds the partials
    constexpr int kPer = THREADS / kCols;
    const uint32_t j = threadIdx.x % kCols, part = threadIdx.x / kCols;
    double s = 0;
    for (uint32_t q = part; q < kGroups; q += kPer) s += red[q][j];
    __syncthreads();
    red[part][j] = s;
    __syncthreads();
    if (part == 0) {
        double t = 0;
        for (int q = 0; q < kPer && q < kGroups; ++q) t += red[q][j];
        out[strip * kCols + j] = (float)t;
    }
}

__global__ void k_fill(uint32_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u + seed;
        x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13;
        p[i] = 0x3F800000u | (x & 0x007FFFFFu);
    }
}

int main() {
    constexpr int kCopies = 6;
    uint8_t *m[kCopies];
    for (int i = 0; i < kCopies; ++i) {
        CK(hipMalloc(&m[i], (size_t)kRows * kRowBytes));
        k_fill<<<4096, 256>>>((uint32_t *)m[i], (uint64_t)kRows * kRowBytes / 4, 0x9E3779B9u * (i + 1));
    }
    float *out;
    CK(hipMalloc(&out, 4096 * sizeof(float)));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
#define RUN(STRIP, U, TH, XCD)                                                                                  \
    {                                                                                                           \
        const dim3 grid(kRowBytes / STRIP);                                                                     \
        for (int i = 0; i < 6; ++i) hipLaunchKernelGGL((k_full<STRIP, U, TH>), grid, dim3(TH), 0, 0, m[i % kCopies], XCD, out); \
        CK(hipGetLastError());                                                                                  \
        CK(hipEventRecord(e0));                                                                                 \
        for (int i = 0; i < 30; ++i) hipLaunchKernelGGL((k_full<STRIP, U, TH>), grid, dim3(TH), 0, 0, m[i % kCopies], XCD, out); \
        CK(hipEventRecord(e1));                                                                                 \
        CK(hipEventSynchronize(e1));                                                                            \
        float ms;                                                                                               \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                   \
        printf("{\"probe\": \"cols_full\", \"strip\": %d, \"U\": %d, \"threads\": %d, \"xcd\": %d, \"wgs\": %u, \"us\": %.2f, \"frac\": %.4f}\n", \
               STRIP, U, TH, XCD, grid.x, ms * 1e3 / 30, (double)kRows * kRowBytes / (ms / 30 * 1e-3) / 8e12);     \
        fflush(stdout);                                                                                         \
    }
    RUN(64, 8, 1024, 0) RUN(64, 8, 1024, 1) RUN(64, 16, 1024, 1) RUN(64, 8, 512, 1)
    RUN(128, 8, 1024, 0) RUN(128, 16, 1024, 0) RUN(128, 8, 512, 0) RUN(128, 4, 1024, 0)
    RUN(32, 8, 1024, 1) RUN(32, 16, 512, 1)
    RUN(256, 8, 1024, 0) RUN(256, 16, 1024, 0)
    return 0;
}
