// Column-reduction access-shape probe (tuning tool, not product code): sum over axis 0 of a
// [4096, 4096] f32 matrix (64 MiB, 6 rotating copies > Infinity Cache).  A workgroup owns a strip of
// STRIP bytes of every row in its slice of rows; each lane reads 16 B; the 256 threads cover
// 256*16/STRIP rows per step; U loads in flight per lane.  Only the streaming phase (per-lane partials
// written out, no cross-workgroup fold), to find the access shape that streams at the read ceiling.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <type_traits>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;
constexpr uint32_t kRows = 4096, kRowBytes = 4096 * 4;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint32_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u + seed;
        x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13;
        p[i] = 0x3F800000u | (x & 0x007FFFFFu);   // finite floats in [1, 2)
    }
}

template <int STRIP, int U, bool F64 = false>
__global__ __launch_bounds__(kB) void k_cols(const uint8_t *m, uint32_t slices, float *out) {
    constexpr int kLanesPerRow = STRIP / 16, kRowsPerStep = kB / kLanesPerRow;
    const uint32_t strip = blockIdx.x, s = blockIdx.y;
    const uint32_t c = threadIdx.x % kLanesPerRow, rr = threadIdx.x / kLanesPerRow;
    const uint32_t r_lo = s * kRows / slices, r_hi = (s + 1) * kRows / slices;
    const uint8_t *base = m + (uint64_t)strip * STRIP + c * 16;
    using Acc = std::conditional_t<F64, double, float>;
    Acc acc[4] = {0, 0, 0, 0};
    for (uint32_t r0 = r_lo + rr; r0 < r_hi; r0 += kRowsPerStep * U) {
        u32x4_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t r = r0 + u * kRowsPerStep;
            if (r >= r_hi) r = r0;
            typedef const __attribute__((address_space(1))) u32x4_t GV;
            v[u] = __builtin_nontemporal_load((GV *)(base + (uint64_t)r * kRowBytes));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (r0 + u * kRowsPerStep < r_hi)
                for (int k = 0; k < 4; ++k) acc[k] += (Acc)__builtin_bit_cast(float, v[u][k]);
    }
    if (acc[0] == (Acc)1.2345f) out[blockIdx.x] = (float)(acc[1] + acc[2] + acc[3]);
}

int main(int argc, char **argv) {
    const bool rnd = argc > 1 && !strcmp(argv[1], "random");   // random finite floats instead of zeros
    constexpr int kCopies = 6;
    uint8_t *m[kCopies];
    for (int i = 0; i < kCopies; ++i) {
        CK(hipMalloc(&m[i], (size_t)kRows * kRowBytes));
        CK(hipMemset(m[i], 0, (size_t)kRows * kRowBytes));
        if (rnd) k_fill<<<4096, 256>>>((uint32_t *)m[i], (uint64_t)kRows * kRowBytes / 4, 0x9E3779B9u * (i + 1));
    }
    float *out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    printf("data %s\n", rnd ? "random" : "zeros");
#define RUN(STRIP, U, SL, ...)                                                                                      \
    {                                                                                                          \
        const dim3 grid(kRowBytes / STRIP, SL);                                                                \
        for (int i = 0; i < 6; ++i) hipLaunchKernelGGL((k_cols<STRIP, U, ##__VA_ARGS__>), grid, dim3(kB), 0, 0, m[i % kCopies], SL, out); \
        CK(hipEventRecord(e0));                                                                                \
        for (int i = 0; i < 30; ++i) hipLaunchKernelGGL((k_cols<STRIP, U, ##__VA_ARGS__>), grid, dim3(kB), 0, 0, m[i % kCopies], SL, out); \
        CK(hipEventRecord(e1));                                                                                \
        CK(hipEventSynchronize(e1));                                                                           \
        float ms;                                                                                              \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                  \
        printf("strip %5d U %2d slices %4d %s(wgs %6u): %6.2f us  %5.0f GB/s\n", STRIP, U, SL, #__VA_ARGS__, grid.x * grid.y, \
               ms * 1e3 / 30, (double)kRows * kRowBytes / (ms / 30) / 1e6);                                   \
    }
    RUN(256, 16, 16) RUN(256, 16, 32) RUN(512, 8, 32) RUN(512, 16, 32) RUN(512, 16, 32, true) RUN(512, 16, 64)
    RUN(1024, 8, 64) RUN(1024, 16, 64) RUN(2048, 8, 64)
    return 0;
}
