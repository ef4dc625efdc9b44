// Column-reduction access-shape probe (tuning tool, not product code): sum over axis 0 of a
// [4096, 4096] f32 matrix (64 MiB, 6 rotating copies > Infinity Cache).  A workgroup owns a strip of
// STRIP bytes of every row in its slice of rows; each lane reads 16 B; the 256 threads cover
// 256*16/STRIP rows per step; U loads in flight per lane.  Only the streaming phase (per-lane partials
// written out, no cross-workgroup fold), to find the access shape that streams at the read ceiling.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;
constexpr uint32_t kRows = 4096, kRowBytes = 4096 * 4;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int STRIP, int U>
__global__ __launch_bounds__(kB) void k_cols(const uint8_t *m, uint32_t slices, float *out) {
    constexpr int kLanesPerRow = STRIP / 16, kRowsPerStep = kB / kLanesPerRow;
    const uint32_t strip = blockIdx.x, s = blockIdx.y;
    const uint32_t c = threadIdx.x % kLanesPerRow, rr = threadIdx.x / kLanesPerRow;
    const uint32_t r_lo = s * kRows / slices, r_hi = (s + 1) * kRows / slices;
    const uint8_t *base = m + (uint64_t)strip * STRIP + c * 16;
    float acc[4] = {0, 0, 0, 0};
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
                for (int k = 0; k < 4; ++k) acc[k] += __builtin_bit_cast(float, v[u][k]);
    }
    if (acc[0] == 1.2345f) out[blockIdx.x] = acc[1] + acc[2] + acc[3];
}

int main() {
    constexpr int kCopies = 6;
    uint8_t *m[kCopies];
    for (int i = 0; i < kCopies; ++i) {
        CK(hipMalloc(&m[i], (size_t)kRows * kRowBytes));
        CK(hipMemset(m[i], 0, (size_t)kRows * kRowBytes));
    }
    float *out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
#define RUN(STRIP, U, SL)                                                                                      \
    {                                                                                                          \
        const dim3 grid(kRowBytes / STRIP, SL);                                                                \
        for (int i = 0; i < 6; ++i) hipLaunchKernelGGL((k_cols<STRIP, U>), grid, dim3(kB), 0, 0, m[i % kCopies], SL, out); \
        CK(hipEventRecord(e0));                                                                                \
        for (int i = 0; i < 30; ++i) hipLaunchKernelGGL((k_cols<STRIP, U>), grid, dim3(kB), 0, 0, m[i % kCopies], SL, out); \
        CK(hipEventRecord(e1));                                                                                \
        CK(hipEventSynchronize(e1));                                                                           \
        float ms;                                                                                              \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                  \
        printf("strip %5d U %2d slices %4d (wgs %6u): %6.2f us  %5.0f GB/s\n", STRIP, U, SL, grid.x * grid.y, \
               ms * 1e3 / 30, (double)kRows * kRowBytes / (ms / 30) / 1e6);                                   \
    }
    RUN(512, 8, 32) RUN(512, 8, 64) RUN(512, 16, 32)
    RUN(1024, 4, 16) RUN(1024, 8, 16) RUN(1024, 8, 32) RUN(1024, 8, 64) RUN(1024, 16, 32)
    RUN(2048, 4, 16) RUN(2048, 8, 16) RUN(2048, 8, 32) RUN(2048, 8, 64)
    RUN(4096, 4, 16) RUN(4096, 4, 32) RUN(4096, 8, 32) RUN(4096, 8, 64)
    RUN(16384, 2, 64) RUN(16384, 4, 64) RUN(16384, 4, 128) RUN(16384, 8, 256)
    return 0;
}
