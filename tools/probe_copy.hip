// Copy-bandwidth probe for the C5 select shape (tuning tool, not product code): a [512,256,256] i64
// chunk (256 MiB), selection [:, 64:192, :] = 512 contiguous 256 KiB runs -> 128 MiB contiguous
// output.  3 input chunks and 2 outputs rotate (working set > Infinity Cache).  Variants:
//   store policy: plain / nt;  load policy: plain / nt;  loads in flight per lane U;  WGs per CU.
// Each workgroup owns a contiguous stretch of the output.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;
constexpr uint64_t kIn = 256ull << 20, kOut = 128ull << 20;
constexpr uint64_t kRun = 256ull << 10;      // bytes per contiguous run
constexpr uint64_t kRunStride = 512ull << 10;
constexpr uint64_t kRunOff = 128ull << 10;   // 64 rows x 256 x 8 B

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4_t GV;
typedef __attribute__((address_space(1))) u32x4_t GW;

template <bool NTL>
__device__ __forceinline__ u32x4_t ld(const uint8_t *p) {
    if constexpr (NTL) return __builtin_nontemporal_load((GV *)p);
    else return *(GV *)p;
}
template <bool NTS>
__device__ __forceinline__ void st(uint8_t *p, u32x4_t v) {
    if constexpr (NTS) __builtin_nontemporal_store(v, (GW *)p);
    else *(GW *)p = v;
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(kB) void k_copy(const uint8_t *in, uint8_t *out) {
    const uint64_t nv = kOut / 16;
    const uint64_t per = ((nv + gridDim.x - 1) / gridDim.x + kB - 1) / kB * kB;
    const uint64_t g_begin = (uint64_t)blockIdx.x * per;
    const uint64_t g_end = g_begin + per < nv ? g_begin + per : nv;
    for (uint64_t g0 = g_begin + threadIdx.x; g0 < g_end; g0 += (uint64_t)kB * U) {
        u32x4_t v[U];
        uint64_t go[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint64_t g = g0 + (uint64_t)u * kB;
            if (g >= g_end) g = g0;
            go[u] = g;
            const uint64_t ob = g * 16, run = ob / kRun, w = ob - run * kRun;
            v[u] = ld<NTL>(in + run * kRunStride + kRunOff + w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (g0 + (uint64_t)u * kB < g_end) st<NTS>(out + go[u] * 16, v[u]);
    }
}

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 4; ++i) f(i);
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f(i);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *in[3], *out[2];
    for (int i = 0; i < 3; ++i) {
        CK(hipMalloc(&in[i], kIn));
        CK(hipMemset(in[i], i + 1, kIn));
    }
    for (int i = 0; i < 2; ++i) CK(hipMalloc(&out[i], kOut));
    const double bytes = 2.0 * kOut;
#define RUN(U, L, S)                                                                                        \
    {                                                                                                       \
        float ms = time_it([&](int i) { hipLaunchKernelGGL((k_copy<U, L, S>), dim3(grid), dim3(kB), 0, 0, in[i % 3], out[i % 2]); }, 30); \
        printf("wgpcu %d U %d ntload %d ntstore %d : %6.1f us  %5.0f GB/s (read+write)\n", wg, U, L, S, ms * 1e3, bytes / ms / 1e6); \
    }
    for (int wg : {1, 2, 4, 8}) {
        const uint32_t grid = cus * wg;
        RUN(4, false, false) RUN(4, true, false) RUN(4, true, true) RUN(4, false, true)
        RUN(8, true, false) RUN(8, true, true) RUN(2, true, false)
    }
    CK(hipDeviceSynchronize());
    return 0;
}
