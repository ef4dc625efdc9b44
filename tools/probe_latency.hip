// Small-launch latency probe (tuning tool, not product code): where do the ~5 us of a 4-16 MiB
// single-chunk reduction go?  Variants over one 16 MiB f64 buffer (rotating over 24 buffers so the
// data comes from HBM), grid G workgroups of 256 threads, each lane VPL x 16 B loads:
//   empty      : no loads, no hand-off
//   load       : loads + block reduce + plain partial store (no cross-workgroup hand-off)
//   hand1      : load + sc1 partial + drain + ONE agent counter, last arriver folds partials
//   hand2      : load + sc1 partial + drain + 8-way sharded counter, then the main counter (k_all today)
//   handonly   : hand1 without the loads
//   c3gather   : hand2 with C3's gather pattern ([128]^3 f64, sel [[8,120],[0,128,2],[16,112]], 16 B lanes)
// Run under rocprofv3 --kernel-trace --stats for per-kernel durations; prints event times too.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;
constexpr int kBufs = 24;
constexpr uint64_t kBytes = 16ull << 20;

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldnt(const uint8_t *p) {
    typedef const __attribute__((address_space(1))) u32x4_t GV;
    const u32x4_t v = __builtin_nontemporal_load((GV *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ double block_sum(double s) {
    __shared__ double part[kB / 64];
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    double t = 0;
    for (int k = 0; k < kB / 64; ++k) t += part[k];
    return t;
}

// MODE: 0 empty, 1 load, 2 hand1, 3 hand2, 4 handonly
template <int MODE, int VPL>
__global__ __launch_bounds__(kB) void k_probe(const uint8_t *buf, uint64_t nvec, uint64_t *partials,
                                              uint32_t *tickets, double *out) {
    double s = 0;
    if (MODE == 5) {
        uint4 v[VPL];
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            uint64_t g = ((uint64_t)blockIdx.x * VPL + u) * kB + threadIdx.x;
            if (g >= nvec) g = 0;
            const uint32_t i0 = (uint32_t)(g % 48), r = (uint32_t)(g / 48), i1 = r % 64, i2 = r / 64;
            const uint64_t e = ((uint64_t)(8 + i2) * 128 + 2 * i1) * 128 + 16 + 2 * i0;
            v[u] = ldnt(buf + e * 8);
        }
#pragma unroll
        for (int u = 0; u < VPL; ++u) s += __builtin_bit_cast(double, ((uint64_t)v[u].y << 32) | v[u].x) +
                                          __builtin_bit_cast(double, ((uint64_t)v[u].w << 32) | v[u].z);
    }
    if (MODE == 1 || MODE == 2 || MODE == 3) {
        uint4 v[VPL];
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            uint64_t g = ((uint64_t)blockIdx.x * VPL + u) * kB + threadIdx.x;
            if (g >= nvec) g = 0;
            v[u] = ldnt(buf + g * 16);
        }
#pragma unroll
        for (int u = 0; u < VPL; ++u) s += __builtin_bit_cast(double, ((uint64_t)v[u].y << 32) | v[u].x) +
                                          __builtin_bit_cast(double, ((uint64_t)v[u].w << 32) | v[u].z);
    }
    if (MODE == 0) {
        if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1.0;
        return;
    }
    const double t = block_sum(s);
    if (MODE == 1) {
        if (threadIdx.x == 0) partials[blockIdx.x] = __builtin_bit_cast(uint64_t, t);
        return;
    }
    __shared__ uint32_t s_last;
    const uint32_t nb = gridDim.x;
    if (threadIdx.x == 0) {
        __hip_atomic_store(partials + blockIdx.x, __builtin_bit_cast(uint64_t, t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bool last;
        if (MODE == 3 || MODE == 5) {
            const uint32_t sh = blockIdx.x % 8, nsh = nb < 8 ? nb : 8;
            const uint32_t members = (nb - sh + 7) / 8;
            last = false;
            const uint32_t p1 = __hip_atomic_fetch_add(tickets + (1 + sh) * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (p1 == members - 1) {
                __hip_atomic_store(tickets + (1 + sh) * 64, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1;
            }
        } else {
            last = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    double a = 0;
    for (uint32_t j = threadIdx.x; j < nb; j += kB)
        a += __builtin_bit_cast(double, __hip_atomic_load(partials + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    a = block_sum(a);
    if (threadIdx.x == 0) {
        out[0] = a;
        __hip_atomic_store(tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main() {
    uint8_t *bufs[kBufs];
    for (int i = 0; i < kBufs; ++i) {
        CK(hipMalloc(&bufs[i], kBytes));
        CK(hipMemset(bufs[i], 0, kBytes));
    }
    uint64_t *partials;
    uint32_t *tickets;
    double *out;
    CK(hipMalloc(&partials, 1 << 20));
    CK(hipMalloc(&tickets, 1 << 16));
    CK(hipMemset(tickets, 0, 1 << 16));
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[6] = {"empty", "load", "hand1", "hand2", "handonly", "c3gather"};
    // bytes read: 5.5 MB (C3's selected bytes) and 16 MiB
    for (uint64_t bytes : {(uint64_t)5505024, kBytes}) {
        const uint64_t nvec = bytes / 16;
#define RUN(M, V)                                                                                          \
    {                                                                                                      \
        const uint32_t grid = (uint32_t)((nvec + (uint64_t)V * kB - 1) / ((uint64_t)V * kB));                \
        for (int i = 0; i < 8; ++i)                                                                        \
            hipLaunchKernelGGL((k_probe<M, V>), dim3(grid), dim3(kB), 0, 0, bufs[i % kBufs], nvec, partials, tickets, out); \
        CK(hipDeviceSynchronize());                                                                        \
        const int reps = 96;                                                                               \
        CK(hipEventRecord(e0));                                                                            \
        for (int i = 0; i < reps; ++i)                                                                     \
            hipLaunchKernelGGL((k_probe<M, V>), dim3(grid), dim3(kB), 0, 0, bufs[i % kBufs], nvec, partials, tickets, out); \
        CK(hipEventRecord(e1));                                                                            \
        CK(hipEventSynchronize(e1));                                                                       \
        float ms;                                                                                          \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                              \
        printf("%-8s bytes %9llu vpl %2d grid %5u : %.2f us/launch (events, back-to-back)\n", names[M],   \
               (unsigned long long)bytes, V, grid, ms * 1e3 / reps);                                       \
    }
        if (bytes != kBytes) { RUN(5, 4) RUN(5, 1) RUN(5, 8) RUN(5, 16) }
        RUN(0, 4) RUN(1, 4) RUN(2, 4) RUN(3, 4) RUN(4, 4)
        RUN(1, 1) RUN(2, 1) RUN(3, 1) RUN(1, 8) RUN(2, 8) RUN(3, 8) RUN(1, 16) RUN(2, 16) RUN(3, 16)
    }
    return 0;
}
