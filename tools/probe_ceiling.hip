// Read-bandwidth ceiling probe for the C2 workload shape (tuning tool, not product code).
// 8 x 64 MiB buffers (512 MiB > Infinity Cache); every launch reads all 8 once.  Variants:
//   gs   : grid-stride over one flat index space, UNR x 16 B loads per lane in flight
//   blk  : contiguous per-workgroup ranges of 4-plane tiles (the k_all_contig traversal)
//   nt   : blk with non-temporal loads
// Prints GB/s per (variant, blocks per CU, UNR).  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;
constexpr uint64_t kChunk = 64ull << 20;
constexpr int kN = 8;

struct Ptrs { const uint8_t *p[kN]; };

__device__ __forceinline__ uint4 ld(const uint8_t *p, bool nt) {
    if (nt) {
        const uint4 *q = (const uint4 *)p;
        return make_uint4(__builtin_nontemporal_load(&q->x), __builtin_nontemporal_load(&q->y),
                          __builtin_nontemporal_load(&q->z), __builtin_nontemporal_load(&q->w));
    }
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) u32x4 GV;
    const u32x4 v = *(GV *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// flat grid-stride over all chunks: element index space of 16-B granules
template <int UNR>
__global__ __launch_bounds__(kB) void k_gs(Ptrs P, uint64_t granules_per_chunk, uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t total = granules_per_chunk * kN;
    const uint64_t stride = (uint64_t)gridDim.x * kB;
    for (uint64_t g = (uint64_t)blockIdx.x * kB + threadIdx.x; g < total; g += stride * UNR) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            uint64_t gg = g + u * stride;
            if (gg >= total) gg = g;
            const uint64_t c = gg / granules_per_chunk, o = gg - c * granules_per_chunk;
            v[u] = ld(P.p[c] + o * 16, false);
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// per-chunk workgroups with contiguous tile ranges; a tile = 4 planes x (256 lanes x 16 B)
template <int UNR, bool NT, bool F64>
__global__ __launch_bounds__(kB) void k_blk(Ptrs P, uint32_t bpc, uint32_t *out, double *outd) {
    const uint32_t c = blockIdx.x / bpc, b = blockIdx.x - c * bpc;
    const uint8_t *base = P.p[c];
    const uint64_t plane = kChunk / 4;
    const uint64_t tiles = plane / (kB * 16);
    const uint64_t per = (tiles + bpc - 1) / bpc;
    const uint64_t t0 = b * per, t1 = t0 + per < tiles ? t0 + per : tiles;
    uint32_t acc = 0;
    double s = 0;
    uint64_t t = t0;
    for (; t + UNR <= t1; t += UNR) {
        uint4 v[UNR][4];
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) v[u][k] = ld(base + k * plane + (t + u) * kB * 16 + threadIdx.x * 16, NT);
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (F64) s += (double)__builtin_bit_cast(float, v[u][k].x) + (double)__builtin_bit_cast(float, v[u][k].y) +
                              (double)__builtin_bit_cast(float, v[u][k].z) + (double)__builtin_bit_cast(float, v[u][k].w);
                else acc ^= v[u][k].x ^ v[u][k].y ^ v[u][k].z ^ v[u][k].w;
            }
    }
    for (; t < t1; ++t)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint4 v = ld(base + k * plane + t * kB * 16 + threadIdx.x * 16, NT);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
    if (F64 && s == 1.2345) outd[blockIdx.x] = s;
}

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    Ptrs P;
    for (int i = 0; i < kN; ++i) {
        void *p;
        CK(hipMalloc(&p, kChunk));
        CK(hipMemset(p, i + 1, kChunk));
        P.p[i] = (const uint8_t *)p;
    }
    uint32_t *out;
    double *outd;
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMalloc(&outd, 1 << 24));
    const double bytes = (double)kChunk * kN;
    const int reps = 40;
    printf("cus %d\n", cus);
    for (int bpcu : {1, 2, 4, 8}) {
        const uint32_t grid = cus * bpcu;
#define GS(U) { float ms = time_it([&] { hipLaunchKernelGGL((k_gs<U>), dim3(grid), dim3(kB), 0, 0, P, kChunk / 16, out); }, reps); \
                printf("gs  bpcu %d unr %d : %.1f us  %.0f GB/s\n", bpcu, U, ms * 1e3, bytes / ms / 1e6); }
        GS(4) GS(8) GS(16)
    }
    for (int bpcu : {1, 2, 3, 4, 8}) {
        const uint32_t bpc = cus * bpcu / kN;
        const uint32_t grid = bpc * kN;
#define BLK(U, NT, F) { float ms = time_it([&] { hipLaunchKernelGGL((k_blk<U, NT, F>), dim3(grid), dim3(kB), 0, 0, P, bpc, out, outd); }, reps); \
                printf("blk bpcu %d unr %d nt %d f64 %d : %.1f us  %.0f GB/s\n", bpcu, U, NT, F, ms * 1e3, bytes / ms / 1e6); }
        BLK(1, false, false) BLK(2, false, false) BLK(4, false, false) BLK(2, true, false) BLK(2, false, true)
    }
    // single 64 MiB chunk per launch (rotating)
    for (int bpcu : {1, 2, 4}) {
        const uint32_t bpc = cus * bpcu;
        int i = 0;
        float ms = time_it([&] {
            Ptrs Q;
            for (int k = 0; k < kN; ++k) Q.p[k] = P.p[(i + k) % kN];
            ++i;
            hipLaunchKernelGGL((k_blk<2, false, false>), dim3(bpc), dim3(kB), 0, 0, Q, bpc, out, outd);
        }, 64);
        printf("single-chunk blk bpcu %d : %.2f us  %.0f GB/s\n", bpcu, ms * 1e3, kChunk / ms / 1e6);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
