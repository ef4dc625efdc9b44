// Read-bandwidth probe, round 2 (tuning tool, not product code): traversal order x cache policy for
// the C2 shape (8 x 64 MiB shuffled chunks, 4 byte-planes each, every launch reads all 8 once).
//   blk : workgroup b of a chunk owns tiles [b*per, (b+1)*per)         (k_all_contig today)
//   il  : workgroup b of a chunk owns tiles b, b+bpc, b+2*bpc, ...      (all workgroups of a chunk
//         sweep it together)
//   flat: one interleaved sweep over all chunks' tiles (chunk-major)
// cache policy through buffer loads: aux 0 default, 2 nt, 1 sc0, 3 sc0|nt, 16 sc1, 18 sc1|nt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;
constexpr uint64_t kChunk = 64ull << 20;
constexpr uint64_t kPlane = kChunk / 4;
constexpr uint64_t kTiles = kPlane / (kB * 16);  // tiles per chunk
constexpr int kN = 8;

struct Ptrs { const uint8_t *p[kN]; };

template <int AUX>
__device__ __forceinline__ void tile_load(const uint8_t *base, uint64_t t, uint4 (&v)[4]) {
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)base >> 32));
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)base);
    const uint8_t *b = (const uint8_t *)(((uint64_t)hi << 32) | lo);
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)b, 0, 0x7fffffff, 0x00020000);
    // buffer offsets are 32-bit: chunk size 64 MiB fits
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t off = (uint32_t)(k * kPlane + t * kB * 16 + threadIdx.x * 16);
        auto w = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
        v[k] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__device__ __forceinline__ uint32_t fold(const uint4 (&v)[4]) {
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) a ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    return a;
}

// MODE 0 blk, 1 il, 2 flat
template <int MODE, int AUX, int UNR>
__global__ __launch_bounds__(kB) void k_read(Ptrs P, uint32_t bpc, uint32_t *out) {
    uint32_t acc = 0;
    if (MODE == 2) {
        const uint64_t total = kTiles * kN, stride = gridDim.x;
        for (uint64_t t = blockIdx.x; t < total; t += stride * UNR) {
            uint4 v[UNR][4];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                uint64_t tt = t + u * stride;
                if (tt >= total) tt = t;
                const uint32_t c = (uint32_t)(tt / kTiles);
                tile_load<AUX>(P.p[c], tt - (uint64_t)c * kTiles, v[u]);
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) acc ^= fold(v[u]);
        }
    } else {
        const uint32_t c = blockIdx.x / bpc, b = blockIdx.x - c * bpc;
        const uint8_t *base = P.p[c];
        if (MODE == 0) {
            const uint64_t per = (kTiles + bpc - 1) / bpc;
            const uint64_t t0 = b * per, t1 = t0 + per < kTiles ? t0 + per : kTiles;
            uint64_t t = t0;
            for (; t + UNR <= t1; t += UNR) {
                uint4 v[UNR][4];
#pragma unroll
                for (int u = 0; u < UNR; ++u) tile_load<AUX>(base, t + u, v[u]);
#pragma unroll
                for (int u = 0; u < UNR; ++u) acc ^= fold(v[u]);
            }
            for (; t < t1; ++t) {
                uint4 v[4];
                tile_load<AUX>(base, t, v);
                acc ^= fold(v);
            }
        } else {
            uint64_t t = b;
            for (; t + (UNR - 1) * bpc < kTiles; t += (uint64_t)UNR * bpc) {
                uint4 v[UNR][4];
#pragma unroll
                for (int u = 0; u < UNR; ++u) tile_load<AUX>(base, t + u * bpc, v[u]);
#pragma unroll
                for (int u = 0; u < UNR; ++u) acc ^= fold(v[u]);
            }
            for (; t < kTiles; t += bpc) {
                uint4 v[4];
                tile_load<AUX>(base, t, v);
                acc ^= fold(v);
            }
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
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
    CK(hipMalloc(&out, 1 << 24));
    const double bytes = (double)kChunk * kN;
    const int reps = 40;
    const char *mn[3] = {"blk", "il", "flat"};
#define RUN(M, A, U) { float ms = time_it([&] { hipLaunchKernelGGL((k_read<M, A, U>), dim3(grid), dim3(kB), 0, 0, P, bpc, out); }, reps); \
        printf("%-4s aux %2d unr %d bpcu %d : %6.1f us  %5.0f GB/s\n", mn[M], A, U, bpcu, ms * 1e3, bytes / ms / 1e6); }
    for (int bpcu : {1, 2, 4, 8}) {
        const uint32_t bpc = cus * bpcu / kN, grid = bpc * kN;
        RUN(0, 0, 2) RUN(0, 2, 2) RUN(1, 0, 2) RUN(1, 2, 2) RUN(2, 0, 2) RUN(2, 2, 2)
        RUN(1, 1, 2) RUN(1, 3, 2) RUN(1, 16, 2) RUN(1, 18, 2) RUN(1, 2, 1) RUN(1, 2, 4)
    }
    CK(hipDeviceSynchronize());
    return 0;
}
