// Host-side wait and host-memory read probe (tuning tool, not product code).  Round 5: what does the
// host pay to wait for a request whose chunk is in host memory, and can the reduce kernel read a
// page-locked chunk over PCIe itself instead of a DMA copy followed by a launch?
//
// Part 1 (wait primitives): a kernel that spins for K us on the device clock and then writes a tagged
// word into page-locked host memory; the host waits for it with
//   stream_sync  hipStreamSynchronize (the engine's host path today)
//   ev_default   hipEventRecord + hipEventSynchronize, default event
//   ev_blocking  the same with hipEventBlockingSync | hipEventDisableTiming
//   slot_spin    poll the host word with pause (the direct path today)
//   slot_block   poll the host word for W us, then hipEventSynchronize on a blocking event
// Reported per method and kernel length: wall time per request over the kernel length, the waiting
// thread's CPU time (CLOCK_THREAD_CPUTIME_ID) and the whole process's (getrusage: HIP's own threads).
//
// Part 2 (host-memory reads): G workgroups of 256 lanes sum a 1 / 4 MiB f32 chunk that lives in
// page-locked host memory (hipHostMalloc default / coherent / non-coherent), 16 B loads (plain,
// non-temporal, system scope), UNR loads in flight per lane; against hipMemcpyAsync H2D of the same bytes,
// and the copy + an HBM-resident reduction.  Staleness check: the buffer is rewritten by the CPU between
// launches and the sum must follow.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <time.h>
#include <x86intrin.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <atomic>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kB = 256;

__global__ void k_spin(uint64_t ticks, uint64_t *slot, uint64_t tag) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    __hip_atomic_store(slot, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int LD>
__device__ __forceinline__ uint4 ld16(const uint4 *p) {
    if (LD == 0) return *p;
    if (LD == 1) {
        typedef const __attribute__((address_space(1))) u32x4_t GV;
        const u32x4_t v = __builtin_nontemporal_load((GV *)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n" : "=v"(v) : "v"(p) : "memory");
    return v;
}

template <int LD, int UNR>
__global__ __launch_bounds__(kB) void k_hread(const uint4 *src, uint64_t nvec, uint64_t *slot, uint64_t tag) {
    double s = 0;
    // tag = 1: each workgroup streams its own contiguous range (fewer pages touched at once per WG pair)
    uint64_t stride = (uint64_t)gridDim.x * kB * UNR, lo = (uint64_t)blockIdx.x * kB * UNR, hi = nvec;
    if (tag == 1) {
        const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
        lo = blockIdx.x * per;
        hi = lo + per < nvec ? lo + per : nvec;
        stride = (uint64_t)kB * UNR;
    }
    for (uint64_t base = lo + threadIdx.x; base < hi; base += stride) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint64_t g = base + (uint64_t)u * kB;
            v[u] = g < hi ? ld16<LD>(src + g) : make_uint4(0, 0, 0, 0);
        }
        if (LD == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            s += (double)__uint_as_float(v[u].x) + __uint_as_float(v[u].y) + __uint_as_float(v[u].z) +
                 __uint_as_float(v[u].w);
    }
    __shared__ double part[kB / 64];
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = part[0] + part[1] + part[2] + part[3];
        // integer-valued test data: the sum is exact; fixed point in the low bits of the slot
        __hip_atomic_fetch_add(slot, (uint64_t)(int64_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    }

static std::atomic<uint32_t> g_word{0};
static void host_cb(void *) {   // hipLaunchHostFunc: runs on HIP's callback thread
    g_word.store(1, std::memory_order_release);
    syscall(SYS_futex, (uint32_t *)&g_word, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double thread_cpu_us() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}
static double proc_cpu_us() {
    rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    return ru.ru_utime.tv_sec * 1e6 + ru.ru_utime.tv_usec + ru.ru_stime.tv_sec * 1e6 + ru.ru_stime.tv_usec;
}

int main(int argc, char **argv) {
    const int part = argc > 1 ? atoi(argv[1]) : 3;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint64_t *slot;
    CK(hipHostMalloc((void **)&slot, 4096, hipHostMallocCoherent));
    std::memset(slot, 0, 4096);
    hipEvent_t ev_def, ev_blk;
    CK(hipEventCreateWithFlags(&ev_def, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_blk, hipEventBlockingSync | hipEventDisableTiming));
    // device clock: 100 MHz
    if (part & 4) CK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
    if (part & 8) CK(hipSetDeviceFlags(hipDeviceScheduleYield));
    if (part & 5) {
        const char *names[] = {"stream_sync", "ev_default", "ev_blocking", "slot_spin", "slot_block20", "slot_block60", "hostfunc_futex"};
        uint64_t tag = 1;
        for (int kus : {5, 20, 50, 200, 1000}) {
            for (int m = 0; m < 7; ++m) {
                const int reps = kus >= 1000 ? 100 : 400;
                for (int warm = 0; warm < 2; ++warm) {
                    double wall = 0, tcpu = 0, pcpu = 0, worst = 0;
                    const double p0 = proc_cpu_us();
                    for (int r = 0; r < reps; ++r) {
                        ++tag;
                        const double t0 = now_us(), c0 = thread_cpu_us();
                        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, (uint64_t)kus * 100, slot, tag);
                        if (m == 0) {
                            CK(hipStreamSynchronize(s));
                        } else if (m == 1 || m == 2) {
                            CK(hipEventRecord(m == 1 ? ev_def : ev_blk, s));
                            CK(hipEventSynchronize(m == 1 ? ev_def : ev_blk));
                        } else if (m == 6) {
                            g_word.store(0, std::memory_order_relaxed);
                            CK(hipLaunchHostFunc(s, host_cb, nullptr));
                            while (g_word.load(std::memory_order_acquire) == 0)
                                syscall(SYS_futex, (uint32_t *)&g_word, FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
                        } else if (m == 3) {
                            while (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != tag) _mm_pause();
                        } else {
                            CK(hipEventRecord(ev_blk, s));
                            const double lim = m == 4 ? 20 : 60;
                            while (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != tag) {
                                if (now_us() - t0 > lim) {
                                    CK(hipEventSynchronize(ev_blk));
                                    break;
                                }
                                _mm_pause();
                            }
                        }
                        if (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != tag) { printf("slot not written\n"); return 1; }
                        const double t1 = now_us();
                        wall += t1 - t0;
                        worst = std::max(worst, t1 - t0);
                        tcpu += thread_cpu_us() - c0;
                    }
                    pcpu = proc_cpu_us() - p0;
                    CK(hipStreamSynchronize(s));
                    if (warm)
                        printf("{\"probe\": \"wait\", \"method\": \"%s\", \"kernel_us\": %d, \"wall_us\": %.2f, "
                               "\"over_kernel_us\": %.2f, \"worst_us\": %.1f, \"thread_cpu_us\": %.2f, \"proc_cpu_us\": %.2f}\n",
                               names[m], kus, wall / reps, wall / reps - kus, worst, tcpu / reps, pcpu / reps);
                }
            }
        }
    }
    if (part & 2) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const unsigned kinds[3] = {hipHostMallocDefault, hipHostMallocCoherent, hipHostMallocNonCoherent};
        const char *kname[4] = {"default", "coherent", "noncoherent", "thp_registered"};
        const char *lname[3] = {"plain", "nt", "sys"};
        for (uint64_t bytes : {1ull << 20, 4ull << 20}) {
            const uint64_t nvec = bytes / 16, n = bytes / 4;
            void *dbuf;
            CK(hipMalloc(&dbuf, bytes));
            // the DMA copy of the same bytes (pinned default)
            {
                void *h;
                CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
                for (int w = 0; w < 2; ++w) {
                    const int reps = 200;
                    CK(hipEventRecord(e0, s));
                    for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dbuf, h, bytes, hipMemcpyHostToDevice, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    // one copy + its wait, host wall clock
                    double wall = 0;
                    for (int r = 0; r < 100; ++r) {
                        const double t0 = now_us();
                        CK(hipMemcpyAsync(dbuf, h, bytes, hipMemcpyHostToDevice, s));
                        CK(hipStreamSynchronize(s));
                        wall += now_us() - t0;
                    }
                    if (w)
                        printf("{\"probe\": \"h2d_copy\", \"bytes\": %llu, \"us_back_to_back\": %.2f, \"GBs\": %.1f, "
                               "\"us_one_synchronous\": %.2f}\n", (unsigned long long)bytes, ms * 1e3 / reps,
                               bytes / (ms * 1e-3 / reps) / 1e9, wall / 100);
                }
                CK(hipHostFree(h));
            }
            for (int k = 0; k < 4; ++k) {
                float *h;
                void *thp = nullptr;
                if (k < 3) {
                    CK(hipHostMalloc((void **)&h, bytes, kinds[k]));
                } else {   // transparent huge pages, registered: 2 MiB-aligned anonymous memory
                    const size_t al = 2u << 20, sz = (bytes + al - 1) / al * al;
                    void *m = mmap(nullptr, sz + al, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                    if (m == MAP_FAILED) return 3;
                    thp = (void *)(((uintptr_t)m + al - 1) / al * al);
                    madvise(thp, sz, MADV_HUGEPAGE);
                    memset(thp, 0, sz);
                    CK(hipHostRegister(thp, sz, hipHostRegisterMapped));
                    void *dp = nullptr;
                    CK(hipHostGetDevicePointer(&dp, thp, 0));
                    h = (float *)dp;
                    if (dp != thp) printf("{\"note\": \"registered device pointer differs\"}\n");
                    // the DMA copy from it
                    void *dbuf2;
                    CK(hipMalloc(&dbuf2, bytes));
                    const int reps = 200;
                    CK(hipEventRecord(e0, s));
                    for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dbuf2, thp, bytes, hipMemcpyHostToDevice, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    double wall = 0;
                    for (int r = 0; r < 100; ++r) {
                        const double t0 = now_us();
                        CK(hipMemcpyAsync(dbuf2, thp, bytes, hipMemcpyHostToDevice, s));
                        CK(hipStreamSynchronize(s));
                        wall += now_us() - t0;
                    }
                    printf("{\"probe\": \"h2d_copy_thp\", \"bytes\": %llu, \"us_back_to_back\": %.2f, \"GBs\": %.1f, "
                           "\"us_one_synchronous\": %.2f}\n", (unsigned long long)bytes, ms * 1e3 / reps,
                           bytes / (ms * 1e-3 / reps) / 1e9, wall / 100);
                    CK(hipFree(dbuf2));
                }
#define RUNH(LD, UNR, G, LAY)                                                                                       \
    {                                                                                                          \
        bool stale = false;                                                                                    \
        for (int r = 0; r < 6 && !stale; ++r) { /* rewrite between launches: the sum must follow */           \
            for (uint64_t i = 0; i < n; ++i) h[i] = (float)((i + r) % 7);                                      \
            uint64_t want = 0;                                                                                 \
            for (uint64_t i = 0; i < n; ++i) want += (i + r) % 7;                                              \
            slot[8] = 0;                                                                                       \
            hipLaunchKernelGGL((k_hread<LD, UNR>), dim3(G), dim3(kB), 0, s, (const uint4 *)h, nvec, slot + 8, (uint64_t)LAY); \
            CK(hipStreamSynchronize(s));                                                                       \
            if (slot[8] != want) stale = true;                                                                 \
        }                                                                                                      \
        const int reps = 100;                                                                                  \
        CK(hipEventRecord(e0, s));                                                                             \
        for (int r = 0; r < reps; ++r)                                                                         \
            hipLaunchKernelGGL((k_hread<LD, UNR>), dim3(G), dim3(kB), 0, s, (const uint4 *)h, nvec, slot + 8, (uint64_t)LAY); \
        CK(hipEventRecord(e1, s));                                                                             \
        CK(hipEventSynchronize(e1));                                                                           \
        float ms;                                                                                              \
        CK(hipEventElapsedTime(&ms, e0, e1));                                                                  \
        double wall = 0;                                                                                       \
        for (int r = 0; r < 50; ++r) {                                                                         \
            const double t0 = now_us();                                                                        \
            hipLaunchKernelGGL((k_hread<LD, UNR>), dim3(G), dim3(kB), 0, s, (const uint4 *)h, nvec, slot + 8, (uint64_t)LAY); \
            CK(hipStreamSynchronize(s));                                                                       \
            wall += now_us() - t0;                                                                             \
        }                                                                                                      \
        printf("{\"probe\": \"hread\", \"mem\": \"%s\", \"load\": \"%s\", \"unr\": %d, \"grid\": %d, \"layout\": %d, \"bytes\": %llu, " \
               "\"us_back_to_back\": %.2f, \"GBs\": %.1f, \"us_one_synchronous\": %.2f, \"stale\": %s}\n",      \
               kname[k], lname[LD], UNR, G, LAY, (unsigned long long)bytes, ms * 1e3 / reps,                        \
               bytes / (ms * 1e-3 / reps) / 1e9, wall / 50, stale ? "true" : "false");                        \
    }
                if (k == 1 || k == 2) { CK(hipHostFree(h)); continue; }
                RUNH(1, 1, 4, 0) RUNH(1, 2, 4, 0) RUNH(1, 4, 4, 0) RUNH(1, 8, 4, 0)
                RUNH(1, 1, 8, 0) RUNH(1, 2, 8, 0) RUNH(1, 4, 8, 0) RUNH(1, 8, 8, 0)
                RUNH(1, 1, 16, 0) RUNH(1, 2, 16, 0) RUNH(1, 4, 16, 0) RUNH(1, 8, 16, 0)
                RUNH(1, 1, 32, 0) RUNH(1, 2, 32, 0) RUNH(1, 4, 32, 0) RUNH(1, 8, 32, 0)
                RUNH(1, 4, 8, 1) RUNH(1, 4, 16, 1) RUNH(1, 4, 32, 1) RUNH(1, 4, 64, 1) RUNH(1, 8, 16, 1)
                RUNH(0, 4, 16, 0) RUNH(0, 4, 16, 1)
                if (k < 3) CK(hipHostFree(h));
                else CK(hipHostUnregister(thp));
            }
            CK(hipFree(dbuf));
        }
    }
    return 0;
}
