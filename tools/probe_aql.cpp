// The submission floor of a small launch: hipModuleLaunchKernel against
// AQL dispatch packets written straight into a user-mode HSA queue, for the same kernels (one code object,
// tools/probe_aql_kernels.hip), on one MI355X.  One JSON line per measurement:
//   issue_us       host time per launch call, N launches back to back (the dispatcher's cost per launch)
//   rate_us        wall time per launch over the same N, launch of the first to completion of the last
//   rtt_slot_us    one launch at a time on an idle queue: launch -> the kernel's host-slot write seen by the
//                  host (spinning on page-locked memory, as the engine's coalescer polls its slots)
//   rtt_sync_us    the same with hipStreamSynchronize / an HSA completion signal wait instead of the slot
// Build: tools/build_probe_aql.sh.  Run: tools/probe_aql tools/probe_aql_kernels.co [N]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)
#define SK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_ = ""; hsa_status_string(s_, &m_); std::fprintf(stderr, "%s: %s\n", #x, m_); std::exit(1); } } while (0)

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

static void emit(const char *path, const char *what, const char *kernel, double v, int n) {
    std::printf("{\"probe\": \"aql\", \"path\": \"%s\", \"what\": \"%s\", \"kernel\": \"%s\", \"us\": %.3f, \"n\": %d}\n", path,
                what, kernel, v, n);
    std::fflush(stdout);
}

// spin until *slot == want, bounded (a lost write must not hang the probe)
static bool wait_slot(volatile uint64_t *slot, uint64_t want) {
    const auto t0 = clk::now();
    while (__atomic_load_n(slot, __ATOMIC_ACQUIRE) != want)
        if (us_since(t0) > 2e6) return false;
    return true;
}

struct Gpu {
    hsa_agent_t agent{};
    hsa_region_t kernarg{};
};

static hsa_status_t find_gpu(hsa_agent_t a, void *d) {
    hsa_device_type_t t;
    SK(hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t));
    if (t == HSA_DEVICE_TYPE_GPU) {
        static_cast<Gpu *>(d)->agent = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg(hsa_region_t r, void *d) {
    hsa_region_segment_t seg;
    SK(hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg));
    if (seg != HSA_REGION_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    SK(hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags));
    if (flags & HSA_REGION_GLOBAL_FLAG_KERNARG) {
        static_cast<Gpu *>(d)->kernarg = r;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

struct Kern {
    uint64_t object = 0;
    uint32_t kernarg_size = 0, group = 0, priv = 0;
};

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s kernels.co [N]\n", argv[0]);
        return 2;
    }
    const int N = argc > 2 ? std::atoi(argv[2]) : 2000;
    std::ifstream f(argv[1], std::ios::binary);
    std::vector<char> co((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (co.empty()) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    uint64_t *slot = nullptr;   // page-locked, device-visible
    HK(hipHostMalloc((void **)&slot, 4096, hipHostMallocCoherent));
    std::memset(slot, 0, 4096);

    // ---- HIP: the same code object through the module API ----------------------------------------------
    hipModule_t mod;
    HK(hipModuleLoadData(&mod, co.data()));
    hipFunction_t fe, fs;
    HK(hipModuleGetFunction(&fe, mod, "k_empty"));
    HK(hipModuleGetFunction(&fs, mod, "k_slot"));
    hipStream_t st;
    HK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct {
        uint64_t *p;
        uint64_t tag;
    } a{slot, 0};
    size_t asz = sizeof(a);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
    for (int i = 0; i < 50; ++i) HK(hipModuleLaunchKernel(fe, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg));
    HK(hipStreamSynchronize(st));
    {
        double issue = 0;
        const auto t0 = clk::now();
        for (int i = 0; i < N; ++i) {
            const auto ti = clk::now();
            HK(hipModuleLaunchKernel(fe, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg));
            issue += us_since(ti);
        }
        HK(hipStreamSynchronize(st));
        emit("hip", "issue_us", "k_empty", issue / N, N);
        emit("hip", "rate_us", "k_empty", us_since(t0) / N, N);
    }
    {
        double tot = 0;
        for (int i = 1; i <= N; ++i) {
            a.tag = 0x1000000ull + i;
            const auto t0 = clk::now();
            HK(hipModuleLaunchKernel(fs, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg));
            if (!wait_slot(slot, a.tag)) {
                std::fprintf(stderr, "hip slot lost at %d\n", i);
                return 1;
            }
            tot += us_since(t0);
        }
        emit("hip", "rtt_slot_us", "k_slot", tot / N, N);
        HK(hipStreamSynchronize(st));
    }
    {
        double tot = 0;
        for (int i = 0; i < N; ++i) {
            const auto t0 = clk::now();
            HK(hipModuleLaunchKernel(fe, 1, 1, 1, 64, 1, 1, 0, st, nullptr, cfg));
            HK(hipStreamSynchronize(st));
            tot += us_since(t0);
        }
        emit("hip", "rtt_sync_us", "k_empty", tot / N, N);
    }

    // ---- HSA: packets written into our own queue ----------------------------------------------------------
    SK(hsa_init());
    Gpu g;
    SK(hsa_iterate_agents(find_gpu, &g) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR);
    if (hsa_agent_iterate_regions(g.agent, find_kernarg, &g) != HSA_STATUS_INFO_BREAK) {
        std::fprintf(stderr, "no kernarg region on the GPU agent\n");
        return 1;
    }
    hsa_code_object_reader_t reader;
    SK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader));
    hsa_executable_t exe;
    SK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    SK(hsa_executable_load_agent_code_object(exe, g.agent, reader, nullptr, nullptr));
    SK(hsa_executable_freeze(exe, nullptr));
    auto kern = [&](const char *name) {
        hsa_executable_symbol_t sym;
        SK(hsa_executable_get_symbol_by_name(exe, name, &g.agent, &sym));
        Kern k;
        SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object));
        SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg_size));
        SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
        SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
        return k;
    };
    const Kern ke = kern("k_empty.kd"), ks = kern("k_slot.kd");
    hsa_queue_t *q = nullptr;
    SK(hsa_queue_create(g.agent, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    // one kernarg block per ring slot (the explicit arguments, then the hidden ones zeroed)
    const uint32_t kasz = (std::max(ke.kernarg_size, ks.kernarg_size) + 63u) / 64u * 64u;
    uint8_t *ka = nullptr;
    SK(hsa_memory_allocate(g.kernarg, (size_t)kasz * q->size, (void **)&ka));
    std::memset(ka, 0, (size_t)kasz * q->size);
    hsa_signal_t done;
    SK(hsa_signal_create(1, 0, nullptr, &done));
    auto *ring = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address);
    auto submit = [&](const Kern &k, uint64_t tag, bool signal) {
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        }
        hsa_kernel_dispatch_packet_t *p = &ring[idx % q->size];
        uint8_t *args = ka + (idx % q->size) * kasz;
        std::memcpy(args, &slot, sizeof(slot));
        std::memcpy(args + 8, &tag, sizeof(tag));
        p->workgroup_size_x = 64;
        p->workgroup_size_y = p->workgroup_size_z = 1;
        p->grid_size_x = 64;
        p->grid_size_y = p->grid_size_z = 1;
        p->private_segment_size = k.priv;
        p->group_segment_size = k.group;
        p->kernel_object = k.object;
        p->kernarg_address = args;
        p->reserved2 = 0;
        p->completion_signal = signal ? done : hsa_signal_t{0};
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                ((signal ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |   // (the signalled one waits for all before it)
                                (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n(reinterpret_cast<uint32_t *>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
    };
    auto wait_done = [&]() {
        const hsa_signal_value_t v = hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 2000000000ull,
                                                              HSA_WAIT_STATE_ACTIVE);
        if (v >= 1) {
            std::fprintf(stderr, "hsa completion signal not seen\n");
            std::exit(1);
        }
        hsa_signal_store_relaxed(done, 1);
    };
    for (int i = 0; i < 50; ++i) submit(ke, 0, i == 49);
    wait_done();
    {
        double issue = 0;
        const auto t0 = clk::now();
        for (int i = 0; i < N; ++i) {
            const auto ti = clk::now();
            submit(ke, 0, i == N - 1);
            issue += us_since(ti);
        }
        wait_done();
        emit("aql", "issue_us", "k_empty", issue / N, N);
        emit("aql", "rate_us", "k_empty", us_since(t0) / N, N);
    }
    {
        double tot = 0;
        for (int i = 1; i <= N; ++i) {
            const uint64_t tag = 0x2000000ull + i;
            const auto t0 = clk::now();
            submit(ks, tag, false);
            if (!wait_slot(slot, tag)) {
                std::fprintf(stderr, "aql slot lost at %d\n", i);
                return 1;
            }
            tot += us_since(t0);
        }
        emit("aql", "rtt_slot_us", "k_slot", tot / N, N);
    }
    {
        double tot = 0;
        for (int i = 0; i < N; ++i) {
            const auto t0 = clk::now();
            submit(ke, 0, true);
            wait_done();
            tot += us_since(t0);
        }
        emit("aql", "rtt_sync_us", "k_empty", tot / N, N);
    }
    // drain and tear down
    submit(ke, 0, true);
    wait_done();
    SK(hsa_signal_destroy(done));
    SK(hsa_queue_destroy(q));
    SK(hsa_memory_free(ka));
    SK(hsa_executable_destroy(exe));
    SK(hsa_code_object_reader_destroy(reader));
    SK(hsa_shut_down());
    HK(hipStreamDestroy(st));
    HK(hipModuleUnload(mod));
    HK(hipHostFree(slot));
    return 0;
}
