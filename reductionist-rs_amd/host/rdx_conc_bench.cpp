// Concurrent single-chunk requests from native threads (no Python, no GIL): the way the Rust server
// issues them — every Tokio / Rayon worker runs one request at a time to completion (src/app.rs:147-152,
// thread_limit = num_cpus - 1, src/app_state.rs:22).  T threads, each with its own rdx_workspace and HIP
// stream, each request = rdx_execute_device on an HBM-resident chunk + a stream synchronize (the result
// is needed before the HTTP response); chunks rotate over buffers larger than the Infinity Cache.
// Also the host path: rdx_execute from page-locked chunks (PCIe-bound).
//
//   rdx_conc_bench <config c1|c3|c2> <threads> <requests per thread> [device|host]
// prints one JSON line: requests/s, GB/s of selected bytes, us per request per thread.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rdx.h"

#define CHECK_HIP(x)                                                        \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            std::fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 2;                                                       \
        }                                                                   \
    } while (0)

struct Config {
    std::string name;
    uint32_t op, dtype, byte_order = 0;
    std::vector<uint64_t> shape;
    std::vector<rdx_slice> sel;
    std::vector<rdx_filter> filters;
    uint32_t miss_kind = 0;
    double miss_value = 0;
    uint64_t bytes;          // chunk bytes
    uint64_t alg_bytes;      // selected bytes read
};

static Config make_config(const std::string &n) {
    Config c;
    c.name = n;
    if (n == "c1") {         // BASELINE configs[0]: f32 4 MiB contiguous sum
        c.op = RDX_OP_SUM;
        c.dtype = RDX_DTYPE_FLOAT32;
        c.bytes = 4u << 20;
        c.alg_bytes = c.bytes;
    } else if (n == "c2") {  // configs[1]: f32 64 MiB, big-endian, shuffle es=4, sum
        c.op = RDX_OP_SUM;
        c.dtype = RDX_DTYPE_FLOAT32;
        c.byte_order = RDX_BYTE_ORDER_BIG;
        c.filters = {{RDX_FILTER_SHUFFLE, 0, 4}};
        c.bytes = 64u << 20;
        c.alg_bytes = c.bytes;
    } else {                 // configs[2]: f64 [128,128,128] hyperslab, missing_value -9999, min
        c.op = RDX_OP_MIN;
        c.dtype = RDX_DTYPE_FLOAT64;
        c.shape = {128, 128, 128};
        c.sel = {{8, 120, 1}, {0, 128, 2}, {16, 112, 1}};
        c.miss_kind = RDX_MISSING_VALUE;
        c.miss_value = -9999.0;
        c.bytes = 16u << 20;
        c.alg_bytes = 112ull * 64 * 96 * 8;
    }
    return c;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s c1|c2|c3 threads requests_per_thread [device|host]\n", argv[0]);
        return 1;
    }
    const Config cfg = make_config(argv[1]);
    const int T = std::max(1, std::atoi(argv[2]));
    const int R = std::max(1, std::atoi(argv[3]));
    const bool host = argc > 4 && std::string(argv[4]) == "host";
    rdx_context *ctx = nullptr;
    if (rdx_context_create(nullptr, 0, &ctx) != RDX_OK) {
        std::fprintf(stderr, "no device\n");
        return 2;
    }
    // request
    double mv = cfg.miss_value;
    rdx_request req{};
    req.abi_version = RDX_ABI_VERSION;
    req.op = cfg.op;
    req.dtype = cfg.dtype;
    req.byte_order = cfg.byte_order;
    req.ndim = (uint32_t)cfg.shape.size();
    req.shape = cfg.shape.empty() ? nullptr : cfg.shape.data();
    req.selection = cfg.sel.empty() ? nullptr : cfg.sel.data();
    req.n_filters = (uint32_t)cfg.filters.size();
    req.filters = cfg.filters.empty() ? nullptr : cfg.filters.data();
    if (cfg.miss_kind) {
        req.missing.kind = cfg.miss_kind;
        req.missing.n_values = 1;
        req.missing.values = &mv;
    }
    rdx_response_info info{};
    if (rdx_plan(&req, cfg.bytes, &info) != RDX_OK) return 3;
    // host data: random values of the dtype (min/max config: N(0,1)*100 with -9999 at 5 %)
    std::vector<uint8_t> hostdata(cfg.bytes);
    std::mt19937_64 g(0x5EED0005);
    if (cfg.dtype == RDX_DTYPE_FLOAT64) {
        std::normal_distribution<double> nd(0, 100);
        std::uniform_real_distribution<double> u(0, 1);
        for (uint64_t i = 0; i < cfg.bytes / 8; ++i) {
            double x = u(g) < 0.05 ? -9999.0 : nd(g);
            std::memcpy(hostdata.data() + 8 * i, &x, 8);
        }
    } else {
        std::uniform_real_distribution<float> u(0, 1);
        for (uint64_t i = 0; i < cfg.bytes / 4; ++i) {
            float x = u(g);
            std::memcpy(hostdata.data() + 4 * i, &x, 4);
        }
    }
    // rotating chunk buffers: > 256 MiB in total
    const int nbuf = (int)std::max<uint64_t>(4, (512ull << 20) / cfg.bytes);
    std::vector<void *> bufs(nbuf);
    for (auto &b : bufs) {
        if (host) {
            if (rdx_host_alloc(ctx, cfg.bytes, &b) != RDX_OK) return 2;
            std::memcpy(b, hostdata.data(), cfg.bytes);
        } else {
            CHECK_HIP(hipMalloc(&b, cfg.bytes));
            CHECK_HIP(hipMemcpy(b, hostdata.data(), cfg.bytes, hipMemcpyHostToDevice));
        }
    }
    std::atomic<int> errors{0}, ready{0};
    std::atomic<bool> go{false};
    std::vector<double> per_thread_us(T);
    // each thread: its workspace, stream and output buffers (set up before the clock starts), a warm-up
    // request, then R timed requests once every thread is ready
    auto worker = [&](int t) {
        rdx_workspace *ws = nullptr;
        hipStream_t s = nullptr;
        void *d_body = nullptr, *d_counts = nullptr, *d_status = nullptr;
        std::vector<uint8_t> body(std::max<uint64_t>(info.body_bytes, 16));
        std::vector<int64_t> counts(std::max<uint64_t>(info.n_counts, 1));
        bool ok = true;
        if (!host)
            ok = rdx_workspace_create(ctx, 0, &ws) == RDX_OK && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
                 hipMalloc(&d_body, 64) == hipSuccess && hipMalloc(&d_counts, 64) == hipSuccess &&
                 hipMalloc(&d_status, 64) == hipSuccess;
        auto one = [&](int i) {
            void *chunk = bufs[(i * T + t) % nbuf];
            rdx_response_info out{};
            rdx_status st;
            if (host) {
                st = rdx_execute(ctx, &req, chunk, cfg.bytes, body.data(), body.size(), counts.data(), counts.size(), &out);
            } else {
                st = rdx_execute_device(ws, &req, chunk, cfg.bytes, d_body, (int64_t *)d_counts, (uint32_t *)d_status,
                                        s, &out);
                if (st == RDX_OK && hipStreamSynchronize(s) != hipSuccess) st = RDX_E_DEVICE;
            }
            if (st != RDX_OK) ++errors;
        };
        if (!ok) ++errors;
        else for (int i = 0; i < 3; ++i) one(i);
        ++ready;
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        if (ok)
            for (int i = 0; i < R; ++i) one(i);
        per_thread_us[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
        if (!host) {
            (void)hipFree(d_body);
            (void)hipFree(d_counts);
            (void)hipFree(d_status);
            if (s) (void)hipStreamDestroy(s);
            if (ws) rdx_workspace_destroy(ws);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
    while (ready.load() < T) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    (void)t0;
    for (auto &x : th) x.join();
    // the timed region: from the start signal to the last thread's last completed request (teardown excluded)
    double el = 0;
    for (double v : per_thread_us) el = std::max(el, v * R / 1e6);
    const double reqs = (double)T * R;
    double lat = 0;
    for (double v : per_thread_us) lat += v / T;
    std::printf("{\"config\": \"%s\", \"path\": \"%s\", \"threads\": %d, \"requests\": %.0f, \"requests_per_s\": %.1f, "
                "\"us_per_request_aggregate\": %.3f, \"us_per_request_per_thread\": %.3f, \"GBs_alg\": %.1f, "
                "\"GiBs_chunk\": %.1f, \"roofline_frac\": %.4f, \"errors\": %d}\n",
                cfg.name.c_str(), host ? "rdx_execute (page-locked host chunk)" : "rdx_execute_device + synchronize",
                T, reqs, reqs / el, el / reqs * 1e6, lat, reqs * cfg.alg_bytes / el / 1e9,
                reqs * cfg.bytes / el / (1024.0 * 1024 * 1024), reqs * cfg.alg_bytes / el / 1e9 / 8000.0, errors.load());
    for (auto &b : bufs) {
        if (host) rdx_host_free(ctx, b);
        else (void)hipFree(b);
    }
    rdx_context_destroy(ctx);
    return errors ? 4 : 0;
}
