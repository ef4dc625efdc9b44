// Concurrent single-chunk requests from native threads (no Python, no GIL): the way the Rust server
// issues them — one process (app_state.rs:21-37), every Tokio / Rayon worker running one request at a time
// to completion (src/app.rs:147-152, thread_limit = num_cpus - 1, src/app_state.rs:22).
//
//   rdx_conc_bench <config c1|c2|c3|c4|s1|h4f32|h4f64> <threads> <requests per thread> [path] [devices] [lanes]
//     config  s1: a 1 MiB f32 contiguous sum (a host chunk at the default coalesce_host_max_bytes)
//             h4f32 / h4f64: one 4 MiB f32 / f64 chunk, shuffled (es = sizeof T), big-endian, sum (the
//             north_star's host-inclusive 4 MiB rows)
//     path    device:   each thread its own rdx_workspace + stream, rdx_execute_device on an HBM-resident
//                       chunk + a stream synchronize (independent launches; round-2 form)
//             resident: rdx_execute_resident on an HBM-resident chunk, response into host memory; small
//                       all-axes requests coalesce into shared k_multi launches (the context's pool)
//             host:     rdx_execute from page-locked host chunks (PCIe-bound)
//             owned:    rdx_execute_owned from page-locked host chunks (the plugin's own call: the response in
//                       a pooled page-locked block, freed after each request)
//     devices comma-separated HIP ordinals of ONE context (default 0): the in-process multi-GPU server;
//             host / resident requests are placed by the pool (least outstanding bytes)
//     lanes   coalescer launches in flight per device (default: the engine's)
// Chunks rotate over buffers larger than the Infinity Cache (per device).  Prints one JSON line.
#include <dirent.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sys/resource.h>
#include <time.h>
#include <unistd.h>

#include <fstream>
#include <map>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <sstream>
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
    } else if (n == "s1") {  // a small chunk: 1 MiB f32, native order, sum
        c.op = RDX_OP_SUM;
        c.dtype = RDX_DTYPE_FLOAT32;
        c.bytes = 1u << 20;
        c.alg_bytes = c.bytes;
    } else if (n == "h4f32" || n == "h4f64") {  // 4 MiB shuffled big-endian f32 / f64 sum
        const bool f64 = n == "h4f64";
        c.op = RDX_OP_SUM;
        c.dtype = f64 ? RDX_DTYPE_FLOAT64 : RDX_DTYPE_FLOAT32;
        c.byte_order = RDX_BYTE_ORDER_BIG;
        c.filters = {{RDX_FILTER_SHUFFLE, 0, f64 ? 8u : 4u}};
        c.bytes = 4u << 20;
        c.alg_bytes = c.bytes;
    } else if (n == "c4") {  // configs[3]'s chunk: f32 4 MiB, shuffle es=4, native order, sum
        c.op = RDX_OP_SUM;
        c.dtype = RDX_DTYPE_FLOAT32;
        c.filters = {{RDX_FILTER_SHUFFLE, 0, 4}};
        c.bytes = 4u << 20;
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

// CPU time (us) of every thread of this process by thread name (/proc/self/task/*/stat utime + stime)
static std::map<std::string, double> thread_cpu() {
    std::map<std::string, double> m;
    const double tick = 1e6 / (double)sysconf(_SC_CLK_TCK);
    DIR *d = opendir("/proc/self/task");
    if (!d) return m;
    while (dirent *e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        const std::string base = std::string("/proc/self/task/") + e->d_name;
        std::ifstream fc(base + "/comm"), fs(base + "/stat");
        std::string name, stat;
        std::getline(fc, name);
        std::getline(fs, stat);
        const size_t rp = stat.rfind(')');
        if (rp == std::string::npos) continue;
        std::stringstream ss(stat.substr(rp + 2));
        std::string f;
        double ut = 0, st = 0;
        for (int k = 3; k <= 15 && ss >> f; ++k) {
            if (k == 14) ut = std::atof(f.c_str());
            if (k == 15) st = std::atof(f.c_str());
        }
        m[name] += (ut + st) * tick;
    }
    closedir(d);
    return m;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s c1|c2|c3|c4 threads requests_per_thread [device|resident|host] [devs] [lanes]\n",
                     argv[0]);
        return 1;
    }
    const Config cfg = make_config(argv[1]);
    const int T = std::max(1, std::atoi(argv[2]));
    const int R = std::max(1, std::atoi(argv[3]));
    const std::string path = argc > 4 ? argv[4] : "device";
    const bool owned = path == "owned";
    const bool host = path == "host" || owned, resident = path == "resident";
    std::vector<int> devs;
    {
        std::stringstream ss(argc > 5 ? argv[5] : "0");
        std::string tok;
        while (std::getline(ss, tok, ',')) devs.push_back(std::atoi(tok.c_str()));
    }
    const int D = (int)devs.size();
    rdx_context *ctx = nullptr;
    if (rdx_context_create(devs.data(), D, &ctx) != RDX_OK) {
        std::fprintf(stderr, "no device\n");
        return 2;
    }
    if (argc > 6) {
        rdx_context_config cc{};
        cc.coalesce = 1;
        cc.coalesce_lanes = (uint32_t)std::atoi(argv[6]);
        if (rdx_context_configure(ctx, &cc) != RDX_OK) return 2;
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
    // rotating chunk buffers: > 256 MiB in total per device (host: one shared set of page-locked chunks)
    const int nbuf = (int)std::max<uint64_t>(4, (512ull << 20) / cfg.bytes);
    std::vector<std::vector<void *>> bufs(host ? 1 : D, std::vector<void *>(nbuf));
    for (size_t d = 0; d < bufs.size(); ++d) {
        for (auto &b : bufs[d]) {
            if (host) {
                if (rdx_host_alloc(ctx, cfg.bytes, &b) != RDX_OK) return 2;
                std::memcpy(b, hostdata.data(), cfg.bytes);
            } else {
                CHECK_HIP(hipSetDevice(devs[d]));
                CHECK_HIP(hipMalloc(&b, cfg.bytes));
                CHECK_HIP(hipMemcpy(b, hostdata.data(), cfg.bytes, hipMemcpyHostToDevice));
            }
        }
    }
    // host paths: a plain page-locked H2D copy of the same bytes, one at a time with its wait (the link's
    // time for this request: the reference line the host-inclusive rows are read against)
    double copy_us = 0;
    if (host) {
        void *dst = nullptr;
        hipStream_t cs = nullptr;
        CHECK_HIP(hipSetDevice(devs[0]));
        CHECK_HIP(hipMalloc(&dst, cfg.bytes));
        CHECK_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        for (int i = 0; i < 220; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            CHECK_HIP(hipMemcpyAsync(dst, bufs[0][i % nbuf], cfg.bytes, hipMemcpyHostToDevice, cs));
            CHECK_HIP(hipStreamSynchronize(cs));
            if (i >= 20) copy_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 200;
        }
        CHECK_HIP(hipStreamDestroy(cs));
        CHECK_HIP(hipFree(dst));
    }
    std::atomic<int> errors{0}, ready{0};
    std::atomic<bool> go{false};
    std::vector<double> per_thread_us(T), per_thread_cpu(T);
    // each thread: (device path) its workspace, stream and output buffers, set up before the clock starts;
    // a warm-up request, then R timed requests once every thread is ready
    auto worker = [&](int t) {
        rdx_workspace *ws = nullptr;
        hipStream_t s = nullptr;
        void *d_body = nullptr, *d_counts = nullptr, *d_status = nullptr;
        std::vector<uint8_t> body(std::max<uint64_t>(info.body_bytes, 16));
        std::vector<int64_t> counts(std::max<uint64_t>(info.n_counts, 1));
        const int my_dev = t % D;
        bool ok = true;
        if (path == "device")
            ok = hipSetDevice(devs[my_dev]) == hipSuccess && rdx_workspace_create(ctx, devs[my_dev], &ws) == RDX_OK &&
                 hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess && hipMalloc(&d_body, 64) == hipSuccess &&
                 hipMalloc(&d_counts, 64) == hipSuccess && hipMalloc(&d_status, 64) == hipSuccess;
        auto one = [&](int i) {
            const int k = (i * T + t) % nbuf;
            rdx_response_info out{};
            rdx_status st;
            if (owned) {
                rdx_result *r = nullptr;
                st = rdx_execute_owned(ctx, &req, bufs[0][k], cfg.bytes, &r);
                if (st == RDX_OK) rdx_result_free(ctx, r);
            } else if (host) {
                st = rdx_execute(ctx, &req, bufs[0][k], cfg.bytes, body.data(), body.size(), counts.data(), counts.size(),
                                 &out);
            } else if (resident) {
                const int d = (i * T + t) % D;   // requests spread over the devices holding their chunks
                st = rdx_execute_resident(ctx, devs[d], &req, bufs[d][k], cfg.bytes, body.data(), body.size(),
                                          counts.data(), counts.size(), &out);
            } else {
                st = rdx_execute_device(ws, &req, bufs[my_dev][k], cfg.bytes, d_body, (int64_t *)d_counts,
                                        (uint32_t *)d_status, s, &out);
                if (st == RDX_OK && hipStreamSynchronize(s) != hipSuccess) st = RDX_E_DEVICE;
            }
            if (st != RDX_OK) ++errors;
        };
        if (!ok) ++errors;
        else for (int i = 0; i < 3; ++i) one(i);
        (void)pthread_setname_np(pthread_self(), "rdx-caller");
        ++ready;
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        timespec c0{}, c1{};
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
        if (ok)
            for (int i = 0; i < R; ++i) one(i);
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
        per_thread_us[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / R;
        per_thread_cpu[t] = (c1.tv_sec - c0.tv_sec) * 1e6 + (c1.tv_nsec - c0.tv_nsec) * 1e-3;
        if (path == "device") {
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
    rusage ru0{}, ru1{};
    const auto tc0 = thread_cpu();
    getrusage(RUSAGE_SELF, &ru0);
    go.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
    getrusage(RUSAGE_SELF, &ru1);
    const auto tc1 = thread_cpu();
    // per request: the callers' own CPU, and every other thread by name (the engine's dispatcher, HIP's)
    double callers = 0;
    for (double v : per_thread_cpu) callers += v;
    std::string others;
    for (auto &kv : tc1) {
        if (kv.first == "rdx-caller") continue;
        auto it = tc0.find(kv.first);
        const double dv = kv.second - (it == tc0.end() ? 0.0 : it->second);
        if (dv <= 0) continue;
        char buf[160];
        std::snprintf(buf, sizeof buf, "%s\"%s\": %.2f", others.empty() ? "" : ", ", kv.first.c_str(), dv / ((double)T * R));
        others += buf;
    }
    auto tv = [](const timeval &t) { return t.tv_sec * 1e6 + t.tv_usec; };
    // host CPU time of the whole process over the timed region (callers, dispatchers, HIP's threads)
    const double cpu_us = tv(ru1.ru_utime) - tv(ru0.ru_utime) + tv(ru1.ru_stime) - tv(ru0.ru_stime);
    // the timed region: from the start signal to the last thread's last completed request (teardown excluded)
    double el = 0;
    for (double v : per_thread_us) el = std::max(el, v * R / 1e6);
    const double reqs = (double)T * R;
    double lat = 0;
    for (double v : per_thread_us) lat += v / T;
    uint64_t creq = 0, claunch = 0, waits = 0, wsn = 0, direct = 0, hreads = 0, sleeps = 0;
    std::string per_dev;
    for (int d = 0; d < D; ++d) {
        rdx_device_stats st{};
        if (rdx_context_stats(ctx, (uint32_t)d, &st) == RDX_OK) {
            creq += st.coalesced_requests;
            claunch += st.coalesced_launches;
            waits += st.waits;
            direct += st.direct_requests;
            hreads += st.host_read_requests;
            sleeps += st.sleeps;
            wsn += st.workspaces;
            per_dev += (d ? "," : "") + std::to_string(st.requests);
        }
    }
    const char *pname = owned ? "rdx_execute_owned (page-locked host chunk)"
                        : host ? "rdx_execute (page-locked host chunk)"
                        : resident ? "rdx_execute_resident (coalesced)" : "rdx_execute_device + synchronize";
    std::printf("{\"config\": \"%s\", \"path\": \"%s\", \"devices\": %d, \"threads\": %d, \"requests\": %.0f, "
                "\"requests_per_s\": %.1f, \"us_per_request_aggregate\": %.3f, \"us_per_request_per_thread\": %.3f, "
                "\"GBs_alg\": %.1f, \"GiBs_chunk\": %.1f, \"roofline_frac\": %.4f, \"coalesced_requests\": %llu, "
                "\"coalesced_launches\": %llu, \"direct_requests\": %llu, \"workspaces\": %llu, \"waits\": %llu, "
                "\"requests_per_device\": [%s], \"cpu_us_per_request\": %.2f, \"cpu_cores_busy\": %.2f, \"errors\": %d, "
                "\"host_read_requests\": %llu, \"sleeps\": %llu, \"pinned_copy_us_one\": %.2f, "
                "\"cpu_us_per_request_callers\": %.2f, \"cpu_us_per_request_other_threads\": {%s}}\n",
                cfg.name.c_str(), pname, D, T, reqs, reqs / el, el / reqs * 1e6, lat, reqs * cfg.alg_bytes / el / 1e9,
                reqs * cfg.bytes / el / (1024.0 * 1024 * 1024), reqs * cfg.alg_bytes / el / 1e9 / (8000.0 * D),
                (unsigned long long)creq, (unsigned long long)claunch, (unsigned long long)direct,
                (unsigned long long)wsn, (unsigned long long)waits, per_dev.c_str(), cpu_us / reqs, cpu_us / (el * 1e6),
                errors.load(), (unsigned long long)hreads, (unsigned long long)sleeps, copy_us, callers / reqs,
                others.c_str());
    for (size_t d = 0; d < bufs.size(); ++d)
        for (auto &b : bufs[d]) {
            if (host) rdx_host_free(ctx, b);
            else (void)hipFree(b);
        }
    rdx_context_destroy(ctx);
    return errors ? 4 : 0;
}
