// Phase profile of the device inflate (tuning tool, not product code): compiles k_inflate.hip with
// RDX_INFLATE_PROF (per-wave cycle counters and event counts), compresses a batch of shuffled f32
// chunks with the system zlib, decodes them and prints where each stream's cycles go.
//   build: hipcc -O3 --offload-arch=gfx950 -DRDX_INFLATE_PROF -I include tools/probe_inflate.hip -lz
//   run:   ./probe_inflate [kind=noise|field] [level] [streams] [format 1=gzip 2=zlib]
#define RDX_INFLATE_PROF 1
#include "../reductionist-rs_amd/csrc/k_inflate.hip"

#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

static std::vector<uint8_t> make_chunk(bool field, int seed, size_t n) {
    std::mt19937 rng(seed);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> v(n);
    const size_t side = (size_t)std::sqrt((double)n);
    for (size_t i = 0; i < n; ++i) {
        if (field) {
            const float x = (float)(i % side) / side, y = (float)(i / side) / side;
            const float f = 280.f + 20.f * std::sin(6.3f * x + seed) * std::cos(3.1f * y) + 0.05f * nd(rng);
            v[i] = std::round(f * 200.f) / 200.f;
        } else {
            v[i] = nd(rng);
        }
    }
    std::vector<uint8_t> sh(n * 4);  // byte shuffle, element size 4
    const uint8_t *b = reinterpret_cast<const uint8_t *>(v.data());
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 4; ++k) sh[k * n + i] = b[i * 4 + k];
    return sh;
}

static std::vector<uint8_t> compress(const std::vector<uint8_t> &in, int level, int format) {
    z_stream z{};
    deflateInit2(&z, level, Z_DEFLATED, format == 1 ? 31 : 15, 9, Z_DEFAULT_STRATEGY);
    std::vector<uint8_t> out(deflateBound(&z, in.size()));
    z.next_in = const_cast<uint8_t *>(in.data());
    z.avail_in = (uInt)in.size();
    z.next_out = out.data();
    z.avail_out = (uInt)out.size();
    deflate(&z, Z_FINISH);
    out.resize(z.total_out);
    deflateEnd(&z);
    return out;
}

int main(int argc, char **argv) {
    const bool field = argc > 1 && std::strcmp(argv[1], "field") == 0;
    const int level = argc > 2 ? std::atoi(argv[2]) : 1;
    const int n = argc > 3 ? std::atoi(argv[3]) : 1024;
    const int format = argc > 4 ? std::atoi(argv[4]) : 2;
    const size_t elems = 1 << 20, raw = elems * 4;
    const int distinct = 16;
    std::vector<std::vector<uint8_t>> streams;
    for (int d = 0; d < distinct; ++d) streams.push_back(compress(make_chunk(field, d, elems), level, format));
    size_t total = 0;
    std::vector<size_t> offs;
    for (auto &s : streams) {
        offs.push_back(total);
        total += (s.size() + 255) / 256 * 256;
    }
    std::vector<uint8_t> host(total);
    for (int d = 0; d < distinct; ++d) std::memcpy(host.data() + offs[d], streams[d].data(), streams[d].size());
    uint8_t *d_in, *d_out;
    CK(hipMalloc(&d_in, total));
    CK(hipMemcpy(d_in, host.data(), total, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, (size_t)n * raw));
    std::vector<const uint8_t *> ptrs(n);
    std::vector<uint64_t> lens(n);
    for (int i = 0; i < n; ++i) {
        ptrs[i] = d_in + offs[i % distinct];
        lens[i] = streams[i % distinct].size();
    }
    const uint8_t **d_ptrs;
    uint64_t *d_lens, *d_olen;
    uint32_t *d_err;
    CK(hipMalloc(&d_ptrs, n * sizeof(void *)));
    CK(hipMalloc(&d_lens, n * 8));
    CK(hipMalloc(&d_olen, n * 8));
    CK(hipMalloc(&d_err, n * 4));
    CK(hipMemcpy(d_ptrs, ptrs.data(), n * sizeof(void *), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lens, lens.data(), n * 8, hipMemcpyHostToDevice));
    unsigned long long zero[rdx::P_N] = {};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(rdx::g_prof), zero, sizeof(zero)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    CK(rdx::launch_inflate(format, d_ptrs, d_lens, n, d_out, raw, d_olen, d_err, nullptr));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint32_t> err(n);
    CK(hipMemcpy(err.data(), d_err, n * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += err[i] != 0;
    unsigned long long p[rdx::P_N];
    CK(hipMemcpyFromSymbol(p, HIP_SYMBOL(rdx::g_prof), sizeof(p)));
    double cin = 0;
    for (int i = 0; i < n; ++i) cin += lens[i];
    printf("%s level %d format %d streams %d: %.2f ms, %.2f GB/s out, ratio %.3f, errors %d\n", field ? "field" : "noise",
           level, format, n, ms, (double)n * raw / ms / 1e6, n * (double)raw / cin, bad);
    const double per = 1.0 / n;
    printf("per stream: literals %.0f matches %.0f (avg len %.2f, far %.0f) slow-decodes %.0f blocks %.1f stages %.0f flushes %.0f\n",
           p[rdx::P_LIT] * per, p[rdx::P_MATCH] * per, (double)p[rdx::P_MATCH_BYTES] / std::max(1ull, p[rdx::P_MATCH]),
           p[rdx::P_FAR] * per, p[rdx::P_SLOW] * per, p[rdx::P_BLOCKS] * per, p[rdx::P_STAGE] * per, p[rdx::P_FLUSH] * per);
    const double tot = (double)p[rdx::P_T_TOTAL];
    const double named = (double)p[rdx::P_T_COPY] + p[rdx::P_T_FLUSH] + p[rdx::P_T_TABLES] + p[rdx::P_T_STORED] +
                         p[rdx::P_T_GENERAL];
    printf("cycles per stream %.3g: far copies %.1f%%  flush %.1f%%  tables %.1f%%  stored blocks %.1f%%  general() %.1f%%  "
           "rest (hot loop) %.1f%%\n",
           tot * per, 100 * p[rdx::P_T_COPY] / tot, 100 * p[rdx::P_T_FLUSH] / tot, 100 * p[rdx::P_T_TABLES] / tot,
           100 * p[rdx::P_T_STORED] / tot, 100 * p[rdx::P_T_GENERAL] / tot, 100 * (tot - named) / tot);
    printf("cycles per far copy: %.0f; per flush: %.0f\n", (double)p[rdx::P_T_COPY] / std::max(1ull, p[rdx::P_FAR]),
           (double)p[rdx::P_T_FLUSH] / std::max(1ull, p[rdx::P_FLUSH]));
    return 0;
}
