// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "Race detection /
// sanitizers"): the product planner (reductionist-rs_amd/csrc/rdx_plan.cpp: validate_request, make_plan)
// and the oracle (oracle/rdx_oracle.cpp, oracle/oracle_inflate.cpp) compiled together with
// -fsanitize=address,undefined -fno-sanitize-recover=all (tests/test_sanitize_cpu.py), driven by
//   * random requests (every dtype / op / shape / selection incl. negative strides / axes / order /
//     byte order / filters incl. odd element sizes / missing kind), planner vs oracle: same status, and
//     the same response shape and sizes when both succeed (a NaN status is data-dependent: the planner
//     must then succeed);
//   * the oracle's inflate on random bytes, truncated and bit-flipped stored / fixed-Huffman streams
//     with and without gzip / zlib framing;
//   * the oracle's blosc2 decoder (oracle/oracle_blosc2.cpp) on the golden chunks
//     (tests/golden/blosc2_chunks.json, passed as a seed file) truncated, bit-flipped and with random
//     header fields.
// Any sanitizer report aborts the process (non-zero exit).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/rdx.h"
#include "../../reductionist-rs_amd/csrc/rdx_plan.hpp"

extern "C" int oracle_execute(const rdx_request *req, const void *chunk, uint64_t len, void *body, uint64_t body_cap,
                              int64_t *counts, uint64_t counts_cap, rdx_response_info *info);
extern "C" int oracle_validate_request(const rdx_request *req);
extern "C" uint32_t oracle_decompress(uint32_t compression, const uint8_t *in, uint64_t len, uint8_t *out,
                                      uint64_t cap, uint64_t *out_len);
extern "C" uint32_t oracle_blosc2_decompress(const uint8_t *src, uint64_t len, uint8_t *out, uint64_t cap,
                                             uint64_t *out_len);
extern "C" void oracle_blosc2_sizes(const uint8_t *src, uint64_t len, uint64_t *nbytes, uint64_t *cbytes,
                                   uint64_t *blocksize);

static int failures = 0;
#define EXPECT(c, ...)                                                              \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "FAIL %s:%d: %s | ", __FILE__, __LINE__, #c);      \
            std::fprintf(stderr, __VA_ARGS__);                                      \
            std::fprintf(stderr, "\n");                                             \
            if (++failures > 20) return;                                            \
        }                                                                           \
    } while (0)

using Rng = std::mt19937_64;
static int64_t uni(Rng &g, int64_t lo, int64_t hi) { return std::uniform_int_distribution<int64_t>(lo, hi)(g); }
static double unif(Rng &g) { return std::uniform_real_distribution<double>(0, 1)(g); }

static const uint32_t kEsz[6] = {4, 8, 4, 8, 4, 8};

struct Case {
    rdx_request r{};
    std::vector<uint64_t> shape, axes;
    std::vector<rdx_slice> sel;
    std::vector<rdx_filter> filters;
    std::vector<uint8_t> missing, data;
};

static void fill_value(Rng &g, uint32_t dtype, uint8_t *p, bool nan_ok) {
    const int64_t v = uni(g, -6, 6);
    switch (dtype) {
        case RDX_DTYPE_INT32: { int32_t x = (int32_t)v; std::memcpy(p, &x, 4); break; }
        case RDX_DTYPE_INT64: { int64_t x = v; std::memcpy(p, &x, 8); break; }
        case RDX_DTYPE_UINT32: { uint32_t x = (uint32_t)(v + 6); std::memcpy(p, &x, 4); break; }
        case RDX_DTYPE_UINT64: { uint64_t x = (uint64_t)(v + 6); std::memcpy(p, &x, 8); break; }
        case RDX_DTYPE_FLOAT32: {
            float x = (float)v;
            if (nan_ok && unif(g) < 0.02) x = std::nanf("");
            if (unif(g) < 0.02) x = unif(g) < 0.5 ? INFINITY : -INFINITY;
            if (x == 0 && unif(g) < 0.5) x = -0.0f;
            std::memcpy(p, &x, 4);
            break;
        }
        default: {
            double x = (double)v;
            if (nan_ok && unif(g) < 0.02) x = std::nan("");
            if (x == 0 && unif(g) < 0.5) x = -0.0;
            std::memcpy(p, &x, 8);
        }
    }
}

static void make_case(Rng &g, Case &c) {
    rdx_request &r = c.r;
    r.abi_version = RDX_ABI_VERSION;
    r.op = (uint32_t)uni(g, 0, 4);
    r.dtype = (uint32_t)uni(g, 0, 5);
    const uint32_t es = kEsz[r.dtype];
    uint64_t n = (uint64_t)uni(g, 0, 40);
    if (unif(g) < 0.85) {
        const int nd = (int)uni(g, 1, 4);
        n = 1;
        for (int k = 0; k < nd; ++k) {
            c.shape.push_back((uint64_t)uni(g, 0, 7));
            n *= c.shape.back();
        }
        if (unif(g) < 0.1) n += (uint64_t)uni(g, 0, 5);          // data longer than the shape
        if (unif(g) < 0.05 && n) n -= 1;                          // shorter: ShapeInvalid
        r.ndim = (uint32_t)nd;
        r.shape = c.shape.data();
        if (unif(g) < 0.5) r.order = unif(g) < 0.5 ? RDX_ORDER_F : RDX_ORDER_C;
        if (unif(g) < 0.6) {
            for (int k = 0; k < nd; ++k) {
                const int64_t L = (int64_t)c.shape[k];
                int64_t st = uni(g, 1, 3) * (unif(g) < 0.7 ? 1 : -1);
                if (unif(g) < 0.03) st = 0;                       // validation error
                c.sel.push_back({uni(g, -L - 2, L + 2), uni(g, -L - 2, L + 2), st});
            }
            r.selection = c.sel.data();
        }
        const double a = unif(g);
        if (a < 0.35) {
            r.axes_kind = RDX_AXES_ONE;
            c.axes.push_back((uint64_t)uni(g, 0, nd - (unif(g) < 0.05 ? 0 : 1)));
        } else if (a < 0.7) {
            r.axes_kind = RDX_AXES_MULTI;
            for (int k = 0; k < nd; ++k)
                if (unif(g) < 0.5) c.axes.push_back((uint64_t)k);
            if (unif(g) < 0.05 && !c.axes.empty()) c.axes.push_back(c.axes.front());   // unsorted / duplicate
        }
        r.n_axes = (uint32_t)c.axes.size();
        r.axes = c.axes.empty() ? nullptr : c.axes.data();
    }
    c.data.resize(n * es);
    for (uint64_t i = 0; i < n; ++i) fill_value(g, r.dtype, c.data.data() + i * es, true);
    if (unif(g) < 0.05 && !c.data.empty()) c.data.pop_back();    // FromBytes
    if (unif(g) < 0.4) r.byte_order = unif(g) < 0.6 ? RDX_BYTE_ORDER_BIG : RDX_BYTE_ORDER_LITTLE;
    if (unif(g) < 0.3) {
        const uint32_t kinds[5] = {RDX_MISSING_VALUE, RDX_MISSING_VALUES, RDX_MISSING_VALID_MIN, RDX_MISSING_VALID_MAX,
                                   RDX_MISSING_VALID_RANGE};
        r.missing.kind = kinds[uni(g, 0, 4)];
        const uint64_t m = r.missing.kind == RDX_MISSING_VALUES ? (uint64_t)uni(g, 1, 20)
                           : r.missing.kind == RDX_MISSING_VALID_RANGE ? 2 : 1;
        c.missing.resize(m * es);
        for (uint64_t i = 0; i < m; ++i) fill_value(g, r.dtype, c.missing.data() + i * es, false);
        r.missing.n_values = m;
        r.missing.values = c.missing.data();
    }
    if (unif(g) < 0.4) {
        const uint64_t cands[7] = {1, 2, 3, 4, 8, 16, 0};
        const int nf = unif(g) < 0.3 ? 2 : 1;
        for (int k = 0; k < nf; ++k)
            c.filters.push_back({(uint32_t)(unif(g) < 0.5 ? RDX_FILTER_SHUFFLE : RDX_FILTER_SHUFFLE_SIMD), 0,
                                 unif(g) < 0.6 ? es : cands[uni(g, 0, 6)]});
        r.n_filters = (uint32_t)c.filters.size();
        r.filters = c.filters.data();
    }
    if (unif(g) < 0.1) {
        r.has_size = 1;
        r.size = unif(g) < 0.8 ? c.data.size() : (uint64_t)uni(g, 0, 64);
    }
}

static void requests(uint64_t seed, int count) {
    Rng g(seed);
    for (int i = 0; i < count; ++i) {
        Case c;
        make_case(g, c);
        const rdx_status pv = rdx::validate_request(c.r);
        const int ov = oracle_validate_request(&c.r);
        EXPECT((int)pv == ov, "case %d validate %d vs %d", i, (int)pv, ov);
        rdx::ExecPlan p;
        const rdx_status ps = pv ? pv : rdx::make_plan(c.r, c.data.size(), p);
        std::vector<uint8_t> body(8 * c.data.size() + 64);
        std::vector<int64_t> counts(c.data.size() + 8);
        rdx_response_info oi{};
        const int os = oracle_execute(&c.r, c.data.data(), c.data.size(), body.data(), body.size(), counts.data(),
                                      counts.size(), &oi);
        const int oexp = ov ? ov : os;   // the reference validates (models.rs:242-313) before operation<T>()
        if (oexp == RDX_E_NAN_UNORDERED) {
            EXPECT(ps == RDX_OK, "case %d NaN: planner %d", i, (int)ps);
            continue;
        }
        EXPECT((int)ps == oexp, "case %d op %u dtype %u: planner %d oracle %d", i, c.r.op, c.r.dtype, (int)ps, oexp);
        if (ps || oexp) continue;
        EXPECT(p.info.dtype == oi.dtype && p.info.ndim == oi.ndim && p.info.body_bytes == oi.body_bytes &&
                   p.info.n_counts == oi.n_counts,
               "case %d info", i);
        for (uint32_t k = 0; k < oi.ndim && k < RDX_MAX_NDIM; ++k) EXPECT(p.info.shape[k] == oi.shape[k], "case %d shape", i);
    }
}

// Stored-block and fixed-Huffman DEFLATE streams built by hand, then framed / truncated / bit-flipped.
static std::vector<uint8_t> deflate_stored(Rng &g, size_t n) {
    std::vector<uint8_t> s;
    size_t left = n;
    do {
        const size_t k = std::min<size_t>(left, 65535);
        left -= k;
        s.push_back(left == 0 ? 1 : 0);
        s.push_back((uint8_t)k);
        s.push_back((uint8_t)(k >> 8));
        s.push_back((uint8_t)~k);
        s.push_back((uint8_t)(~k >> 8));
        for (size_t i = 0; i < k; ++i) s.push_back((uint8_t)g());
    } while (left);
    return s;
}

static void inflate_fuzz(uint64_t seed, int count) {
    Rng g(seed);
    std::vector<uint8_t> out(1 << 20);
    for (int i = 0; i < count; ++i) {
        std::vector<uint8_t> s;
        const double kind = unif(g);
        if (kind < 0.3) {
            s.resize((size_t)uni(g, 0, 4096));
            for (auto &b : s) b = (uint8_t)g();
        } else {
            s = deflate_stored(g, (size_t)uni(g, 0, 70000));
            if (kind < 0.55) {   // fixed-Huffman block header with random payload
                s.assign((size_t)uni(g, 1, 3000), 0);
                for (auto &b : s) b = (uint8_t)g();
                s[0] = (uint8_t)((s[0] & ~7u) | 3u);   // BFINAL=1, BTYPE=01
            }
        }
        const uint32_t fmt = unif(g) < 0.5 ? RDX_COMPRESSION_GZIP : RDX_COMPRESSION_ZLIB;
        std::vector<uint8_t> f;
        if (fmt == RDX_COMPRESSION_GZIP) f = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
        else f = {0x78, 0x01};
        f.insert(f.end(), s.begin(), s.end());
        for (int k = 0; k < 8; ++k) f.push_back((uint8_t)g());   // trailer (random checksums)
        if (unif(g) < 0.3 && f.size() > 4) f.resize((size_t)uni(g, 0, (int64_t)f.size() - 1));
        const int flips = unif(g) < 0.5 ? (int)uni(g, 1, 8) : 0;
        for (int k = 0; k < flips && !f.empty(); ++k) f[(size_t)uni(g, 0, (int64_t)f.size() - 1)] ^= (uint8_t)(1u << uni(g, 0, 7));
        uint64_t got = 0;
        const uint64_t cap = unif(g) < 0.2 ? (uint64_t)uni(g, 0, 64) : out.size();
        const uint32_t e = oracle_decompress(fmt, f.data(), f.size(), out.data(), cap, &got);
        EXPECT(e <= RDX_INFLATE_OUTPUT_OVERFLOW, "inflate case %d error code %u", i, e);
    }
}

// seed file: records of {u32 length, bytes}
static void blosc2_fuzz(const char *path, uint64_t seed, int count) {
    std::vector<std::vector<uint8_t>> seeds;
    if (FILE *f = std::fopen(path, "rb")) {
        uint32_t n = 0;
        while (std::fread(&n, 4, 1, f) == 1) {
            std::vector<uint8_t> v(n);
            if (n && std::fread(v.data(), 1, n, f) != n) break;
            seeds.push_back(std::move(v));
        }
        std::fclose(f);
    }
    EXPECT(seeds.size() >= 10, "blosc2 seed file %s: %zu chunks", path, seeds.size());
    Rng g(seed);
    for (int i = 0; i < count && !seeds.empty(); ++i) {
        std::vector<uint8_t> c = seeds[(size_t)uni(g, 0, (int64_t)seeds.size() - 1)];
        const double kind = unif(g);
        if (kind < 0.3 && c.size() > 1) c.resize((size_t)uni(g, 0, (int64_t)c.size() - 1));
        const int flips = (int)uni(g, 0, 6);
        for (int k = 0; k < flips && !c.empty(); ++k) c[(size_t)uni(g, 0, (int64_t)c.size() - 1)] ^= (uint8_t)(1u << uni(g, 0, 7));
        if (kind > 0.8 && c.size() >= 32) {   // a random header field
            const int at = (int)uni(g, 0, 31);
            c[(size_t)at] = (uint8_t)g();
        }
        uint64_t nb = 0, cb = 0, bs = 0, got = 0;
        oracle_blosc2_sizes(c.data(), c.size(), &nb, &cb, &bs);
        const uint64_t cap = nb > (1u << 22) ? (1u << 22) : nb;
        std::vector<uint8_t> out(cap ? cap : 1);
        const uint32_t e = oracle_blosc2_decompress(c.data(), c.size(), out.data(), cap, &got);
        EXPECT(e == 0 || e == RDX_INFLATE_OUTPUT_OVERFLOW || (e >= RDX_BLOSC2_INVALID && e <= RDX_BLOSC2_UNSUPPORTED),
               "blosc2 case %d error code %u", i, e);
        EXPECT(e != 0 || got == nb, "blosc2 case %d: %llu bytes of %llu", i, (unsigned long long)got, (unsigned long long)nb);
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 4000;
    for (uint64_t seed = 1; seed <= 4 && failures == 0; ++seed) requests(seed * 7919, n);
    inflate_fuzz(99, n);
    if (argc > 2) blosc2_fuzz(argv[2], 1234, n);
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("sanitize: ok\n");
    return 0;
}
