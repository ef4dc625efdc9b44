// CPU BASELINES (test / bench infrastructure, never linked into the product): real-library decoders timed on
// the host cores for bench.py's cpu_baseline legs.
//
// blosc2 LZ4 chunks through the real liblz4 (the system's liblz4.so.1, loaded with dlopen; the reference's
// blusc 0.0.2 restates c-blosc2, whose LZ4 codec is liblz4's LZ4_decompress_safe): each chunk's block
// streams decoded by LZ4_decompress_safe, then (mode 1) the block's byte unshuffle (c-blosc2's
// blosc_internal unshuffle; scalar here), on a pool of `threads` std::threads.  Chunks as this repo's
// writer lays them out (datagen/blosc2_chunk.py): 32-byte header, bstarts[nblocks], per block `typesize`
// split streams of (int32 csize + bytes): csize = stream size -> raw copy, < 0 -> byte run, else LZ4.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

using lz4_fn = int (*)(const char *, char *, int, int);

lz4_fn load_lz4() {
    static lz4_fn fn = [] {
        void *h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
        return h ? reinterpret_cast<lz4_fn>(dlsym(h, "LZ4_decompress_safe")) : nullptr;
    }();
    return fn;
}

int32_t rd32(const uint8_t *p) {
    int32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

// one chunk -> out (nbytes); returns 0 ok, else an error
int decode_chunk(lz4_fn lz4, const uint8_t *c, uint64_t len, uint8_t *out, uint8_t *tmp, int mode, uint64_t *lz4_bytes) {
    if (len < 16) return 1;
    const uint32_t flags = c[2], ts = c[3];
    const int32_t nbytes = rd32(c + 4), bs = rd32(c + 8);
    if (nbytes <= 0 || bs <= 0 || ts == 0) return 1;
    const uint64_t overhead = (flags & 1) && (flags & 4) ? 32 : 16;   // extended header: both shuffle bits
    const bool split = !(flags & 0x10);
    const int32_t nblocks = (nbytes + bs - 1) / bs;
    for (int32_t j = 0; j < nblocks; ++j) {
        const int32_t bsize = j + 1 < nblocks ? bs : nbytes - j * bs;
        const uint32_t ns = split && bsize == bs ? ts : 1;   // the leftover block is one stream
        const int32_t ssize = bsize / (int32_t)ns;
        uint64_t pos = (uint64_t)rd32(c + overhead + 4 * j);
        uint8_t *dst = mode ? tmp : out + (uint64_t)j * bs;
        for (uint32_t k = 0; k < ns; ++k) {
            if (pos + 4 > len) return 2;
            const int32_t cs = rd32(c + pos);
            pos += 4;
            uint8_t *d = dst + (uint64_t)k * ssize;
            if (cs == 0) {
                std::memset(d, 0, ssize);
            } else if (cs < 0) {   // a run of the byte -cs, then a token byte
                std::memset(d, (uint8_t)(-cs), ssize);
                pos += 1;
            } else if (cs == ssize) {
                std::memcpy(d, c + pos, ssize);
                pos += cs;
            } else {
                const int got = lz4(reinterpret_cast<const char *>(c + pos), reinterpret_cast<char *>(d), cs, ssize);
                if (got != ssize) return 3;
                *lz4_bytes += (uint64_t)ssize;
                pos += cs;
            }
        }
        if (mode) {   // byte unshuffle of the block: out[i*ts + b] = tmp[b*n + i]
            const uint64_t n = (uint64_t)bsize / ts;
            uint8_t *o = out + (uint64_t)j * bs;
            if (ts == 4) {   // the bench's f32 chunks: four planes into words (vectorised by the compiler)
                const uint8_t *p0 = tmp, *p1 = tmp + n, *p2 = tmp + 2 * n, *p3 = tmp + 3 * n;
                uint32_t *o32 = reinterpret_cast<uint32_t *>(o);
                for (uint64_t i = 0; i < n; ++i)
                    o32[i] = (uint32_t)p0[i] | (uint32_t)p1[i] << 8 | (uint32_t)p2[i] << 16 | (uint32_t)p3[i] << 24;
            } else {
                for (uint64_t i = 0; i < n; ++i)
                    for (uint32_t b = 0; b < ts; ++b) o[i * ts + b] = tmp[b * n + i];
            }
            std::memcpy(o + n * ts, tmp + n * ts, (uint64_t)bsize - n * ts);
        }
    }
    return 0;
}

}  // namespace

extern "C" {

// 1 when liblz4.so.1 can be loaded here
int cpu_lz4lib_available(void) { return load_lz4() ? 1 : 0; }

// One chunk into out (raw_len bytes + 64 of slack): what the timed pool decodes per job, for the tests to
// check the baseline's output against the golden chunks.  Returns 0 when decoded, else an error.
int cpu_blosc2_lz4lib_one(const uint8_t *chunk, uint64_t len, uint8_t *out, uint64_t raw_len, int mode) {
    const lz4_fn lz4 = load_lz4();
    if (!lz4) return -1;
    std::vector<uint8_t> tmp(raw_len + 64);
    uint64_t bytes = 0;
    return decode_chunk(lz4, chunk, len, out, tmp.data(), mode, &bytes);
}

// Decode jobs 0..n_jobs-1 (job i = chunk i % distinct) on `threads` threads; *seconds = wall time of the
// pool (threads started before the clock), *lz4_bytes = bytes produced by LZ4_decompress_safe.
// Returns the number of chunks that failed (0 expected).
int cpu_blosc2_lz4lib(const uint8_t *const *chunks, const uint64_t *lens, uint64_t distinct, uint64_t n_jobs,
                      uint32_t threads, uint64_t raw_len, int mode, double *seconds, uint64_t *lz4_bytes) {
    const lz4_fn lz4 = load_lz4();
    if (!lz4 || !threads || !distinct) return -1;
    std::atomic<uint64_t> next{0}, bytes{0};
    std::atomic<int> bad{0}, ready{0};
    std::atomic<bool> go{false};
    auto worker = [&] {
        std::vector<uint8_t> out(raw_len + 64), tmp(raw_len + 64);
        uint64_t mine = 0;
        ++ready;
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
        for (;;) {
            const uint64_t i = next.fetch_add(1);
            if (i >= n_jobs) break;
            if (decode_chunk(lz4, chunks[i % distinct], lens[i % distinct], out.data(), tmp.data(), mode, &mine)) ++bad;
        }
        bytes += mine;
    };
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t) th.emplace_back(worker);
    while (ready.load() < (int)threads) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
    *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *lz4_bytes = bytes.load();
    return bad.load();
}

}  // extern "C"
