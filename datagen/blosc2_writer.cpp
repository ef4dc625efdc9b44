// ============================================================================================
//  SYNTHETIC INPUT GENERATION (tests and bench inputs; neither product nor oracle): this repo's own
//  greedy LZ77 encoders for the two LZ codecs a blosc2 chunk may carry, so that blosc2 chunks can be
//  written without a blosc2 library (none exists in this image).
//    BloscLZ: the token format blosclz_decompress reads (FastLZ level-2 style: literal runs of 1-32
//             bytes, matches of length (ctrl >> 5) + 2 with 255-run extensions, 13-bit near distances,
//             8192 + 16-bit far distances behind the (31, 255) escape); the stream ends with literals.
//    LZ4:     the LZ4 block format with its end-of-block rules (last match starts >= 12 bytes before
//             the end, last 5 bytes literals).
//  Greedy with one candidate per 4-byte hash: compression ratio is not the point, covering the token
//  forms is.  Built by datagen/Makefile into datagen/build/libblosc2w.so.
// ============================================================================================
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

// Greedy hash-chain-free LZ77: one candidate per 4-byte hash.
struct Emit {
    std::vector<uint8_t> v;
    void b(uint8_t x) { v.push_back(x); }
};

uint32_t hash4(const uint8_t *p, uint32_t bits) {
    uint32_t x;
    std::memcpy(&x, p, 4);
    return (x * 2654435761u) >> (32 - bits);
}

// BloscLZ tokens as blosclz_dec reads them; the last >= 1 bytes are literals.
std::vector<uint8_t> blosclz_enc(const uint8_t *in, uint64_t n, uint64_t max_dist) {
    Emit e;
    std::vector<int64_t> tab(1u << 14, -1);
    uint64_t i = 0, lit0 = 0;
    auto flush_lits = [&](uint64_t end) {
        while (lit0 < end) {
            const uint64_t r = end - lit0 < 32 ? end - lit0 : 32;
            e.b((uint8_t)(r - 1));
            for (uint64_t k = 0; k < r; ++k) e.b(in[lit0 + k]);
            lit0 += r;
        }
    };
    const uint64_t limit = n > 12 ? n - 12 : 0;
    while (i < limit) {
        const uint32_t hsh = hash4(in + i, 14);
        const int64_t c = tab[hsh];
        tab[hsh] = (int64_t)i;
        uint64_t len = 0, dist = 0;
        if (c >= 0 && i - (uint64_t)c <= max_dist && i > 0) {
            dist = i - (uint64_t)c;
            while (i + len < limit && in[c + len] == in[i + len]) ++len;
        }
        if (len < 3 || (dist > 8191 && len < 5) || i == 0) {
            ++i;
            continue;
        }
        flush_lits(i);
        const uint64_t L = len - 2;   // (ctrl >> 5) for L < 7
        if (dist <= 8191) {
            const uint64_t d = dist - 1;
            if (L < 7) {
                e.b((uint8_t)((L << 5) + (d >> 8)));
            } else {
                e.b((uint8_t)((7u << 5) + (d >> 8)));
                uint64_t rest = len - 9;
                while (rest >= 255) { e.b(255); rest -= 255; }
                e.b((uint8_t)rest);
            }
            e.b((uint8_t)(d & 255));
        } else {
            const uint64_t far = dist - 8192;
            if (L < 7) {
                e.b((uint8_t)((L << 5) + 31));
            } else {
                e.b((uint8_t)((7u << 5) + 31));
                uint64_t rest = len - 9;
                while (rest >= 255) { e.b(255); rest -= 255; }
                e.b((uint8_t)rest);
            }
            e.b(255);
            e.b((uint8_t)(far >> 8));
            e.b((uint8_t)(far & 255));
        }
        i += len;
        lit0 = i;
    }
    flush_lits(n);
    return e.v;
}

std::vector<uint8_t> lz4_enc(const uint8_t *in, uint64_t n) {
    Emit e;
    std::vector<int64_t> tab(1u << 14, -1);
    uint64_t i = 0, lit0 = 0;
    auto ext = [&](uint64_t v) {
        while (v >= 255) { e.b(255); v -= 255; }
        e.b((uint8_t)v);
    };
    const uint64_t mflimit = n > 12 ? n - 12 : 0;   // last match starts before this
    while (i < mflimit) {
        const uint32_t hsh = hash4(in + i, 14);
        const int64_t c = tab[hsh];
        tab[hsh] = (int64_t)i;
        uint64_t len = 0;
        if (c >= 0 && i - (uint64_t)c <= 65535) {
            while (i + len + 5 < n && in[c + len] == in[i + len]) ++len;
        }
        if (len < 4) {
            ++i;
            continue;
        }
        const uint64_t L = i - lit0, M = len - 4, off = i - (uint64_t)c;
        e.b((uint8_t)((L < 15 ? L : 15) << 4 | (M < 15 ? M : 15)));
        if (L >= 15) ext(L - 15);
        for (uint64_t k = 0; k < L; ++k) e.b(in[lit0 + k]);
        e.b((uint8_t)(off & 255));
        e.b((uint8_t)(off >> 8));
        if (M >= 15) ext(M - 15);
        i += len;
        lit0 = i;
    }
    const uint64_t L = n - lit0;
    e.b((uint8_t)((L < 15 ? L : 15) << 4));
    if (L >= 15) ext(L - 15);
    for (uint64_t k = 0; k < L; ++k) e.b(in[lit0 + k]);
    return e.v;
}

// Snappy raw block (google/snappy format_description.txt): varint length, then literals / copies.  Uses
// every element form so a decoder sees them all: copy-1 for len 4..11 with offset < 2048, copy-2 for
// offsets < 65536, copy-4 beyond (when `far` allows); literal lengths with 0-4 extension bytes.
std::vector<uint8_t> snappy_enc(const uint8_t *in, uint64_t n, uint64_t max_dist) {
    Emit e;
    for (uint64_t v = n;;) {   // preamble
        if (v < 128) { e.b((uint8_t)v); break; }
        e.b((uint8_t)(v | 128));
        v >>= 7;
    }
    auto lits = [&](uint64_t from, uint64_t L) {
        while (L) {
            const uint64_t k = L;   // one element (the format allows up to 2^32)
            const uint64_t m = k - 1;
            if (m < 60) e.b((uint8_t)(m << 2));
            else {
                const uint32_t nb = m < (1u << 8) ? 1 : m < (1u << 16) ? 2 : m < (1u << 24) ? 3 : 4;
                e.b((uint8_t)((59 + nb) << 2));
                for (uint32_t q = 0; q < nb; ++q) e.b((uint8_t)(m >> (8 * q)));
            }
            for (uint64_t q = 0; q < k; ++q) e.b(in[from + q]);
            L -= k;
        }
    };
    std::vector<int64_t> tab(1u << 14, -1);
    uint64_t i = 0, lit0 = 0;
    while (i + 4 <= n) {
        const uint32_t hsh = hash4(in + i, 14);
        const int64_t c = tab[hsh];
        tab[hsh] = (int64_t)i;
        uint64_t len = 0;
        if (c >= 0 && i - (uint64_t)c <= max_dist)
            while (i + len < n && in[c + len] == in[i + len]) ++len;
        if (len < 4) {
            ++i;
            continue;
        }
        lits(lit0, i - lit0);
        const uint64_t off = i - (uint64_t)c;
        uint64_t left = len;
        while (left) {
            if (off < 2048 && left >= 4 && left <= 11) {
                e.b((uint8_t)(1 | (left - 4) << 2 | (off >> 8) << 5));
                e.b((uint8_t)off);
                left = 0;
            } else {
                uint64_t k = left > 64 ? 64 : left;
                if (left > 64 && left - 64 < 4) k = left - 4;   // keep the remainder a valid copy-1 length
                if (off < 65536) {
                    e.b((uint8_t)(2 | (k - 1) << 2));
                    e.b((uint8_t)off);
                    e.b((uint8_t)(off >> 8));
                } else {
                    e.b((uint8_t)(3 | (k - 1) << 2));
                    for (int q = 0; q < 4; ++q) e.b((uint8_t)(off >> (8 * q)));
                }
                left -= k;
            }
        }
        i += len;
        lit0 = i;
    }
    lits(lit0, n - lit0);
    return e.v;
}

}  // namespace

extern "C" {

// One LZ stream by this repo's encoder (codec 0 BloscLZ, 1 LZ4, 2 Snappy): returns its length, or -1 when
// it would not fit dst_cap.  max_dist bounds BloscLZ (<= 8191 + 65535) and Snappy match distances.
int64_t blosc2w_lz_compress(uint32_t codec, const uint8_t *src, uint64_t n, uint64_t max_dist, uint8_t *dst,
                                  uint64_t dst_cap) {
    std::vector<uint8_t> v = codec == 0 ? blosclz_enc(src, n, max_dist) : codec == 2 ? snappy_enc(src, n, max_dist)
                                                                                     : lz4_enc(src, n);
    if (v.size() > dst_cap) return -1;
    std::memcpy(dst, v.data(), v.size());
    return (int64_t)v.size();
}

}  // extern "C"
