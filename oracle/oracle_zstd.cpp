// ============================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY: CPU restatement of zstd decompression, the ZSTD codec of the
//  reference's blosc2 branch (src/compression.rs:29-57 -> blusc 0.0.2 -> the `zstd` crate, Cargo.lock:
//  blusc -> zstd; c-blosc2's zstd_wrap_decompress = ZSTD_decompressDCtx over one stream).
//
//  Restated from the published format, RFC 8878 ("Zstandard Compression and the application/zstd Media
//  Type"): frames (magic, frame header, blocks, optional XXH64 content checksum) and skippable frames,
//  concatenated; raw / RLE / compressed blocks; the literals section (raw, RLE, Huffman-coded with one or
//  four streams, treeless = the previous table) with Huffman weights direct or FSE-coded; the sequences
//  section (predefined / RLE / FSE / repeat tables for literal lengths, offsets and match lengths, the
//  backward bitstream, repeat offsets) and sequence execution.  Pinned against the real libzstd through
//  pyarrow's bundled codec (tests/test_zstd_cpu.py: frames written by libzstd at every level decode to
//  the same bytes; corrupted frames fail where libzstd fails).  Dictionaries are not supported (a frame
//  naming a dictionary fails, as libzstd without that dictionary does).
//  Any failure: ZSTD_isError -> blosc2 "failed to decompress blosc2 data" (oracle_blosc2.cpp).
// ============================================================================================
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct ZFail {};

[[noreturn]] void bad() { throw ZFail{}; }

int hibit(uint32_t x) { return 31 - __builtin_clz(x); }   // floor(log2 x), x > 0

// ---- XXH64 (seed 0): the content checksum is its low 32 bits --------------------------------------
constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
uint64_t rd64(const uint8_t *p) { uint64_t v; std::memcpy(&v, p, 8); return v; }
uint32_t rd32u(const uint8_t *p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
uint64_t xround(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * P1 + P4; }

uint64_t xxh64(const uint8_t *p, uint64_t n) {
    const uint8_t *end = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        const uint8_t *lim = end - 32;
        do {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = P5;
    }
    h += n;
    for (; p + 8 <= end; p += 8) h = rotl(h ^ xround(0, rd64(p)), 27) * P1 + P4;
    if (p + 4 <= end) {
        h = rotl(h ^ (uint64_t)rd32u(p) * P1, 23) * P2 + P3;
        p += 4;
    }
    for (; p < end; ++p) h = rotl(h ^ (uint64_t)*p * P5, 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

// ---- bit readers ------------------------------------------------------------------------------------
// Forward little-endian reader (FSE table descriptions).
struct FwdBits {
    const uint8_t *p;
    uint64_t n, pos = 0;   // pos in bits
    uint32_t get(int k) {
        if (pos + (uint64_t)k > 8 * n) bad();
        uint32_t v = 0;
        for (int i = 0; i < k; ++i, ++pos) v |= (uint32_t)((p[pos >> 3] >> (pos & 7)) & 1u) << i;
        return v;
    }
    void rewind(int k) { pos -= (uint64_t)k; }
    uint64_t bytes_used() const { return (pos + 7) / 8; }
};

// Backward reader (RFC 8878 §4.1: read from the end, the last byte's highest set bit is padding):
// `off` is the number of bits left; reading k bits returns bits [off - k, off) (bits below 0 read as 0,
// off goes negative: an overflow the callers check).
struct BackBits {
    const uint8_t *p;
    int64_t off;
    void init(const uint8_t *src, uint64_t n) {
        if (n == 0 || src[n - 1] == 0) bad();
        p = src;
        off = (int64_t)(8 * n) - (8 - hibit(src[n - 1]));
    }
    uint64_t get(int k) {
        if (k == 0) return 0;
        off -= k;
        int64_t o = off;
        int kk = k;
        if (o < 0) {
            kk += (int)o;
            o = 0;
        }
        uint64_t v = 0;
        for (int i = 0; i < kk; ++i) v |= (uint64_t)((p[(o + i) >> 3] >> ((o + i) & 7)) & 1u) << i;
        if (off < 0) v = (-off >= 64) ? 0 : v << (-off);
        return v;
    }
};

// ---- FSE --------------------------------------------------------------------------------------------
struct FseTable {
    int log = 0;
    std::vector<uint8_t> sym, nb;
    std::vector<uint16_t> base;
    bool set = false;
};

void fse_build(FseTable &t, const int16_t *freq, int nsym, int log) {
    const uint32_t size = 1u << log;
    t.log = log;
    t.sym.assign(size, 0);
    t.nb.assign(size, 0);
    t.base.assign(size, 0);
    std::vector<uint32_t> next(256, 0);
    uint32_t high = size;
    for (int s = 0; s < nsym; ++s)
        if (freq[s] == -1) {
            t.sym[--high] = (uint8_t)s;
            next[s] = 1;
        }
    const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    uint32_t pos = 0;
    for (int s = 0; s < nsym; ++s) {
        if (freq[s] <= 0) continue;
        next[s] = (uint32_t)freq[s];
        for (int i = 0; i < freq[s]; ++i) {
            t.sym[pos] = (uint8_t)s;
            do pos = (pos + step) & mask;
            while (pos >= high);
        }
    }
    if (pos != 0) bad();
    for (uint32_t i = 0; i < size; ++i) {
        const uint32_t d = next[t.sym[i]]++;
        t.nb[i] = (uint8_t)(log - hibit(d));
        t.base[i] = (uint16_t)((d << t.nb[i]) - size);
    }
    t.set = true;
}

// FSE table description (RFC 8878 §4.1.1), read forward; returns the bytes it used.
uint64_t fse_read(FseTable &t, const uint8_t *src, uint64_t n, int max_log, int max_sym) {
    FwdBits b{src, n};
    const int log = 5 + (int)b.get(4);
    if (log > max_log) bad();
    int32_t remaining = 1 << log;
    int16_t freq[256];
    int s = 0;
    while (remaining > 0 && s <= max_sym) {
        const int bits = hibit((uint32_t)remaining + 1) + 1;
        uint32_t v = b.get(bits);
        const uint32_t lower = (1u << (bits - 1)) - 1;
        const uint32_t thr = (1u << bits) - 1 - ((uint32_t)remaining + 1);
        if ((v & lower) < thr) {
            b.rewind(1);
            v &= lower;
        } else if (v > lower) {
            v -= thr;
        }
        const int p = (int)v - 1;
        remaining -= p < 0 ? -p : p;
        freq[s++] = (int16_t)p;
        if (p == 0) {
            uint32_t rep = b.get(2);
            for (;;) {
                for (uint32_t i = 0; i < rep; ++i) {
                    if (s > max_sym) bad();
                    freq[s++] = 0;
                }
                if (rep != 3) break;
                rep = b.get(2);
            }
        }
    }
    if (remaining != 0 || s > max_sym + 1) bad();
    fse_build(t, freq, s, log);
    return b.bytes_used();
}

void fse_rle(FseTable &t, uint8_t symbol) {
    t.log = 0;
    t.sym.assign(1, symbol);
    t.nb.assign(1, 0);
    t.base.assign(1, 0);
    t.set = true;
}

// ---- Huffman (literals) -------------------------------------------------------------------------------
struct HufTable {
    int maxbits = 0;
    std::vector<uint8_t> sym, nb;   // 1 << maxbits entries
    bool set = false;
};

// Weights (direct 4-bit or FSE-coded, RFC 8878 §4.2.1); returns the bytes the description used.
uint64_t huf_read(HufTable &h, const uint8_t *src, uint64_t n) {
    if (n < 1) bad();
    const uint8_t hdr = src[0];
    uint8_t w[256];
    std::memset(w, 0, sizeof w);
    int nw = 0;
    uint64_t used;
    if (hdr >= 128) {
        nw = hdr - 127;
        const uint64_t bytes = (uint64_t)(nw + 1) / 2;
        if (1 + bytes > n) bad();
        for (int i = 0; i < nw; ++i) w[i] = (i % 2 == 0) ? src[1 + i / 2] >> 4 : src[1 + i / 2] & 15;
        used = 1 + bytes;
    } else {
        if (1 + (uint64_t)hdr > n || hdr == 0) bad();
        const uint8_t *s = src + 1;
        FseTable t;
        const uint64_t th = fse_read(t, s, hdr, 6, 255);
        if (th >= hdr) bad();
        BackBits b;
        b.init(s + th, hdr - th);
        uint32_t s1 = (uint32_t)b.get(t.log), s2 = (uint32_t)b.get(t.log);
        if (b.off < 0) bad();
        for (;;) {
            if (nw >= 255) bad();
            w[nw++] = t.sym[s1];
            s1 = t.base[s1] + (uint32_t)b.get(t.nb[s1]);
            if (b.off < 0) {
                if (nw >= 255) bad();
                w[nw++] = t.sym[s2];
                break;
            }
            if (nw >= 255) bad();
            w[nw++] = t.sym[s2];
            s2 = t.base[s2] + (uint32_t)b.get(t.nb[s2]);
            if (b.off < 0) {
                if (nw >= 255) bad();
                w[nw++] = t.sym[s1];
                break;
            }
        }
        used = 1 + hdr;
    }
    // the last symbol's weight is implied: it completes the sum of 2^(w-1) to a power of two
    uint32_t total = 0;
    for (int i = 0; i < nw; ++i) {
        if (w[i] > 11) bad();
        if (w[i]) total += 1u << (w[i] - 1);
    }
    if (total == 0) bad();
    const int maxbits = hibit(total) + 1;
    if (maxbits > 11) bad();
    const uint32_t rest = (1u << maxbits) - total;
    if (rest & (rest - 1)) bad();
    if (nw >= 256) bad();
    w[nw++] = (uint8_t)(hibit(rest) + 1);
    h.maxbits = maxbits;
    const uint32_t size = 1u << maxbits;
    h.sym.assign(size, 0);
    h.nb.assign(size, 0);
    uint32_t pos = 0;
    for (int wt = 1; wt <= maxbits; ++wt)
        for (int s = 0; s < nw; ++s) {
            if (w[s] != wt) continue;
            const uint32_t len = 1u << (wt - 1);
            for (uint32_t k = 0; k < len; ++k) {
                h.sym[pos + k] = (uint8_t)s;
                h.nb[pos + k] = (uint8_t)(maxbits + 1 - wt);
            }
            pos += len;
        }
    if (pos != size) bad();
    h.set = true;
    return used;
}

// One Huffman stream of `count` symbols; the stream must be consumed exactly.
void huf_stream(const HufTable &h, const uint8_t *src, uint64_t n, uint8_t *out, uint64_t count) {
    BackBits b;
    b.init(src, n);
    for (uint64_t i = 0; i < count; ++i) {
        // peek maxbits (zero-extended past the start), then consume the symbol's length
        const int64_t save = b.off;
        const uint32_t idx = (uint32_t)b.get(h.maxbits);
        b.off = save - h.nb[idx];
        out[i] = h.sym[idx];
        if (b.off < 0) bad();
    }
    if (b.off != 0) bad();
}

// ---- sequences ------------------------------------------------------------------------------------
const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,    14,    15,    16,    18,
                              20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,  16,   17,   18,   19,   20,
                              21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,  34,   35,   37,   39,   41,
                              43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                             0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
const int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                            1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
const int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

struct FrameState {
    HufTable huf;
    FseTable ll, of, ml;
    uint32_t rep[3] = {1, 4, 8};
};

// One table of the sequences section header: mode 0 predefined, 1 RLE, 2 FSE, 3 repeat.
uint64_t seq_table(FseTable &t, uint32_t mode, const uint8_t *src, uint64_t n, const int16_t *def, int ndef, int deflog,
                   int maxlog, int maxsym) {
    switch (mode) {
        case 0:
            fse_build(t, def, ndef, deflog);
            return 0;
        case 1:
            if (n < 1) bad();
            if (src[0] > maxsym) bad();
            fse_rle(t, src[0]);
            return 1;
        case 2:
            return fse_read(t, src, n, maxlog, maxsym);
        default:
            if (!t.set) bad();
            return 0;
    }
}

// A compressed block: literals, sequences, execution into out[op ..]; returns the new op.
uint64_t compressed_block(FrameState &fs, const uint8_t *src, uint64_t n, uint8_t *out, uint64_t op, uint64_t cap,
                          uint64_t frame_start) {
    if (n < 1) bad();
    // literals section
    const uint32_t ltype = src[0] & 3, sf = (src[0] >> 2) & 3;
    uint64_t regen, csize = 0, hl;
    int nstreams = 1;
    if (ltype <= 1) {
        if (sf == 0 || sf == 2) {
            regen = src[0] >> 3;
            hl = 1;
        } else if (sf == 1) {
            if (n < 2) bad();
            regen = (src[0] >> 4) + ((uint64_t)src[1] << 4);
            hl = 2;
        } else {
            if (n < 3) bad();
            regen = (src[0] >> 4) + ((uint64_t)src[1] << 4) + ((uint64_t)src[2] << 12);
            hl = 3;
        }
    } else {
        if (sf <= 1) {
            if (n < 3) bad();
            const uint32_t h = src[0] | (uint32_t)src[1] << 8 | (uint32_t)src[2] << 16;
            regen = (h >> 4) & 0x3FF;
            csize = (h >> 14) & 0x3FF;
            hl = 3;
            nstreams = sf == 0 ? 1 : 4;
        } else if (sf == 2) {
            if (n < 4) bad();
            const uint32_t h = rd32u(src);
            regen = (h >> 4) & 0x3FFF;
            csize = (h >> 18) & 0x3FFF;
            hl = 4;
            nstreams = 4;
        } else {
            if (n < 5) bad();
            const uint64_t h = rd32u(src) | (uint64_t)src[4] << 32;
            regen = (h >> 4) & 0x3FFFF;
            csize = (h >> 22) & 0x3FFFF;
            hl = 5;
            nstreams = 4;
        }
    }
    if (regen > (128u << 10)) bad();
    std::vector<uint8_t> lit(regen);
    uint64_t p = hl;
    if (ltype == 0) {
        if (p + regen > n) bad();
        std::memcpy(lit.data(), src + p, regen);
        p += regen;
    } else if (ltype == 1) {
        if (p + 1 > n) bad();
        std::memset(lit.data(), src[p], regen);
        p += 1;
    } else {
        if (p + csize > n) bad();
        const uint8_t *ls = src + p;
        uint64_t lp = 0;
        if (ltype == 2) lp = huf_read(fs.huf, ls, csize);
        else if (!fs.huf.set) bad();
        if (lp > csize) bad();
        if (nstreams == 1) {
            huf_stream(fs.huf, ls + lp, csize - lp, lit.data(), regen);
        } else {
            if (csize - lp < 10 || regen < 6) bad();   // HUF_decompress4X: jump table + 1 byte per stream, >= 6 out
            const uint64_t s1 = ls[lp] | (uint64_t)ls[lp + 1] << 8, s2 = ls[lp + 2] | (uint64_t)ls[lp + 3] << 8,
                           s3 = ls[lp + 4] | (uint64_t)ls[lp + 5] << 8;
            const uint64_t total = csize - lp - 6;
            if (s1 + s2 + s3 > total) bad();
            const uint64_t s4 = total - s1 - s2 - s3;
            const uint64_t seg = (regen + 3) / 4;
            if (3 * seg > regen) bad();
            const uint8_t *d = ls + lp + 6;
            huf_stream(fs.huf, d, s1, lit.data(), seg);
            huf_stream(fs.huf, d + s1, s2, lit.data() + seg, seg);
            huf_stream(fs.huf, d + s1 + s2, s3, lit.data() + 2 * seg, seg);
            huf_stream(fs.huf, d + s1 + s2 + s3, s4, lit.data() + 3 * seg, regen - 3 * seg);
        }
        p += csize;
    }
    // sequences section
    if (p >= n) bad();
    uint64_t nseq = src[p++];
    if (nseq >= 128) {
        if (nseq < 255) {
            if (p >= n) bad();
            nseq = ((nseq - 128) << 8) + src[p++];
        } else {
            if (p + 2 > n) bad();
            nseq = src[p] + ((uint64_t)src[p + 1] << 8) + 0x7F00;
            p += 2;
        }
    }
    uint64_t lpos = 0;
    if (nseq > 0) {
        if (p >= n) bad();
        const uint8_t modes = src[p++];
        if (modes & 3) bad();
        p += seq_table(fs.ll, modes >> 6, src + p, n - p, kLLDef, 36, 6, 9, 35);
        p += seq_table(fs.of, (modes >> 4) & 3, src + p, n - p, kOFDef, 29, 5, 8, 31);
        p += seq_table(fs.ml, (modes >> 2) & 3, src + p, n - p, kMLDef, 53, 6, 9, 52);
        if (p >= n) bad();
        BackBits b;
        b.init(src + p, n - p);
        uint32_t sll = (uint32_t)b.get(fs.ll.log), sof = (uint32_t)b.get(fs.of.log), sml = (uint32_t)b.get(fs.ml.log);
        for (uint64_t i = 0; i < nseq; ++i) {
            const uint32_t ofc = fs.of.sym[sof], mlc = fs.ml.sym[sml], llc = fs.ll.sym[sll];
            if (ofc > 31 || mlc > 52 || llc > 35) bad();
            const uint64_t ofv = (1ull << ofc) + b.get((int)ofc);
            const uint64_t ml = kMLBase[mlc] + b.get(kMLBits[mlc]);
            const uint64_t ll = kLLBase[llc] + b.get(kLLBits[llc]);
            uint64_t off;
            if (ofv > 3) {
                off = ofv - 3;
                fs.rep[2] = fs.rep[1];
                fs.rep[1] = fs.rep[0];
                fs.rep[0] = (uint32_t)off;
            } else {
                const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0 ? 1 : 0);   // 0..3
                if (idx == 0) {
                    off = fs.rep[0];
                } else if (idx == 3) {
                    off = (uint64_t)fs.rep[0] - 1;
                    if (off == 0) bad();
                    fs.rep[2] = fs.rep[1];
                    fs.rep[1] = fs.rep[0];
                    fs.rep[0] = (uint32_t)off;
                } else {
                    off = fs.rep[idx];
                    if (idx == 2) fs.rep[2] = fs.rep[1];
                    fs.rep[1] = fs.rep[0];
                    fs.rep[0] = (uint32_t)off;
                }
            }
            if (i + 1 < nseq) {   // state updates: literal lengths, match lengths, offsets
                sll = fs.ll.base[sll] + (uint32_t)b.get(fs.ll.nb[sll]);
                sml = fs.ml.base[sml] + (uint32_t)b.get(fs.ml.nb[sml]);
                sof = fs.of.base[sof] + (uint32_t)b.get(fs.of.nb[sof]);
            }
            if (b.off < 0) bad();
            // execute: ll literals, then ml bytes from off back
            if (ll > regen - lpos || op + ll > cap) bad();
            std::memcpy(out + op, lit.data() + lpos, ll);
            op += ll;
            lpos += ll;
            if (off > op - frame_start || op + ml > cap) bad();
            for (uint64_t k = 0; k < ml; ++k, ++op) out[op] = out[op - off];
        }
        if (b.off != 0) bad();
    } else if (p != n) {
        bad();
    }
    const uint64_t rest = regen - lpos;
    if (op + rest > cap) bad();
    std::memcpy(out + op, lit.data() + lpos, rest);
    return op + rest;
}

// One frame at src[0..); returns the bytes it used; output appended at out[op ..].
uint64_t frame(const uint8_t *src, uint64_t n, uint8_t *out, uint64_t &op, uint64_t cap) {
    if (n < 4) bad();
    const uint32_t magic = rd32u(src);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {   // skippable frame
        if (n < 8) bad();
        const uint64_t sz = rd32u(src + 4);
        if (8 + sz > n) bad();
        return 8 + sz;
    }
    if (magic != 0xFD2FB528u) bad();
    uint64_t p = 4;
    if (p >= n) bad();
    const uint8_t fhd = src[p++];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (fhd & 0x08) bad();   // reserved bit
    uint64_t window = 0;
    if (!single) {
        if (p >= n) bad();
        const uint8_t wd = src[p++];
        const uint32_t exp = wd >> 3, man = wd & 7;
        const uint64_t wlog = 10 + exp;
        if (wlog > 31) bad();
        const uint64_t wbase = 1ull << wlog;
        window = wbase + (wbase / 8) * man;
        if (wlog > 27) bad();   // ZSTD_WINDOWLOG_LIMIT_DEFAULT: "Frame requires too much memory"
    }
    const uint32_t did_bytes = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    if (p + did_bytes > n) bad();
    uint64_t did = 0;
    for (uint32_t k = 0; k < did_bytes; ++k) did |= (uint64_t)src[p + k] << (8 * k);
    p += did_bytes;
    if (did != 0) bad();   // no dictionary available
    const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (p + fcs_bytes > n) bad();
    uint64_t fcs = 0;
    bool has_fcs = fcs_bytes > 0;
    for (uint32_t k = 0; k < fcs_bytes; ++k) fcs |= (uint64_t)src[p + k] << (8 * k);
    if (fcs_bytes == 2) fcs += 256;
    p += fcs_bytes;
    if (single) window = fcs;
    const uint64_t bmax = window < (128u << 10) ? window : (128u << 10);
    const uint64_t start = op;
    FrameState fs;
    for (;;) {
        if (p + 3 > n) bad();
        const uint32_t bh = src[p] | (uint32_t)src[p + 1] << 8 | (uint32_t)src[p + 2] << 16;
        p += 3;
        const uint32_t last = bh & 1, type = (bh >> 1) & 3, bsize = bh >> 3;
        if (type == 3) bad();
        if (type == 0) {
            if (bsize > bmax || p + bsize > n || op + bsize > cap) bad();
            std::memcpy(out + op, src + p, bsize);
            op += bsize;
            p += bsize;
        } else if (type == 1) {
            if (bsize > bmax || p + 1 > n || op + bsize > cap) bad();
            std::memset(out + op, src[p], bsize);
            op += bsize;
            p += 1;
        } else {
            if (bsize > bmax || p + bsize > n) bad();
            const uint64_t before = op;
            op = compressed_block(fs, src + p, bsize, out, op, cap, start);
            if (op - before > bmax) bad();
            p += bsize;
        }
        if (last) break;
    }
    if (has_fcs && op - start != fcs) bad();
    if (checksum) {
        if (p + 4 > n) bad();
        if ((uint32_t)xxh64(out + start, op - start) != rd32u(src + p)) bad();
        p += 4;
    }
    return p;
}

}  // namespace

extern "C" {

// ZSTD_decompressDCtx over src (concatenated frames, skippable frames skipped): 0 and *out_len, or -1.
int oracle_zstd_decompress(const uint8_t *src, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    uint64_t op = 0;
    *out_len = 0;
    try {
        if (n == 0) bad();
        uint64_t p = 0;
        while (p < n) p += frame(src + p, n - p, out, op, cap);
    } catch (const ZFail &) {
        return -1;
    }
    *out_len = op;
    return 0;
}

uint64_t oracle_xxh64(const uint8_t *p, uint64_t n) { return xxh64(p, n); }

}  // extern "C"
