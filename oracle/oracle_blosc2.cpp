// ============================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY: CPU restatement of the blosc2 branch of the reference's
//  decompression stage (src/compression.rs:29-57 decompress_blusc_blosc2).
//
//  The reference calls the un-vendored crate blusc 0.0.2 (Cargo.lock; a pure-Rust port of c-blosc2):
//    blosc2_cbuffer_sizes(data) -> (nbytes, cbytes, blocksize); nbytes == 0 => "invalid blosc2
//        compressed data" (compression.rs:33-39)
//    blosc2_decompress(data, out) -> written; <= 0 => "failed to decompress blosc2 data";
//        != nbytes => "unexpected decompressed size for blosc2 data" (compression.rs:44-55)
//  Neither blusc nor c-blosc2 is present in this image, so this file restates the PUBLISHED blosc2
//  chunk format (c-blosc2 README_CHUNK_FORMAT: 16-byte header, 32-byte extended header, bstarts,
//  per-block streams with the 4-byte csize prefix, runs and memcpy'ed streams, special-value chunks)
//  and codecs (BloscLZ = FastLZ level-2 token format; the LZ4 block format; zlib = RFC 1950 through
//  oracle_inflate.cpp; Snappy = the raw format of google/snappy format_description.txt, which blusc
//  decodes through the `snap` crate, Cargo.lock: blusc -> snap; zstd frames through oracle_zstd.cpp), and the filters' published definitions (byte shuffle per block, bitshuffle
//  = bshuf_trans_bit_elem over the first size - size % 8 elements).
//  PARITY UNPINNED beyond the reference's own tests (compression.rs:90-143,164-175: the "hello world"
//  round trip, which blosc stores memcpy'ed, and the invalid-header message), because no blosc2
//  library, fixture or encoder exists here: chunks are written by this repo's own writer
//  (datagen/blosc2_chunk.py + datagen/blosc2_writer.cpp), so decoder and writer are checked against
//  each other and the format description only.
//  dictionaries / delta / user-defined codecs: RDX_BLOSC2_UNSUPPORTED.
// ============================================================================================
#include "../include/rdx.h"

#include <cstdint>
#include <cstring>
#include <vector>

extern "C" int oracle_zstd_decompress(const uint8_t *src, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
extern "C" uint32_t oracle_decompress(uint32_t compression, const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap,
                                      uint64_t *out_len);

namespace {

constexpr uint32_t kMinHeader = 16, kExtHeader = 32;
constexpr int32_t kMaxBlock = 536866816;      // BLOSC2_MAXBLOCKSIZE
constexpr uint8_t kVersionMax = 5;            // BLOSC2_VERSION_FORMAT (c-blosc2 2.x)
enum : uint8_t { F_SHUFFLE = 1, F_MEMCPYED = 2, F_BITSHUFFLE = 4, F_DELTA = 8, F_DONT_SPLIT = 0x10 };
enum : uint8_t { FLT_NONE = 0, FLT_SHUFFLE = 1, FLT_BITSHUFFLE = 2, FLT_DELTA = 3, FLT_TRUNC = 4 };
enum : uint8_t { C_BLOSCLZ = 0, C_LZ4 = 1, C_SNAPPY = 2, C_ZLIB = 3, C_ZSTD = 4 };

struct Fail {
    uint32_t code;
};

int32_t rd32(const uint8_t *p) { return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24); }

struct Header {
    uint8_t version, versionlz, flags, typesize;
    int32_t nbytes, blocksize, cbytes;
    bool ext;
    uint8_t filters[6];
    uint8_t udcodec, b2flags;
    uint32_t overhead;
};

// read_chunk_header's checks on the first 16 bytes (what blosc2_cbuffer_sizes reads)
bool read_min(const uint8_t *s, uint64_t len, Header &h) {
    if (len < kMinHeader) return false;
    h.version = s[0];
    h.versionlz = s[1];
    h.flags = s[2];
    h.typesize = s[3];
    h.nbytes = rd32(s + 4);
    h.blocksize = rd32(s + 8);
    h.cbytes = rd32(s + 12);
    if (h.cbytes < (int32_t)kMinHeader) return false;
    if (h.version == 0 || h.version > kVersionMax) return false;
    if (h.blocksize <= 0 || (h.nbytes > 0 && h.blocksize > h.nbytes)) return false;
    if (h.blocksize > kMaxBlock) return false;
    if (h.typesize == 0) return false;
    if (h.nbytes <= 0) return false;   // compression.rs:35: nbytes == 0 is invalid
    return true;
}

// BloscLZ stream (blosclz_decompress): literal runs ctrl < 32 (ctrl + 1 bytes); matches ctrl >= 32:
// length (ctrl >> 5) + 2 (7: + extension bytes until one is not 255), distance ((ctrl & 31) << 8) +
// code + 1, or 8192 + a 16-bit big-endian offset after the escape (ctrl & 31) == 31, code == 255.
// A match must be followed by at least one more token.  Returns bytes written or -1.
int64_t blosclz_dec(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t maxout) {
    if (n == 0) return 0;
    const uint8_t *ip = in, *ipl = in + n;
    uint64_t op = 0;
    uint32_t ctrl = *ip++ & 31u;
    for (;;) {
        if (ctrl >= 32) {
            uint64_t len = (ctrl >> 5) - 1;
            uint64_t ofs = (uint64_t)(ctrl & 31u) << 8;
            if (len == 6) {
                uint8_t c;
                do {
                    if (ip + 1 >= ipl) return -1;
                    c = *ip++;
                    len += c;
                } while (c == 255);
            } else if (ip + 1 >= ipl) {
                return -1;
            }
            const uint8_t code = *ip++;
            len += 3;
            uint64_t dist = ofs + code + 1;
            if (code == 255 && ofs == (31u << 8)) {
                if (ip + 1 >= ipl) return -1;
                ofs = (uint64_t)ip[0] << 8 | ip[1];
                ip += 2;
                dist = ofs + 8192;
            }
            if (op + len > maxout) return -1;
            if (dist > op) return -1;
            if (ip >= ipl) return -1;   // the match would be dropped: short output
            ctrl = *ip++;
            for (uint64_t k = 0; k < len; ++k, ++op) out[op] = out[op - dist];
        } else {
            const uint64_t run = ctrl + 1;
            if (op + run > maxout || ip + run > ipl) return -1;
            std::memcpy(out + op, ip, run);
            op += run;
            ip += run;
            if (ip >= ipl) break;
            ctrl = *ip++;
        }
    }
    return (int64_t)op;
}

// LZ4 block (LZ4_decompress_safe): token = literal length (4 bits) | match length - 4 (4 bits), 255-run
// extensions, literals, 2-byte little-endian offset.  End-of-block rules: a sequence whose literals end
// within 12 bytes of the output end (MFLIMIT) or within 8 bytes of the input end must be the last
// and end the input exactly; a match must end at least 5 bytes before the output end (LASTLITERALS).
int64_t lz4_dec(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t maxout) {
    const uint8_t *ip = in, *iend = in + n;
    uint64_t op = 0;
    if (n == 0) return -1;
    for (;;) {
        if (ip >= iend) return -1;
        const uint32_t token = *ip++;
        uint64_t L = token >> 4;
        if (L == 15) {
            uint8_t b;
            do {
                if (ip >= iend) return -1;
                b = *ip++;
                L += b;
            } while (b == 255);
        }
        if ((uint64_t)(iend - ip) < L || maxout - op < L) return -1;
        std::memcpy(out + op, ip, L);
        op += L;
        ip += L;
        if (op + 12 > maxout || ip + 8 > iend) {   // must be the last sequence
            if (ip != iend) return -1;
            break;
        }
        const uint64_t off = (uint64_t)ip[0] | (uint64_t)ip[1] << 8;
        ip += 2;
        if (off == 0 || off > op) return -1;
        uint64_t M = token & 15u;
        if (M == 15) {
            uint8_t b;
            do {
                if (ip >= iend) return -1;
                b = *ip++;
                M += b;
            } while (b == 255);
        }
        M += 4;
        if (op + M + 5 > maxout) return -1;
        for (uint64_t k = 0; k < M; ++k, ++op) out[op] = out[op - off];
    }
    return (int64_t)op;
}

// Snappy raw block (snap::raw::Decoder::decompress): a varint preamble (<= 5 bytes) holding the decoded
// length, which must fit the output; then elements by the tag's low 2 bits: 0 literal (length
// (tag >> 2) + 1, or for 60..63 a 1-4 byte little-endian length - 1 after the tag), 1 copy with an 11-bit
// offset (length 4 + ((tag >> 2) & 7), offset (tag >> 5) << 8 | next byte), 2 / 3 copies with a 2 / 4
// byte little-endian offset (length (tag >> 2) + 1).  Offset 0, an offset past the bytes written, an
// element overrunning the input or the preamble's length, or an end short of that length: error.
int64_t snappy_dec(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t maxout) {
    uint64_t ip = 0, want = 0;
    for (int sh = 0;; sh += 7) {
        if (ip >= n || sh > 28) return -1;
        const uint8_t b = in[ip++];
        if (sh == 28 && b > 15) return -1;   // beyond 32 bits
        want |= (uint64_t)(b & 127u) << sh;
        if (!(b & 128)) break;
    }
    if (want > maxout) return -1;
    uint64_t op = 0;
    while (ip < n) {
        const uint32_t tag = in[ip++];
        uint64_t len, off = 0;
        if ((tag & 3) == 0) {
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t nb = (uint32_t)len - 59;
                if (ip + nb > n) return -1;
                len = 0;
                for (uint32_t k = 0; k < nb; ++k) len |= (uint64_t)in[ip + k] << (8 * k);
                ip += nb;
            }
            len += 1;
            if (n - ip < len || want - op < len) return -1;
            std::memcpy(out + op, in + ip, len);
            op += len;
            ip += len;
            continue;
        }
        if ((tag & 3) == 1) {
            if (ip + 1 > n) return -1;
            len = 4 + ((tag >> 2) & 7u);
            off = (uint64_t)(tag >> 5) << 8 | in[ip];
            ip += 1;
        } else {
            const uint32_t nb = (tag & 3) == 2 ? 2 : 4;
            if (ip + nb > n) return -1;
            len = (tag >> 2) + 1;
            for (uint32_t k = 0; k < nb; ++k) off |= (uint64_t)in[ip + k] << (8 * k);
            ip += nb;
        }
        if (off == 0 || off > op || want - op < len) return -1;
        for (uint64_t k = 0; k < len; ++k, ++op) out[op] = out[op - off];
    }
    return op == want ? (int64_t)op : -1;
}

// unshuffle (blosc shuffle.c): the first (bsize / ts) * ts bytes are ts planes; the rest copied
void unshuffle(uint32_t ts, uint64_t bsize, const uint8_t *src, uint8_t *dst) {
    const uint64_t ne = bsize / ts;
    for (uint64_t i = 0; i < ne; ++i)
        for (uint32_t k = 0; k < ts; ++k) dst[i * ts + k] = src[k * ne + i];
    std::memcpy(dst + ne * ts, src + ne * ts, bsize - ne * ts);
}

// bitunshuffle: over size = bsize / ts elements rounded down to a multiple of 8, row r = 8 * byte + bit
// holds that bit of every element (element e at byte e / 8, bit e % 8 of the row); the rest copied.
// Chunks of header version 2 (written by c-blosc 1.x, e.g. numcodecs' Blosc) follow the older rule of
// c-blosc2's bitunshuffle(..., format_version): a block whose element count is not a multiple of 8 was
// stored unshuffled and is copied whole.
void bitunshuffle(uint32_t ts, uint64_t bsize, const uint8_t *src, uint8_t *dst, uint32_t version) {
    uint64_t size = bsize / ts;
    if (version == 2 && size % 8 != 0) {
        std::memcpy(dst, src, bsize);
        return;
    }
    size -= size % 8;
    const uint64_t rowb = size / 8;
    std::memset(dst, 0, size * ts);
    for (uint32_t k = 0; k < ts; ++k)
        for (uint32_t b = 0; b < 8; ++b) {
            const uint8_t *row = src + (uint64_t)(k * 8 + b) * rowb;
            for (uint64_t e = 0; e < size; ++e)
                if ((row[e / 8] >> (e % 8)) & 1) dst[e * ts + k] |= (uint8_t)(1u << b);
        }
    std::memcpy(dst + size * ts, src + size * ts, bsize - size * ts);
}

// blosc2_decompress: the full header, then every block (blosc_d) and its filters backwards
uint64_t decompress(const uint8_t *s, uint64_t len, uint8_t *out, uint64_t cap) {
    Header h{};
    if (!read_min(s, len, h)) throw Fail{RDX_BLOSC2_INVALID};
    if ((uint64_t)h.cbytes > len) throw Fail{RDX_BLOSC2_FAILED};
    if ((uint64_t)h.nbytes > cap) throw Fail{RDX_INFLATE_OUTPUT_OVERFLOW};
    const uint64_t srcsize = (uint64_t)h.cbytes;
    h.ext = (h.flags & F_SHUFFLE) && (h.flags & F_BITSHUFFLE);
    std::memset(h.filters, 0, sizeof h.filters);
    if (h.ext) {
        if (srcsize < kExtHeader) throw Fail{RDX_BLOSC2_FAILED};
        std::memcpy(h.filters, s + 16, 6);
        h.udcodec = s[22];
        h.b2flags = s[31];
        h.overhead = kExtHeader;
        const uint32_t special = (h.b2flags >> 4) & 7u;
        if (special) {
            const uint64_t nb = (uint64_t)h.nbytes;
            if (nb % h.typesize) throw Fail{RDX_BLOSC2_FAILED};
            switch (special) {
                case 1:   // BLOSC2_SPECIAL_ZERO
                case 4:   // BLOSC2_SPECIAL_UNINIT (contents undefined: zeros here)
                    std::memset(out, 0, nb);
                    return nb;
                case 2: {  // BLOSC2_SPECIAL_NAN: typesize 4 or 8
                    if (h.typesize != 4 && h.typesize != 8) throw Fail{RDX_BLOSC2_FAILED};
                    const uint64_t nan8 = 0x7FF8000000000000ull;
                    const uint32_t nan4 = 0x7FC00000u;
                    for (uint64_t i = 0; i < nb; i += h.typesize)
                        std::memcpy(out + i, h.typesize == 4 ? (const void *)&nan4 : (const void *)&nan8, h.typesize);
                    return nb;
                }
                case 3: {  // BLOSC2_SPECIAL_VALUE: the value follows the header, typesize = cbytes - 32
                    const int32_t vts = h.cbytes - (int32_t)kExtHeader;
                    if (vts <= 0 || vts > 255 || vts > h.nbytes || nb % (uint64_t)vts) throw Fail{RDX_BLOSC2_FAILED};
                    for (uint64_t i = 0; i < nb; i += (uint64_t)vts) std::memcpy(out + i, s + kExtHeader, (size_t)vts);
                    return nb;
                }
                default:
                    throw Fail{RDX_BLOSC2_FAILED};
            }
        }
        if (h.b2flags & 0x08) throw Fail{RDX_BLOSC2_FAILED};          // lazy chunk: frames only
        if (h.b2flags & (0x01 | 0x80)) throw Fail{RDX_BLOSC2_UNSUPPORTED};  // dictionary / instrumented
    } else {
        h.overhead = kMinHeader;
        if (h.flags & F_SHUFFLE) h.filters[5] = FLT_SHUFFLE;
        if (h.flags & F_BITSHUFFLE) h.filters[5] = FLT_BITSHUFFLE;
        if (h.flags & F_DELTA) h.filters[4] = FLT_DELTA;
    }
    const uint64_t nbytes = (uint64_t)h.nbytes, bs = (uint64_t)h.blocksize;
    if (h.flags & F_MEMCPYED) {
        if (nbytes + h.overhead != srcsize) throw Fail{RDX_BLOSC2_FAILED};
        std::memcpy(out, s + h.overhead, nbytes);
        return nbytes;
    }
    const uint32_t codec = h.flags >> 5;
    if (codec == 6) throw Fail{RDX_BLOSC2_UNSUPPORTED};   // BLOSC_CODEC_USER_DEFINED
    if (codec > C_ZSTD) throw Fail{RDX_BLOSC2_FAILED};
    for (uint8_t f : h.filters) {
        if (f == FLT_DELTA || f > FLT_TRUNC) throw Fail{RDX_BLOSC2_UNSUPPORTED};
    }
    const uint64_t nblocks = (nbytes + bs - 1) / bs, leftover = nbytes % bs;
    if (h.overhead + 4 * nblocks > srcsize) throw Fail{RDX_BLOSC2_FAILED};
    const bool dont_split = (h.flags & F_DONT_SPLIT) != 0;
    std::vector<uint8_t> tmp(bs), tmp2(bs);
    for (uint64_t j = 0; j < nblocks; ++j) {
        const bool left = leftover && j == nblocks - 1;
        const uint64_t bsize = left ? leftover : bs;
        const uint32_t nstreams = (!dont_split && !left) ? h.typesize : 1;
        if (bsize % nstreams) throw Fail{RDX_BLOSC2_FAILED};
        const uint64_t neblock = bsize / nstreams;
        const int32_t b0 = rd32(s + h.overhead + 4 * j);
        if (b0 < (int32_t)(h.overhead + 4 * nblocks) || (uint64_t)b0 >= srcsize) throw Fail{RDX_BLOSC2_FAILED};
        uint64_t pos = (uint64_t)b0;
        uint8_t *blk = tmp.data();
        for (uint32_t k = 0; k < nstreams; ++k) {
            uint8_t *d = blk + k * neblock;
            if (pos + 4 > srcsize) throw Fail{RDX_BLOSC2_FAILED};
            const int32_t cb = rd32(s + pos);
            pos += 4;
            if (cb == 0) {
                std::memset(d, 0, neblock);
            } else if (cb < 0) {   // a run: -cb is the byte, a token byte with bit 0 set follows
                if (pos + 1 > srcsize) throw Fail{RDX_BLOSC2_FAILED};
                const uint8_t token = s[pos++];
                if (!(token & 1) || cb < -255) throw Fail{RDX_BLOSC2_FAILED};
                std::memset(d, (uint8_t)(-cb), neblock);
            } else {
                if (pos + (uint64_t)cb > srcsize) throw Fail{RDX_BLOSC2_FAILED};
                if ((uint64_t)cb == neblock) {
                    std::memcpy(d, s + pos, neblock);
                } else {
                    int64_t got = -1;
                    if (codec == C_BLOSCLZ) got = blosclz_dec(s + pos, (uint64_t)cb, d, neblock);
                    else if (codec == C_LZ4) got = lz4_dec(s + pos, (uint64_t)cb, d, neblock);
                    else if (codec == C_SNAPPY) got = snappy_dec(s + pos, (uint64_t)cb, d, neblock);
                    else if (codec == C_ZSTD) {   // zstd_wrap_decompress: ZSTD_decompressDCtx, capacity neblock
                        uint64_t ol = 0;
                        got = oracle_zstd_decompress(s + pos, (uint64_t)cb, d, neblock, &ol) == 0 ? (int64_t)ol : -1;
                    }
                    else {
                        uint64_t ol = 0;
                        const uint32_t e = oracle_decompress(RDX_COMPRESSION_ZLIB, s + pos, (uint64_t)cb, d, neblock, &ol);
                        got = e == RDX_INFLATE_OK ? (int64_t)ol : -1;
                    }
                    if (got != (int64_t)neblock) throw Fail{RDX_BLOSC2_FAILED};
                }
                pos += (uint64_t)cb;
            }
        }
        // pipeline_backward: filters[5] .. filters[0]
        uint8_t *cur = tmp.data(), *nxt = tmp2.data();
        for (int f = 5; f >= 0; --f) {
            if (h.filters[f] == FLT_SHUFFLE && h.typesize > 1) {
                unshuffle(h.typesize, bsize, cur, nxt);
                std::swap(cur, nxt);
            } else if (h.filters[f] == FLT_BITSHUFFLE) {
                bitunshuffle(h.typesize, bsize, cur, nxt, h.version);
                std::swap(cur, nxt);
            }
        }
        std::memcpy(out + j * bs, cur, bsize);
    }
    return nbytes;
}

}  // namespace

extern "C" {

// blosc2_cbuffer_sizes (compression.rs:33): nbytes = 0 when the 16-byte header is invalid.
void oracle_blosc2_sizes(const uint8_t *src, uint64_t len, uint64_t *nbytes, uint64_t *cbytes, uint64_t *blocksize) {
    Header h{};
    if (!read_min(src, len, h)) {
        *nbytes = *cbytes = *blocksize = 0;
        return;
    }
    *nbytes = (uint64_t)h.nbytes;
    *cbytes = (uint64_t)h.cbytes;
    *blocksize = (uint64_t)h.blocksize;
}

// decompress_blusc_blosc2 (compression.rs:29-57): an rdx_inflate_error code; *out_len = bytes produced.
uint32_t oracle_blosc2_decompress(const uint8_t *src, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    *out_len = 0;
    try {
        *out_len = decompress(src, len, out, cap);
    } catch (const Fail &f) {
        return f.code;
    }
    return RDX_INFLATE_OK;
}

}  // extern "C"
