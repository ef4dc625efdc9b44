// k_blosc2 — the blosc2 branch of the decompression stage (src/compression.rs:29-57
// decompress_blusc_blosc2 -> blusc 0.0.2, a pure-Rust port of c-blosc2) on gfx950.
//
// A blosc2 chunk is block-parallel by construction: a 16/32-byte header, a table of block starts, and
// per block `typesize` independently compressed streams (one per byte plane when the block is split)
// or one.  So unlike DEFLATE (k_inflate: one serial stream per chunk) a single chunk already holds
// hundreds of independent streams (4 MiB at 64 KiB blocks and typesize 4: 256), and the device
// parallelism is within the chunk:
//   k_blosc2_decode  one WAVEFRONT per stream (work items = (block, stream), looped over the chunk's
//                    waves).  Every wave parses the header itself (no host round trip for a
//                    device-resident chunk) and validates it exactly as the oracle does, so all waves
//                    agree on a header-level error.  A stream is a zero run, a byte run, a raw copy or
//                    a BloscLZ / LZ4 / Snappy stream.  LZ decoding is wave-uniform serial control (token fields
//                    made scalar with readfirstlane) over an LDS input ring (1 KiB units, the next unit
//                    prefetched into registers) and an LDS output ring holding the recent window;
//                    literal runs and matches move 64 bytes per step, one per lane (a match of
//                    distance d < 64 reads o - d + (t mod d), so every source is history written before
//                    the step); the ring is flushed to HBM in RING/4 units with 16-byte stores; a match
//                    source farther back than the ring reads the flushed output (agent-scope loads,
//                    after the flush's stores drained).
//   k_blosc2_filter  one workgroup per block: the block's filters backwards (byte unshuffle,
//                    bitunshuffle) from the decode scratch into the output.  Chunks without an active
//                    filter are decoded straight into the output and skip this launch's work.
// Memcpy'ed and special-value chunks (zeros, NaN, a repeated value, uninitialised) are copied / filled
// by the decode launch in 4 KiB units.
// zlib-coded streams are not decoded here: each becomes a row of a stream table (source, length,
// destination, expected size) that k_inflate decodes in the next launch, k_blosc2_zcheck folds their
// results into the chunks' errors, then k_blosc2_filter runs.
// zstd-coded streams go through the same table (its second half) to k_blosc2_zstd (below).
// Unsupported here (RDX_BLOSC2_UNSUPPORTED): dictionaries, delta, user-defined codecs / filters, zstd
// frames with a content checksum, more than 512 zlib- or zstd-coded streams per chunk of a batch.
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

// (A/B builds: RDX_B2_RING / RDX_B2_IN set the per-wave LDS, which bounds the waves per CU of k_blosc2_decode;
// RDX_B2_WPE > 0 asks the compiler for that many waves per SIMD)
#ifndef RDX_B2_RING
#define RDX_B2_RING 8192
#endif
#ifndef RDX_B2_IN
#define RDX_B2_IN 2048
#endif
#ifndef RDX_B2_WPE
#define RDX_B2_WPE 0
#endif
constexpr uint32_t kWaves = 4;
constexpr uint32_t kRing = RDX_B2_RING;
constexpr uint32_t kInBytes = RDX_B2_IN, kInWords = kInBytes / 4, kStage = kInBytes / 2;
constexpr uint32_t kUnit = 4096;   // memcpy'ed / special chunks: bytes per work item

template <uint32_t R>
struct __attribute__((aligned(16))) WaveLdsT {
    uint8_t win[R];
    uint32_t in[kInWords];
};
using WaveLds = WaveLdsT<kRing>;

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return (uint64_t)rfl((uint32_t)x) | (uint64_t)rfl((uint32_t)(x >> 32)) << 32;
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// a little-endian i32 at any byte address (all lanes load the same bytes: one round trip)
__device__ __forceinline__ int32_t ld_i32(const uint8_t *p) {
    const uint32_t v = (uint32_t)gld<uint8_t>(p) | (uint32_t)gld<uint8_t>(p + 1) << 8 |
                       (uint32_t)gld<uint8_t>(p + 2) << 16 | (uint32_t)gld<uint8_t>(p + 3) << 24;
    return (int32_t)rfl(v);
}
__device__ __forceinline__ void fail(uint32_t *err, uint32_t code) {
    if ((threadIdx.x & 63) == 0) atomicCAS(err, 0u, code);
}

enum : uint32_t { M_BLOCKS = 0, M_MEMCPY = 1, M_SPECIAL = 2 };

// The chunk header as the oracle reads it (oracle_blosc2.cpp read_min / decompress), wave-uniform.
struct Hdr {
    uint32_t code;        // 0 or the rdx_inflate_error every wave of this chunk reports
    uint32_t mode, flags, ts, codec, special, vts, overhead, nstreams;
    uint32_t filt;        // active decode filters, filters[5] first: 2 bits each (1 shuffle, 2 bitshuffle)
    uint32_t nfilt;
    uint32_t version;     // header byte 0: version 2 (c-blosc 1.x) keeps the old bitshuffle leftover rule
    uint64_t nbytes, bs, cbytes, nblocks, leftover, items;
};

__device__ Hdr parse(const uint8_t *src, uint64_t len, uint64_t cap, bool zlib) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t b = 0;
    if (lane < 32 && lane < len) b = gld<uint8_t>(src + lane);
    auto hb = [&](uint32_t k) { return rfl((uint32_t)__shfl((int)b, (int)k, 64) & 0xffu); };
    auto h32 = [&](uint32_t k) { return (int32_t)(hb(k) | hb(k + 1) << 8 | hb(k + 2) << 16 | hb(k + 3) << 24); };
    Hdr h{};
    const uint32_t version = hb(0);
    h.flags = hb(2);
    h.ts = hb(3);
    const int32_t nb = h32(4), bs = h32(8), cb = h32(12);
    h.code = 0;
    h.version = version;
    if (len < 16 || cb < 16 || version == 0 || version > 5 || bs <= 0 || (nb > 0 && bs > nb) || bs > 536866816 ||
        h.ts == 0 || nb <= 0) {
        h.code = RDX_BLOSC2_INVALID;
        return h;
    }
    h.nbytes = (uint64_t)nb;
    h.bs = (uint64_t)bs;
    h.cbytes = (uint64_t)cb;
    if (h.cbytes > len) { h.code = RDX_BLOSC2_FAILED; return h; }
    if (h.nbytes > cap) { h.code = RDX_INFLATE_OUTPUT_OVERFLOW; return h; }
    const bool ext = (h.flags & 1) && (h.flags & 4);
    uint32_t f[6] = {0, 0, 0, 0, 0, 0};
    if (ext) {
        if (h.cbytes < 32) { h.code = RDX_BLOSC2_FAILED; return h; }
        for (int k = 0; k < 6; ++k) f[k] = hb(16 + k);
        const uint32_t b2 = hb(31);
        h.overhead = 32;
        h.special = (b2 >> 4) & 7u;
        if (h.special) {
            h.mode = M_SPECIAL;
            if (h.nbytes % h.ts) h.code = RDX_BLOSC2_FAILED;
            else if (h.special == 2 && h.ts != 4 && h.ts != 8) h.code = RDX_BLOSC2_FAILED;
            else if (h.special == 3) {
                const int32_t v = cb - 32;
                if (v <= 0 || v > 255 || v > nb || h.nbytes % (uint64_t)v) h.code = RDX_BLOSC2_FAILED;
                h.vts = (uint32_t)v;
            } else if (h.special > 4) h.code = RDX_BLOSC2_FAILED;
            h.items = (h.nbytes + kUnit - 1) / kUnit;
            return h;
        }
        if (b2 & 0x08) { h.code = RDX_BLOSC2_FAILED; return h; }
        if (b2 & 0x81) { h.code = RDX_BLOSC2_UNSUPPORTED; return h; }
    } else {
        h.overhead = 16;
        if (h.flags & 1) f[5] = 1;
        if (h.flags & 4) f[5] = 2;
        if (h.flags & 8) f[4] = 3;
    }
    if (h.flags & 2) {
        h.mode = M_MEMCPY;
        if (h.nbytes + h.overhead != h.cbytes) h.code = RDX_BLOSC2_FAILED;
        h.items = (h.nbytes + kUnit - 1) / kUnit;
        return h;
    }
    h.mode = M_BLOCKS;
    h.codec = h.flags >> 5;
    // zlib-coded streams go to k_inflate through the stream table (refused when the caller gave none)
    if (h.codec == 6 || ((h.codec == 3 || h.codec == 4) && !zlib)) {
        h.code = RDX_BLOSC2_UNSUPPORTED;
        return h;
    }
    if (h.codec > 4) { h.code = RDX_BLOSC2_FAILED; return h; }
    for (int k = 0; k < 6; ++k)
        if (f[k] == 3 || f[k] > 4) { h.code = RDX_BLOSC2_UNSUPPORTED; return h; }
    h.filt = 0;
    h.nfilt = 0;
    for (int k = 5; k >= 0; --k) {
        const uint32_t a = (f[k] == 1 && h.ts > 1) ? 1u : (f[k] == 2 ? 2u : 0u);
        if (a) h.filt |= a << (2 * h.nfilt++);
    }
    h.nblocks = (h.nbytes + h.bs - 1) / h.bs;
    h.leftover = h.nbytes % h.bs;
    if (h.overhead + 4 * h.nblocks > h.cbytes) { h.code = RDX_BLOSC2_FAILED; return h; }
    h.nstreams = (h.flags & 0x10) ? 1u : h.ts;
    const uint64_t nfull = h.nbytes / h.bs;
    if (nfull && h.bs % h.nstreams) { h.code = RDX_BLOSC2_FAILED; return h; }
    h.items = nfull * h.nstreams + (h.leftover ? 1 : 0);
    return h;
}

// Wave-cooperative copy of n bytes (dst any alignment, src any alignment): dword stores once dst is
// 4-byte aligned, each lane's dword assembled from two aligned source dwords.
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t head = (4 - ((uintptr_t)dst & 3)) & 3;
    if (head > n) head = n;
    if (lane < head) dst[lane] = gld<uint8_t>(src + lane);
    dst += head;
    src += head;
    n -= head;
    const uint32_t sk = (uint32_t)((uintptr_t)src & 3);
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(src - sk);
    const uint64_t nw = n / 4;
    for (uint64_t w = lane; w < nw; w += 64) {
        uint32_t v;
        if (sk == 0) v = gld<uint32_t>(sw + w);
        else v = __builtin_amdgcn_alignbyte(gld<uint32_t>(sw + w + 1), gld<uint32_t>(sw + w), sk);
        gst<uint32_t>(reinterpret_cast<uint32_t *>(dst) + w, v);
    }
    const uint64_t t = nw * 4;
    if (lane < n - t) dst[t + lane] = gld<uint8_t>(src + t + lane);
}

// Fill n bytes with one byte value: 16-byte stores once dst is aligned.
__device__ __forceinline__ void wave_fill(uint8_t *dst, uint64_t n, uint8_t v) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    if (head > n) head = n;
    if (lane < head) dst[lane] = v;
    const uint32_t w = v * 0x01010101u;
    const uint4 q = make_uint4(w, w, w, w);
    const uint64_t nq = (n - head) / 16;
    for (uint64_t i = lane; i < nq; i += 64) gst<uint4>(dst + head + 16 * i, q);
    for (uint64_t i = head + 16 * nq + lane; i < n; i += 64) dst[i] = v;
}

template <uint32_t R>   // output ring bytes (power of two)
struct LzStreamT {
    static constexpr uint32_t kR = R, kRM = R - 1, kF = R / 4;
    static_assert(R >= 4096 && (R & (R - 1)) == 0, "flush() stores 16-byte slices: kF / 64 >= 16");
    WaveLdsT<R> &L;
    const uint32_t lane;
    const uint32_t *srcw;   // stream as dwords from its 4-byte aligned base
    // positions are 32-bit: a stream is at most a block (BLOSC2_MAXBLOCKSIZE < 2^29), and the token
    // chain is scalar code whose length per token sets the decode rate (64-bit adds cost two SALU ops)
    uint32_t end;           // skew + csize (aligned-stream coordinates)
    uint32_t staged;        // [.., staged) is in the input ring
    uint32_t pf[kStage / 4 / 64];
    uint8_t *dst;
    uint32_t n, op, flushed;

    __device__ __forceinline__ void load_unit(uint32_t start) {
        const uint32_t w0 = start / 4 + (uint32_t)lane * (kStage / 4 / 64);
#pragma unroll
        for (int k = 0; k < (int)(kStage / 4 / 64); ++k) {
            const uint32_t w = w0 + k;
            pf[k] = 0;
            if (w * 4 < end) {
                pf[k] = gld<uint32_t>(srcw + w);
                const uint32_t valid = end - w * 4;
                if (valid < 4) pf[k] &= (1u << (8 * valid)) - 1;
            }
        }
    }
    __device__ __forceinline__ void stage() {
        const uint32_t i0 = (uint32_t)(staged / 4 + (uint32_t)lane * (kStage / 4 / 64));
#pragma unroll
        for (int k = 0; k < (int)(kStage / 4 / 64); ++k) L.in[(i0 + k) & (kInWords - 1)] = pf[k];
        staged += kStage;
        load_unit(staged);
        wave_sync();
    }
    __device__ __forceinline__ void ensure(uint32_t p) {
        while (p > staged) stage();
    }
    // bytes p .. p+7 (aligned-stream coordinates), wave-uniform
    __device__ __forceinline__ uint64_t peek8(uint32_t p) {
        ensure(p + 12);
        const uint32_t i = (uint32_t)(p >> 2), sh = (uint32_t)(p & 3) * 8;
        const uint32_t a = L.in[i & (kInWords - 1)], b = L.in[(i + 1) & (kInWords - 1)],
                       c = L.in[(i + 2) & (kInWords - 1)];
        const uint64_t lo = (uint64_t)a | (uint64_t)b << 32;
        const uint64_t v = sh ? (lo >> sh) | ((uint64_t)c << (64 - sh)) : lo;
        return rfl64(v);
    }
    __device__ __forceinline__ uint8_t in_byte(uint32_t p) const {
        return (uint8_t)(L.in[(p >> 2) & (kInWords - 1)] >> ((p & 3) * 8));
    }

    // write [flushed, flushed + m) of the ring to HBM (m <= kF)
    __device__ __forceinline__ void flush(uint32_t m) {
        constexpr uint32_t kSl = kF / 64;
        wave_sync();
        const uint32_t base = (uint32_t)(flushed & kRM);
        const uint32_t lo = lane * kSl;
        const uint32_t cnt = lo >= m ? 0 : (m - lo < kSl ? m - lo : kSl);
        uint8_t *d = dst + flushed + lo;
        if (cnt == kSl && ((uintptr_t)d & 15) == 0) {
#pragma unroll
            for (uint32_t k = 0; k < kSl / 16; ++k)
                gst<uint4>(d + 16 * k, *reinterpret_cast<const uint4 *>(&L.win[base + lo + 16 * k]));
        } else {
            for (uint32_t k = 0; k < cnt; ++k) gst<uint8_t>(d + k, L.win[(base + lo + k) & kRM]);
        }
        flushed += m;
        // far match sources read these bytes back: their stores must be in L2 first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_sync();
    }
    __device__ __forceinline__ void room() {
        if (op - flushed > kR - 64) flush(kF);
    }
    __device__ __forceinline__ uint8_t far_byte(uint32_t q) const {
        const uintptr_t a = (uintptr_t)(dst + q);
        const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return (uint8_t)(w >> (8 * (a & 3)));
    }
    // literal run of `run` bytes from input position ip
    __device__ __forceinline__ void literals(uint32_t ip, uint32_t run) {
        for (uint32_t s = 0; s < run; s += 64) {
            ensure(ip + s + 64);
            room();
            const uint32_t k = run - s < 64 ? run - s : 64;
            if (lane < k) L.win[(op + lane) & kRM] = in_byte(ip + s + lane);
            op += k;
            asm volatile("" ::: "memory");
        }
    }
    // match of len bytes at distance dist (1 <= dist <= op)
    __device__ __forceinline__ void match(uint32_t len, uint32_t dist) {
        for (uint32_t s = 0; s < len; s += 64) {
            room();
            const uint32_t k = len - s < 64 ? len - s : 64;
            if (lane < k) {
                // lane % dist for dist < 64 without an integer division: (lane + 0.5) / dist stays >= 0.5 / 63
                // away from an integer, far beyond v_rcp_f32's error
                const uint32_t m =
                    dist < 64 ? lane - dist * (uint32_t)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)dist)) : lane;
                const uint32_t back = dist - m, q = op - back;
                const uint8_t v = back <= kR - 64 ? L.win[q & kRM] : far_byte(q);
                L.win[(op + lane) & kRM] = v;
            }
            op += k;
            asm volatile("" ::: "memory");
        }
    }
    __device__ __forceinline__ void finish() {
        while (op > flushed) flush(op - flushed < kF ? (uint32_t)(op - flushed) : kF);
    }
    // stage a new source (zstd: raw literals in the input, or decoded literals in HBM): `avail` bytes at p;
    // returns the aligned-coordinate position of p's first byte (the ip literals() takes)
    __device__ __forceinline__ uint32_t source(const uint8_t *p, uint32_t avail) {
        const uint32_t skew = (uint32_t)((uintptr_t)p & 3);
        srcw = reinterpret_cast<const uint32_t *>(p - skew);
        end = skew + avail;
        staged = 0;
        load_unit(0);
        stage();
        return skew;
    }
    // len copies of byte b (zstd RLE blocks)
    __device__ __forceinline__ void run(uint8_t b, uint32_t len) {
        for (uint32_t s = 0; s < len; s += 64) {
            room();
            const uint32_t k = len - s < 64 ? len - s : 64;
            if (lane < k) L.win[(op + lane) & kRM] = b;
            op += k;
            asm volatile("" ::: "memory");
        }
    }

    // blosclz_decompress (oracle_blosc2.cpp blosclz_dec); returns false on a malformed stream
    __device__ bool blosclz(uint32_t ip) {
        uint32_t ctrl = (uint32_t)(peek8(ip) & 31u);
        ++ip;
        for (;;) {
            if (ctrl >= 32) {
                uint32_t len = (ctrl >> 5) - 1;
                uint32_t ofs = (uint32_t)(ctrl & 31u) << 8;
                if (len == 6) {
                    uint32_t c;
                    do {
                        if (ip + 1 >= end) return false;
                        c = (uint32_t)(peek8(ip) & 255u);
                        ++ip;
                        len += c;
                        if (len > n) return false;   // (32-bit positions: no wrap on hostile input)
                    } while (c == 255);
                } else if (ip + 1 >= end) {
                    return false;
                }
                const uint64_t w = peek8(ip);
                const uint32_t code = (uint32_t)(w & 255u);
                ++ip;
                len += 3;
                uint32_t dist = ofs + code + 1;
                uint32_t nx = (uint32_t)((w >> 8) & 255u);
                if (code == 255 && ofs == (31u << 8)) {
                    if (ip + 1 >= end) return false;
                    ofs = ((w >> 8) & 255u) << 8 | ((w >> 16) & 255u);
                    ip += 2;
                    dist = ofs + 8192;
                    nx = (uint32_t)((w >> 24) & 255u);
                }
                if (op + len > n || dist > op || ip >= end) return false;
                ctrl = nx;
                ++ip;
                match(len, dist);
            } else {
                const uint32_t run = ctrl + 1;
                if (op + run > n || ip + run > end) return false;
                literals(ip, run);
                ip += run;
                if (ip >= end) break;
                ctrl = (uint32_t)(peek8(ip) & 255u);
                ++ip;
            }
        }
        return true;
    }

    // LZ4_decompress_safe (oracle_blosc2.cpp lz4_dec)
    __device__ bool lz4(uint32_t ip) {
        if (ip >= end) return false;
        for (;;) {
            if (ip >= end) return false;
            uint64_t w = peek8(ip);
            const uint32_t token = (uint32_t)(w & 255u);
            ++ip;
            uint32_t L = token >> 4;
            if (L == 15) {
                uint32_t b;
                do {
                    if (ip >= end) return false;
                    b = (uint32_t)(peek8(ip) & 255u);
                    ++ip;
                    L += b;
                    if (L > n) return false;
                } while (b == 255);
            }
            if (end - ip < L || n - op < L) return false;
            literals(ip, L);
            ip += L;
            if (op + 12 > n || ip + 8 > end) {
                if (ip != end) return false;
                break;
            }
            // a short literal run leaves the offset inside the token's 8-byte window: no second LDS trip
            const uint32_t off = (uint32_t)((token >> 4) <= 5 ? (w >> (8 * (1 + (token >> 4)))) & 0xffffu
                                                               : peek8(ip) & 0xffffu);
            ip += 2;
            if (off == 0 || off > op) return false;
            uint32_t M = token & 15u;
            if (M == 15) {
                uint32_t b;
                do {
                    if (ip >= end) return false;
                    b = (uint32_t)(peek8(ip) & 255u);
                    ++ip;
                    M += b;
                    if (M > n) return false;
                } while (b == 255);
            }
            M += 4;
            if (op + M + 5 > n) return false;
            match(M, off);
        }
        return true;
    }

    // Snappy raw block (oracle_blosc2.cpp snappy_dec): varint preamble = the decoded length (must be n:
    // a shorter one is the caller's size error, a longer one does not fit), then tagged elements; every
    // element's fields sit in the tag's 8-byte window (one LDS trip per element).
    __device__ bool snappy(uint32_t ip) {
        uint32_t want = 0;
        {
            const uint64_t w = peek8(ip);
            uint32_t k = 0;
            for (;; ++k) {
                if (k == 5 || ip + k >= end) return false;
                const uint32_t b = (uint32_t)(w >> (8 * k)) & 255u;
                if (k == 4 && b > 15) return false;
                want |= (b & 127u) << (7 * k);
                if (!(b & 128)) break;
            }
            ip += k + 1;
        }
        if (want > n) return false;
        while (ip < end) {
            const uint64_t w = peek8(ip);
            const uint32_t tag = (uint32_t)(w & 255u);
            uint32_t len, off;
            if ((tag & 3) == 0) {
                len = tag >> 2;
                uint32_t hb = 1;
                if (len >= 60) {
                    const uint32_t nb = len - 59;
                    if (ip + 1 + nb > end) return false;
                    len = (uint32_t)(w >> 8) & (nb == 4 ? 0xffffffffu : (1u << (8 * nb)) - 1);
                    if (len == 0xffffffffu) return false;
                    hb += nb;
                }
                len += 1;
                ip += hb;
                if (end - ip < len || want - op < len) return false;
                literals(ip, len);
                ip += len;
                continue;
            }
            if ((tag & 3) == 1) {
                if (ip + 2 > end) return false;
                len = 4 + ((tag >> 2) & 7u);
                off = (tag >> 5) << 8 | ((uint32_t)(w >> 8) & 255u);
                ip += 2;
            } else if ((tag & 3) == 2) {
                if (ip + 3 > end) return false;
                len = (tag >> 2) + 1;
                off = (uint32_t)(w >> 8) & 0xffffu;
                ip += 3;
            } else {
                if (ip + 5 > end) return false;
                len = (tag >> 2) + 1;
                off = (uint32_t)(w >> 8);
                ip += 5;
            }
            if (off == 0 || off > op || want - op < len) return false;
            match(len, off);
        }
        return op == want;
    }
};
using LzStream = LzStreamT<kRing>;

// ---- zstd (codec 4): RFC 8878, restated from oracle/oracle_zstd.cpp -------------------------------------
// One wavefront per zstd-coded stream (a row of the stream table, rows [z_capacity, z_capacity + count)),
// in its own launch (k_blosc2_zstd) with its own LDS: the decode tables beside the output ring.  Control
// is wave-uniform scalar code; the compressed bytes are read through 256-byte windows held one dword per
// lane (v_readlane extracts the dword a bit read needs; a window reload is one coalesced load), so no bit
// read waits on memory except at a window boundary.  Literals are Huffman-decoded into the tail of the
// stream's own output region (bytes the sequences have not reached yet: the write position never passes the
// read position) and copied from there by the sequences through LzStream's staged input ring; matches use
// LzStream's LDS window / flushed-output reads.  Frames with a content checksum are not decoded here
// (RDX_BLOSC2_UNSUPPORTED: the host decodes that chunk); neither are dictionaries (a failure, as libzstd).
constexpr uint32_t kZHufMax = 11;   // Max_Number_of_Bits

// Probe builds: per-row phase cycles of k_blosc2_zstd (s_memtime) and event counts, read back by
// rdx_probe_zprof_read: [0] row total, [1] literals section, [2] sequence tables, [3] sequence loop,
// [4] of which literal copies, [5] of which match copies, [6] sequences, [7] far match steps,
// [8] literal bytes (regenerated), [9] match bytes, [10] ring flushes, [11] compressed blocks.
#if RDX_PROBES
constexpr uint32_t kZProfRows = 4096, kZProfK = 12;
static __device__ uint64_t g_zprof[kZProfRows * kZProfK];
#define ZP_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ZP_ADD(k, v) prof[k] += __builtin_amdgcn_s_memtime() - (v)
#define ZP_CNT(k, x) prof[k] += (x)
#else
#define ZP_T(v) \
    do {        \
    } while (0)
#define ZP_ADD(k, v) \
    do {             \
    } while (0)
#define ZP_CNT(k, x) \
    do {             \
    } while (0)
#endif

// zstd waves: a 4 KiB output ring (matches farther back read the flushed output from HBM) and two waves per
// workgroup, so the LDS (15.6 KiB per wave) admits 10 waves per CU instead of 8
#ifndef RDX_ZRING
#define RDX_ZRING 4096
#endif
#ifndef RDX_ZWAVES
#define RDX_ZWAVES 2
#endif
#ifndef RDX_ZWPE
#define RDX_ZWPE 3
#endif
constexpr uint32_t kZRing = RDX_ZRING, kZWaves = RDX_ZWAVES;

struct __attribute__((aligned(16))) ZLds {
    WaveLdsT<kZRing> w;                                  // output ring + staged literal source
    uint32_t ll[512], of[256], ml[512];          // FSE decode entries: symbol | nb << 8 | base << 16
    uint32_t wt[64];                             // the FSE table of the Huffman weights (accuracy <= 6)
    uint16_t huf[1 << kZHufMax];                 // Huffman: symbol | nb << 8
};

__constant__ int16_t kZLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
                                    -1, -1, -1, -1};
__constant__ int16_t kZMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kZOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t kZLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,  12,   13,   14,   15,   16,    18,
                                      20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kZLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kZMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,  16,   17,   18,   19,   20,
                                      21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,  34,   35,   37,   39,   41,
                                      43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kZMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                     0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

__device__ __forceinline__ uint32_t zhibit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

// 64 dwords of a byte range, one per lane; bit reads take their dwords with v_readlane (uniform index)
struct ZWin {
    const uint32_t *w;
    uint32_t nw, lane;
    int32_t wd0;
    uint32_t v;
    __device__ __forceinline__ void load(int32_t d0) {
        wd0 = d0;
        const int32_t d = d0 + (int32_t)lane;
        v = (d >= 0 && (uint32_t)d < nw) ? gld<uint32_t>(w + d) : 0u;
    }
    __device__ __forceinline__ uint32_t dw(int32_t d, bool back) {
        if (d < wd0 || d >= wd0 + 64) load(back ? (d > 61 ? d - 61 : 0) : d);
        return __builtin_amdgcn_readlane(v, (int)rfl((uint32_t)(d - wd0)));
    }
};

// Bits of a byte range [p, p + n): forward (FSE descriptions, header bytes) or backward (RFC 8878 §4.1
// bitstreams: from the end, the last byte's highest set bit is padding; bits below the start read as 0
// and `off` goes negative, which the callers check).
struct ZBits {
    ZWin win;
    uint32_t sb;       // skew bits
    uint64_t nbytes;
    int64_t off;       // backward: bits left; forward: next bit
    __device__ __forceinline__ void setup(const uint8_t *p, uint64_t n, uint32_t lane) {
        const uint32_t skew = (uint32_t)((uintptr_t)p & 3);
        win.w = reinterpret_cast<const uint32_t *>(p - skew);
        win.nw = (uint32_t)((skew + n + 3) / 4);
        win.lane = lane;
        win.wd0 = -1000;
        win.v = 0;
        sb = 8 * skew;
        nbytes = n;
        off = 0;
    }
    // k (<= 32) bits at relative bit position r (>= 0)
    __device__ __forceinline__ uint32_t at(uint64_t r, uint32_t k, bool back) {
        const uint64_t a = sb + r;
        const int32_t d = (int32_t)(a >> 5);
        const uint32_t sh = (uint32_t)(a & 31);
        uint32_t v = win.dw(d, back) >> sh;
        if (sh + k > 32) v |= win.dw(d + 1, back) << (32 - sh);
        return k >= 32 ? v : v & ((1u << k) - 1);
    }
    __device__ __forceinline__ uint32_t byte(uint64_t i) { return at(8 * i, 8, false); }
    __device__ __forceinline__ bool init_back(const uint8_t *p, uint64_t n, uint32_t lane) {
        setup(p, n, lane);
        if (n == 0) return false;
        const uint32_t last = at(8 * (n - 1), 8, true);
        if (last == 0) return false;
        off = (int64_t)(8 * n) - (int64_t)(8 - zhibit(last));
        return true;
    }
    __device__ __forceinline__ uint32_t get(uint32_t k) {   // backward, k <= 32
        if (k == 0) return 0;
        off -= k;
        if (off >= 0) return at((uint64_t)off, k, true);
        const int64_t avail = (int64_t)k + off;
        if (avail <= 0) return 0;
        return at(0, (uint32_t)avail, true) << (uint32_t)(-off);
    }
    __device__ __forceinline__ uint32_t fwd(uint32_t k, bool &ok) {   // forward, k <= 25
        if ((uint64_t)off + k > 8 * nbytes) {
            ok = false;
            return 0;
        }
        const uint32_t v = at((uint64_t)off, k, false);
        off += k;
        return v;
    }
};

// Backward reader with a 64-bit container (the sequence section): c holds the stream's bits [cb - 64, cb),
// bits below the stream start reading as 0.  A field comes out of the container with 64-bit shifts; a
// refill (every ~57 bits) reads three dwords of a 256-byte LDS window of the stream (the Huffman weights'
// table area, free once the literals are decoded), which the wave restages when the read position leaves it.
struct ZBitC {
    ZBits b;   // init_back only; b.off = the read position (bits left), negative once overread
    uint64_t c;
    int64_t cb;
    const uint8_t *sp;   // the stream [sp, sp + sn)
    uint32_t sn;
    uint32_t *lw;        // LDS: stream bytes [wb, wb + 256)
    int32_t wb;
    __device__ __forceinline__ void setup(const uint8_t *p, uint32_t n, uint32_t *lds) {
        sp = p;
        sn = n;
        lw = lds;
        wb = 1 << 30;   // nothing staged
    }
    __device__ __forceinline__ void stage(int32_t B) {
        const int32_t nw = B - 240;
        wb = (nw > 0 ? nw : 0) & ~3;
        const uint32_t lane = b.win.lane;
        const uint8_t *a = sp + wb;
        const uint32_t sk = (uint32_t)((uintptr_t)a & 3);
        const uint32_t *aw = reinterpret_cast<const uint32_t *>(a - sk) + lane;
        const uintptr_t lo_w = (uintptr_t)sp & ~(uintptr_t)3, hi_b = (uintptr_t)(sp + sn);
        const uint32_t w0 = (uintptr_t)aw >= lo_w && (uintptr_t)aw < hi_b ? gld<uint32_t>(aw) : 0u;
        const uint32_t w1 = (uintptr_t)(aw + 1) >= lo_w && (uintptr_t)(aw + 1) < hi_b ? gld<uint32_t>(aw + 1) : 0u;
        lw[lane] = sk ? __builtin_amdgcn_alignbyte(w1, w0, sk) : w0;
        wave_sync();
    }
    // bytes [B, B + 8) of the stream, B >= 0
    __device__ __forceinline__ uint64_t read8(int64_t B64) {
        const int32_t B = (int32_t)B64;
        if (B < wb || B + 12 > wb + 256) stage(B);
        const uint32_t rel = (uint32_t)(B - wb), i = rel >> 2, sh = (rel & 3) * 8;
        const uint64_t w01 = (uint64_t)lw[i] | (uint64_t)lw[i + 1] << 32;
        if (!sh) return w01;
        return (w01 >> sh) | (uint64_t)lw[i + 2] << (64 - sh);
    }
    __device__ __forceinline__ void refill() {
        const int64_t nb = (b.off + 7) >> 3;   // c = bytes [nb - 8, nb)
        cb = 8 * nb;
        const int64_t B = nb - 8;
        if (B >= 0) c = read8(B);
        else if (B > -8) c = read8(0) << (8 * (uint32_t)(-B));
        else c = 0;
    }
    __device__ __forceinline__ uint32_t get(uint32_t k) {   // k <= 32
        if (k == 0) return 0;
        if (b.off - (int64_t)k < cb - 64) refill();
        b.off -= k;
        const uint32_t v = (uint32_t)(c >> (uint32_t)(b.off - (cb - 64)));
        return k >= 32 ? v : v & ((1u << k) - 1u);
    }
};

// weight wv of symbol s into lane s % 64 of w[s / 64]
__device__ __forceinline__ void zput(uint32_t lane, uint32_t s, uint32_t wv, uint32_t &w0, uint32_t &w1, uint32_t &w2,
                                     uint32_t &w3) {
    const uint32_t k = s >> 6;
    if (lane == (s & 63)) {
        if (k == 0) w0 = wv;
        else if (k == 1) w1 = wv;
        else if (k == 2) w2 = wv;
        else w3 = wv;
    }
}

struct ZDec {
    ZLds &Z;
    LzStreamT<kZRing> z;   // by value (a reference member kept the stream in scratch and its LDS accesses flat)
    const uint32_t lane;
    bool have_huf = false, have_ll = false, have_of = false, have_ml = false;
    bool pre_ll = false, pre_of = false, pre_ml = false;   // the LDS table holds the predefined distribution
    uint32_t huf_bits = 0, ll_log = 0, of_log = 0, ml_log = 0;
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
#if RDX_PROBES
    uint64_t prof[kZProfK] = {};
#endif

    // FSE decode table from a per-lane distribution (lane s: symbol s's normalised count; nsym <= 64):
    // the spread by one lane's LDS stores, then the states' bits / baselines in order with the per-symbol
    // counters in a VGPR (lane s), entries assembled in VGPRs and stored coalesced.
    __device__ __forceinline__ bool fse_build(uint32_t *tab, int freq_v, uint32_t nsym, uint32_t log) {
        const uint32_t size = 1u << log;
        uint32_t high = size;
        for (uint32_t s = 0; s < nsym; ++s) {
            if ((int)__builtin_amdgcn_readlane(freq_v, (int)s) == -1) {
                --high;
                if (lane == 0) tab[high] = s;
            }
        }
        const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
        uint32_t pos = 0;
        for (uint32_t s = 0; s < nsym; ++s) {
            const int f = (int)__builtin_amdgcn_readlane(freq_v, (int)s);
            for (int i = 0; i < f; ++i) {
                if (lane == 0) tab[pos] = s;
                do pos = (pos + step) & mask;
                while (pos >= high);
            }
        }
        if (pos != 0) return false;
        wave_sync();
        uint32_t cnt = lane < nsym ? (freq_v == -1 ? 1u : (freq_v > 0 ? (uint32_t)freq_v : 0u)) : 0u;
        for (uint32_t j = 0; j * 64 < size; ++j) {
            const uint32_t c = j * 64 + lane;
            const uint32_t symv = c < size ? (tab[c] & 0xffu) : 0u;
            uint32_t e = 0;
            const uint32_t m = size - j * 64 < 64 ? size - j * 64 : 64;
            for (uint32_t l = 0; l < m; ++l) {
                const uint32_t sym = __builtin_amdgcn_readlane(symv, (int)l);
                const uint32_t d = __builtin_amdgcn_readlane(cnt, (int)sym);
                cnt += lane == sym ? 1u : 0u;
                const uint32_t nb = log - zhibit(d);
                const uint32_t base = ((d << nb) - size) & 0xffffu;
                if (lane == l) e = sym | nb << 8 | base << 16;
            }
            wave_sync();
            if (c < size) tab[c] = e;
        }
        wave_sync();
        return true;
    }

    // FSE table description (forward bits at b.off); symbols <= max_sym (< 64), accuracy <= max_log.
    __device__ __forceinline__ bool fse_read(ZBits &b, uint32_t *tab, uint32_t max_log, uint32_t max_sym, uint32_t &log_out) {
        bool ok = true;
        const uint32_t log = 5 + b.fwd(4, ok);
        if (!ok || log > max_log) return false;
        int remaining = 1 << log;
        int freq_v = 0;
        uint32_t s = 0;
        while (remaining > 0 && s <= max_sym) {
            const uint32_t bits = zhibit((uint32_t)remaining + 1) + 1;
            uint32_t v = b.fwd(bits, ok);
            if (!ok) return false;
            const uint32_t lower = (1u << (bits - 1)) - 1;
            const uint32_t thr = (1u << bits) - 1 - ((uint32_t)remaining + 1);
            if ((v & lower) < thr) {
                b.off -= 1;
                v &= lower;
            } else if (v > lower) {
                v -= thr;
            }
            const int pr = (int)v - 1;
            remaining -= pr < 0 ? -pr : pr;
            if (lane == s) freq_v = pr;
            ++s;
            if (pr == 0) {
                uint32_t rep = b.fwd(2, ok);
                for (;;) {
                    if (!ok) return false;
                    for (uint32_t i = 0; i < rep; ++i) {
                        if (s > max_sym) return false;
                        if (lane == s) freq_v = 0;
                        ++s;
                    }
                    if (rep != 3) break;
                    rep = b.fwd(2, ok);
                }
            }
        }
        if (remaining != 0 || s > max_sym + 1) return false;
        b.off = (b.off + 7) & ~(int64_t)7;   // the description ends on a byte boundary
        log_out = log;
        return fse_build(tab, freq_v, s, log);
    }

    // Huffman tree description at stream bytes [p, p + n) -> Z.huf; returns the bytes used (0: corrupt)
    __device__ __forceinline__ uint32_t huf_read(const uint8_t *p, uint64_t n) {
        ZBits h;
        h.setup(p, n, lane);
        if (n < 1) return 0;
        const uint32_t hdr = h.byte(0);
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;   // weight of symbol 64k + lane in wk
        uint32_t nw = 0, used;
#define put(s_, wv_) zput(lane, (s_), (wv_), w0, w1, w2, w3)
        if (hdr >= 128) {
            nw = hdr - 127;
            const uint32_t bytes = (nw + 1) / 2;
            if (1 + bytes > n) return 0;
            for (uint32_t i = 0; i < nw; ++i) {
                const uint32_t by = h.byte(1 + i / 2);
                put(i, (i % 2 == 0) ? by >> 4 : by & 15u);
            }
            used = 1 + bytes;
        } else {
            if (hdr == 0 || 1 + (uint64_t)hdr > n) return 0;
            ZBits f;
            f.setup(p + 1, hdr, lane);
            uint32_t log = 0;
            if (!fse_read(f, Z.wt, 6, 63, log)) return 0;
            const uint64_t th = (uint64_t)f.off / 8;
            if (th >= hdr) return 0;
            ZBits b;
            if (!b.init_back(p + 1 + th, hdr - th, lane)) return 0;
            uint32_t s1 = b.get(log), s2 = b.get(log);
            if (b.off < 0) return 0;
            for (;;) {
                uint32_t e = rfl(Z.wt[s1]);
                if (nw >= 255) return 0;
                put(nw++, e & 0xffu);
                s1 = (e >> 16) + b.get((e >> 8) & 0xffu);
                if (b.off < 0) {
                    if (nw >= 255) return 0;
                    put(nw++, rfl(Z.wt[s2]) & 0xffu);
                    break;
                }
                e = rfl(Z.wt[s2]);
                if (nw >= 255) return 0;
                put(nw++, e & 0xffu);
                s2 = (e >> 16) + b.get((e >> 8) & 0xffu);
                if (b.off < 0) {
                    if (nw >= 255) return 0;
                    put(nw++, rfl(Z.wt[s1]) & 0xffu);
                    break;
                }
            }
            used = 1 + hdr;
        }
        // the implied last weight, Max_Number_of_Bits
        const uint32_t ws[4] = {w0, w1, w2, w3};
        uint32_t total = 0, bad = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t wv = (64u * k + lane) < nw ? ws[k] : 0u;
            bad |= wv > kZHufMax;
            uint32_t t = wv ? 1u << (wv - 1) : 0u;
            for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m, 64);
            total += t;
        }
        if (__builtin_amdgcn_ballot_w64(bad) || total == 0) return 0;
        total = rfl(total);
        const uint32_t maxbits = zhibit(total) + 1;
        if (maxbits > kZHufMax) return 0;
        const uint32_t rest = (1u << maxbits) - total;
        if (rest & (rest - 1)) return 0;
        put(nw++, zhibit(rest) + 1);
        if (nw > 256) return 0;
        // ranges by weight ascending, symbols in order: a per-weight start (lane wt) from the counts
        uint32_t start = 0;   // lane wt: first entry of weight wt
        {
            uint32_t acc = 0;
            for (uint32_t wt = 1; wt <= maxbits; ++wt) {
                uint32_t c = 0;
                const uint32_t ws2[4] = {w0, w1, w2, w3};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    c += __builtin_popcountll(__builtin_amdgcn_ballot_w64((64u * k + lane) < nw && ws2[k] == wt));
                if (lane == wt) start = acc;
                acc += c << (wt - 1);
            }
            if (acc != (1u << maxbits)) return 0;
        }
        const uint32_t wsf[4] = {w0, w1, w2, w3};
        for (uint32_t sidx = 0; sidx < nw; ++sidx) {
            const uint32_t k = sidx >> 6;
            const uint32_t wv = __builtin_amdgcn_readlane(k == 0 ? wsf[0] : k == 1 ? wsf[1] : k == 2 ? wsf[2] : wsf[3],
                                                          (int)(sidx & 63));
            if (wv == 0) continue;
            const uint32_t at = __builtin_amdgcn_readlane(start, (int)wv);
            const uint32_t len = 1u << (wv - 1);
            if (lane == wv) start += len;
            const uint16_t ent = (uint16_t)(sidx | (maxbits + 1 - wv) << 8);
            for (uint32_t q = lane; q < len; q += 64) Z.huf[at + q] = ent;
        }
        wave_sync();
        huf_bits = maxbits;
        have_huf = true;
        return used;
#undef put
    }

    // Huffman literal streams, decoded SIMT-style: 1X in lane 0, 4X in lanes 0-3 (stream k in lane k, one
    // symbol of each per step).  Each lane keeps its own backward bit position and reads its stream from a
    // 512-byte LDS window (its quarter of the staged-input area, which the sequences restage afterwards);
    // the whole wave restages the windows when any lane's next read would fall below its own.  Table reads
    // are per-lane LDS gathers, symbols per-lane byte stores.  (The first form ran one wave-uniform bit
    // reader per stream in scalar code: ~500 cycles per literal byte, profiles/r03_zstd_phase_probe.jsonl.)
    // Stream k is [d + o_k, d + o_k + n_k) with o_k the sum of the lengths before it; it yields `seg`
    // symbols (stream 3 of 4X: `last`), consumed exactly.
    __device__ __forceinline__ bool huf_lanes(const uint8_t *d, uint32_t ns, uint32_t s1, uint32_t s2, uint32_t s3,
                                              uint32_t s4, uint8_t *dst, uint32_t seg, uint32_t last) {
        const uint32_t k = lane & 3;
        const bool mine = lane < ns;
        const uint32_t o_k = k == 0 ? 0u : k == 1 ? s1 : k == 2 ? s1 + s2 : s1 + s2 + s3;
        const uint32_t n_k = k == 0 ? s1 : k == 1 ? s2 : k == 2 ? s3 : s4;
        const uint32_t cnt = !mine ? 0u : (ns == 1 || k < 3 ? seg : last);
        bool bad = false;
        int32_t pos = 0;
        if (mine) {   // below the last byte's highest set bit
            const uint32_t lb = n_k ? (uint32_t)gld<uint8_t>(d + o_k + n_k - 1) : 0u;
            if (lb == 0) bad = true;
            else pos = (int32_t)(8 * n_k) - (int32_t)(8 - zhibit(lb));
        }
        if (__builtin_amdgcn_ballot_w64(bad)) return false;
        const uint32_t mb = rfl(huf_bits);
        uint32_t *win = Z.w.in;   // stream k: words [128 k, 128 k + 128) = stream bytes [wb, wb + 512)
        int32_t wb = 1 << 30;     // nothing staged yet
        uint8_t *out = dst + (uint64_t)k * seg;
        const uint32_t q = lane >> 4, j = lane & 15;   // restaging: lane copies 32 B of stream q's window
        const uint32_t o_q = q == 0 ? 0u : q == 1 ? s1 : q == 2 ? s1 + s2 : s1 + s2 + s3;
        const uint32_t n_q = q == 0 ? s1 : q == 1 ? s2 : q == 2 ? s3 : s4;
        const uintptr_t lo_w = (uintptr_t)(d + o_q) & ~(uintptr_t)3, hi_b = (uintptr_t)(d + o_q + n_q);
        for (uint32_t i = 0; i < seg; ++i) {
            const bool act = i < cnt;
            const int32_t p = pos - (int32_t)mb, pc = p > 0 ? p : 0;
            if (__builtin_amdgcn_ballot_w64(act && (pc >> 3) < wb)) {
                if (mine) {
                    const int32_t nwb = ((pos + 7) >> 3) - 500;
                    wb = (nwb > 0 ? nwb : 0) & ~3;
                }
                const int32_t wq = __shfl(wb, (int)q, 64);
                if (q < ns) {
                    const uint8_t *a = d + o_q + wq + 32 * j;
                    const uint32_t skew = (uint32_t)((uintptr_t)a & 3);
                    const uint32_t *aw = reinterpret_cast<const uint32_t *>(a - skew);
                    uint32_t w[9];
#pragma unroll
                    for (int t = 0; t < 9; ++t) {
                        const uintptr_t ad = (uintptr_t)(aw + t);
                        w[t] = ad >= lo_w && ad < hi_b ? gld<uint32_t>(aw + t) : 0u;
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t)
                        win[128 * q + 8 * j + t] = skew ? __builtin_amdgcn_alignbyte(w[t + 1], w[t], skew) : w[t];
                }
                wave_sync();
            }
            if (act) {
                const uint32_t wi = (uint32_t)((pc >> 3) - wb) >> 2;
                const uint64_t qv = (uint64_t)win[128 * k + wi + 1] << 32 | win[128 * k + wi];
                const uint32_t sh = (uint32_t)(pc - 8 * (wb + 4 * (int32_t)wi));
                const uint32_t nbits = (uint32_t)(pos - pc);   // mb, or what is left near the stream start
                const uint32_t v = ((uint32_t)(qv >> sh) & ((1u << nbits) - 1u)) << (uint32_t)(pc - p);
                const uint32_t e = Z.huf[v];
                pos -= (int32_t)(e >> 8);
                bad |= pos < 0;
                gst<uint8_t>(out + i, (uint8_t)e);
            }
            if (__builtin_amdgcn_ballot_w64(bad)) return false;
        }
        return __builtin_amdgcn_ballot_w64(mine && pos != 0) == 0;
    }

    // a sequence table: mode 0 predefined, 1 RLE, 2 FSE, 3 repeat; bytes used at p (or -1)
    __device__ __forceinline__ int64_t seq_table(uint32_t mode, const uint8_t *p, uint64_t n, uint32_t *tab, uint32_t &log, bool &have,
                                 bool &predef, const int16_t *def, uint32_t ndef, uint32_t deflog, uint32_t maxlog,
                                 uint32_t maxsym) {
        if (mode == 0) {
            if (!predef) {   // (the table keeps the predefined distribution until another mode replaces it)
                const int fv = lane < ndef ? (int)def[lane] : 0;
                if (!fse_build(tab, fv, ndef, deflog)) return -1;
                predef = true;
            }
            log = deflog;
            have = true;
            return 0;
        }
        if (mode != 3) predef = false;
        if (mode == 1) {
            if (n < 1) return -1;
            ZBits h;
            h.setup(p, n, lane);
            const uint32_t sym = h.byte(0);
            if (sym > maxsym) return -1;
            if (lane == 0) tab[0] = sym;   // nb 0, base 0
            wave_sync();
            log = 0;
            have = true;
            return 1;
        }
        if (mode == 2) {
            ZBits f;
            f.setup(p, n, lane);
            if (!fse_read(f, tab, maxlog, maxsym, log)) return -1;
            have = true;
            return f.off / 8;
        }
        return have ? 0 : -1;
    }

    // A compressed block [p, p + n): output appended at z.op; frame output started at fstart
    __device__ __forceinline__ bool compressed_block(const uint8_t *p, uint64_t n, uint64_t fstart) {
        ZBits h;
        h.setup(p, n, lane);
        if (n < 1) return false;
        const uint32_t b0 = h.byte(0);
        const uint32_t ltype = b0 & 3, sf = (b0 >> 2) & 3;
        uint64_t regen, csize = 0, hl;
        uint32_t nstreams = 1;
        if (ltype <= 1) {
            if (sf == 0 || sf == 2) {
                regen = b0 >> 3;
                hl = 1;
            } else if (sf == 1) {
                if (n < 2) return false;
                regen = (b0 >> 4) + ((uint64_t)h.byte(1) << 4);
                hl = 2;
            } else {
                if (n < 3) return false;
                regen = (b0 >> 4) + ((uint64_t)h.byte(1) << 4) + ((uint64_t)h.byte(2) << 12);
                hl = 3;
            }
        } else {
            if (sf <= 1) {
                if (n < 3) return false;
                const uint32_t v = b0 | h.byte(1) << 8 | h.byte(2) << 16;
                regen = (v >> 4) & 0x3FF;
                csize = (v >> 14) & 0x3FF;
                hl = 3;
                nstreams = sf == 0 ? 1 : 4;
            } else if (sf == 2) {
                if (n < 4) return false;
                const uint32_t v = b0 | h.byte(1) << 8 | h.byte(2) << 16 | h.byte(3) << 24;
                regen = (v >> 4) & 0x3FFF;
                csize = (v >> 18) & 0x3FFF;
                hl = 4;
                nstreams = 4;
            } else {
                if (n < 5) return false;
                const uint64_t v = (uint64_t)(b0 | h.byte(1) << 8 | h.byte(2) << 16 | h.byte(3) << 24) |
                                   (uint64_t)h.byte(4) << 32;
                regen = (v >> 4) & 0x3FFFF;
                csize = (v >> 22) & 0x3FFFF;
                hl = 5;
                nstreams = 4;
            }
        }
        if (regen > (128u << 10)) return false;
        // literals: raw ones stay in the input; decoded ones go to the tail of the output region
        const uint8_t *lit = nullptr;
        uint64_t q = hl;
        ZP_T(t_lit);
        ZP_CNT(8, regen);
        ZP_CNT(11, 1);
        if (regen > (uint64_t)z.n - z.op) return false;
        uint8_t *tail = z.dst + z.n - regen;
        if (ltype == 0) {
            if (q + regen > n) return false;
            lit = p + q;
            q += regen;
        } else if (ltype == 1) {
            if (q + 1 > n) return false;
            wave_fill(tail, regen, (uint8_t)h.byte(q));
            lit = tail;
            q += 1;
        } else {
            if (q + csize > n) return false;
            const uint8_t *ls = p + q;
            uint64_t lp = 0;
            if (ltype == 2) {
                lp = huf_read(ls, csize);
                if (lp == 0) return false;
            } else if (!have_huf) {
                return false;
            }
            if (lp > csize) return false;
            if (nstreams == 1) {
                if (!huf_lanes(ls + lp, 1, (uint32_t)(csize - lp), 0, 0, 0, tail, (uint32_t)regen, 0)) return false;
            } else {
                if (csize - lp < 10 || regen < 6) return false;
                ZBits jt;
                jt.setup(ls + lp, 6, lane);
                const uint64_t s1 = jt.byte(0) | jt.byte(1) << 8, s2 = jt.byte(2) | jt.byte(3) << 8,
                               s3 = jt.byte(4) | jt.byte(5) << 8;
                const uint64_t total = csize - lp - 6;
                if (s1 + s2 + s3 > total) return false;
                const uint64_t s4 = total - s1 - s2 - s3, seg = (regen + 3) / 4;
                if (!huf_lanes(ls + lp + 6, 4, (uint32_t)s1, (uint32_t)s2, (uint32_t)s3, (uint32_t)s4, tail, (uint32_t)seg,
                               (uint32_t)(regen - 3 * seg)))
                    return false;
            }
            lit = tail;
            q += csize;
        }
        if (lit == tail) {   // the decoded literals are read back below (through L2, not a stale L1 line)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        const uint32_t lip = regen ? z.source(lit, (uint32_t)regen) : 0;
        ZP_ADD(1, t_lit);
        // sequences
        if (q >= n) return false;
        uint64_t nseq = h.byte(q++);
        if (nseq >= 128) {
            if (nseq < 255) {
                if (q >= n) return false;
                nseq = ((nseq - 128) << 8) + h.byte(q++);
            } else {
                if (q + 2 > n) return false;
                nseq = h.byte(q) + ((uint64_t)h.byte(q + 1) << 8) + 0x7F00;
                q += 2;
            }
        }
        uint64_t lpos = 0;
        if (nseq > 0) {
            if (q >= n) return false;
            const uint32_t modes = h.byte(q++);
            if (modes & 3) return false;
            ZP_T(t_tab);
            int64_t u = seq_table(modes >> 6, p + q, n - q, Z.ll, ll_log, have_ll, pre_ll, kZLLDef, 36, 6, 9, 35);
            if (u < 0) return false;
            q += (uint64_t)u;
            u = seq_table((modes >> 4) & 3, p + q, n - q, Z.of, of_log, have_of, pre_of, kZOFDef, 29, 5, 8, 31);
            if (u < 0) return false;
            q += (uint64_t)u;
            u = seq_table((modes >> 2) & 3, p + q, n - q, Z.ml, ml_log, have_ml, pre_ml, kZMLDef, 53, 6, 9, 52);
            if (u < 0) return false;
            q += (uint64_t)u;
            if (q >= n) return false;
            ZP_ADD(2, t_tab);
            ZP_T(t_seq);
            ZP_CNT(6, nseq);
            ZBitC b;
            if (!b.b.init_back(p + q, n - q, lane)) return false;
            b.setup(p + q, (uint32_t)(n - q), Z.wt);
            b.refill();
            uint32_t sll = b.get(ll_log), sof = b.get(of_log), sml = b.get(ml_log);
            for (uint64_t i = 0; i < nseq; ++i) {
                // the three table reads issued together (the scheduler otherwise waits on each before the next)
                const uint32_t rll = Z.ll[sll], rof = Z.of[sof], rml = Z.ml[sml];
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t ell = rfl(rll), eof = rfl(rof), eml = rfl(rml);
                const uint32_t ofc = eof & 0xffu, mlc = eml & 0xffu, llc = ell & 0xffu;
                if (ofc > 31 || mlc > 52 || llc > 35) return false;
                uint64_t ofv = (1ull << ofc);
                if (ofc > 16) {   // (get() takes <= 32 bits; split the widest offsets)
                    const uint64_t hi = b.get(ofc - 16);
                    ofv += (hi << 16) | b.get(16);
                } else {
                    ofv += b.get(ofc);
                }
                const uint64_t ml = kZMLBase[mlc] + b.get(kZMLBits[mlc]);
                const uint64_t ll = kZLLBase[llc] + b.get(kZLLBits[llc]);
                uint64_t off;
                if (ofv > 3) {
                    off = ofv - 3;
                    rep2 = rep1;
                    rep1 = rep0;
                    rep0 = (uint32_t)off;
                } else {
                    const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0 ? 1u : 0u);
                    if (idx == 0) {
                        off = rep0;
                    } else if (idx == 3) {
                        off = (uint64_t)rep0 - 1;
                        if (off == 0) return false;
                        rep2 = rep1;
                        rep1 = rep0;
                        rep0 = (uint32_t)off;
                    } else {
                        off = idx == 1 ? rep1 : rep2;
                        if (idx == 2) rep2 = rep1;
                        rep1 = rep0;
                        rep0 = (uint32_t)off;
                    }
                }
                if (i + 1 < nseq) {   // state updates: literal lengths, match lengths, offsets
                    sll = (ell >> 16) + b.get((ell >> 8) & 0xffu);
                    sml = (eml >> 16) + b.get((eml >> 8) & 0xffu);
                    sof = (eof >> 16) + b.get((eof >> 8) & 0xffu);
                }
                if (b.b.off < 0) return false;
                if (ll > regen - lpos || ll > (uint64_t)z.n - z.op) return false;
                ZP_T(t_l);
                if (ll) z.literals(lip + (uint32_t)lpos, (uint32_t)ll);
                ZP_ADD(4, t_l);
                lpos += ll;
                if (off > (uint64_t)z.op - fstart || ml > (uint64_t)z.n - z.op) return false;
                ZP_T(t_m);
                z.match((uint32_t)ml, (uint32_t)off);
                ZP_ADD(5, t_m);
                ZP_CNT(9, ml);
                ZP_CNT(7, off > kZRing - 64 ? (ml + 63) / 64 : 0);
            }
            ZP_ADD(3, t_seq);
            if (b.b.off != 0) return false;
        } else if (q != n) {
            return false;
        }
        const uint64_t rest = regen - lpos;
        if (rest > (uint64_t)z.n - z.op) return false;
        if (rest) z.literals(lip + (uint32_t)lpos, (uint32_t)rest);
        return true;
    }

    // ZSTD_decompressDCtx over [p, p + n) into z (capacity z.n): 0, RDX_BLOSC2_FAILED or _UNSUPPORTED
    __device__ __forceinline__ uint32_t stream(const uint8_t *p, uint64_t n) {
        ZBits h;
        h.setup(p, n, lane);
        uint64_t q = 0;
        if (n == 0) return RDX_BLOSC2_FAILED;
        while (q < n) {
            if (q + 4 > n) return RDX_BLOSC2_FAILED;
            const uint32_t magic = h.byte(q) | h.byte(q + 1) << 8 | h.byte(q + 2) << 16 | h.byte(q + 3) << 24;
            if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {   // skippable frame
                if (q + 8 > n) return RDX_BLOSC2_FAILED;
                const uint64_t sz = h.byte(q + 4) | h.byte(q + 5) << 8 | h.byte(q + 6) << 16 | (uint64_t)h.byte(q + 7) << 24;
                if (q + 8 + sz > n) return RDX_BLOSC2_FAILED;
                q += 8 + sz;
                continue;
            }
            if (magic != 0xFD2FB528u) return RDX_BLOSC2_FAILED;
            q += 4;
            if (q >= n) return RDX_BLOSC2_FAILED;
            const uint32_t fhd = h.byte(q++);
            const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
            if (fhd & 0x08) return RDX_BLOSC2_FAILED;
            uint64_t window = 0;
            if (!single) {
                if (q >= n) return RDX_BLOSC2_FAILED;
                const uint32_t wd = h.byte(q++);
                const uint64_t wlog = 10 + (wd >> 3);
                if (wlog > 27) return RDX_BLOSC2_FAILED;
                const uint64_t wbase = 1ull << wlog;
                window = wbase + (wbase / 8) * (wd & 7);
            }
            const uint32_t did_bytes = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
            if (q + did_bytes > n) return RDX_BLOSC2_FAILED;
            uint64_t did = 0;
            for (uint32_t k = 0; k < did_bytes; ++k) did |= (uint64_t)h.byte(q + k) << (8 * k);
            q += did_bytes;
            if (did != 0) return RDX_BLOSC2_FAILED;
            const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
            if (q + fcs_bytes > n) return RDX_BLOSC2_FAILED;
            uint64_t fcs = 0;
            for (uint32_t k = 0; k < fcs_bytes; ++k) fcs |= (uint64_t)h.byte(q + k) << (8 * k);
            if (fcs_bytes == 2) fcs += 256;
            q += fcs_bytes;
            if (single) window = fcs;
            if (checksum) return RDX_BLOSC2_UNSUPPORTED;   // XXH64 of the output: decoded on the host
            const uint64_t bmax = window < (128u << 10) ? window : (128u << 10);
            const uint64_t fstart = z.op;
            have_huf = have_ll = have_of = have_ml = false;
            rep0 = 1;
            rep1 = 4;
            rep2 = 8;
            for (;;) {
                if (q + 3 > n) return RDX_BLOSC2_FAILED;
                const uint32_t bh = h.byte(q) | h.byte(q + 1) << 8 | h.byte(q + 2) << 16;
                q += 3;
                const uint32_t last = bh & 1, type = (bh >> 1) & 3, bsize = bh >> 3;
                if (type == 3 || bsize > bmax) return RDX_BLOSC2_FAILED;
                if (type == 0) {
                    if (q + bsize > n || bsize > (uint64_t)z.n - z.op) return RDX_BLOSC2_FAILED;
                    if (bsize) z.literals(z.source(p + q, bsize), bsize);
                    q += bsize;
                } else if (type == 1) {
                    if (q + 1 > n || bsize > (uint64_t)z.n - z.op) return RDX_BLOSC2_FAILED;
                    z.run((uint8_t)h.byte(q), bsize);
                    q += 1;
                } else {
                    if (q + bsize > n) return RDX_BLOSC2_FAILED;
                    const uint64_t before = z.op;
                    if (!compressed_block(p + q, bsize, fstart)) return RDX_BLOSC2_FAILED;
                    if (z.op - before > bmax) return RDX_BLOSC2_FAILED;
                    q += bsize;
                }
                if (last) break;
            }
            if (fcs_bytes && z.op - fstart != fcs) return RDX_BLOSC2_FAILED;
        }
        return 0;
    }
};

}  // namespace

#if RDX_B2_WPE > 0
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(RDX_B2_WPE))) void k_blosc2_decode(const KBlosc2Args a) {
#else
__global__ __launch_bounds__(64 * kWaves) void k_blosc2_decode(const KBlosc2Args a) {
#endif
    __shared__ WaveLds LW[kWaves];
    // the wave index made scalar: the compiler's uniformity analysis does not see threadIdx.x >> 6 as
    // wave-uniform, and everything below (items, stream positions, the token chain) derives from it
    const uint32_t wave = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x / a.wg_per_chunk;
    if (c >= a.n) return;
    const uint64_t w0 = (uint64_t)(blockIdx.x % a.wg_per_chunk) * kWaves + wave;
    const uint64_t W = (uint64_t)a.wg_per_chunk * kWaves;
    const uint8_t *src = reinterpret_cast<const uint8_t *>(rfl64((uint64_t)gld<const uint8_t *>(a.in + c)));
    const uint64_t len = rfl64(gld<uint64_t>(a.in_len + c));
    const Hdr h = parse(src, len, a.cap, a.z_in != nullptr);
    uint32_t *err = a.err + c;
    if (w0 == 0 && lane == 0) a.out_len[c] = h.code == 0 || h.code == RDX_INFLATE_OUTPUT_OVERFLOW ? h.nbytes : 0;
    if (h.code) {
        if (w0 == 0) fail(err, h.code);
        return;
    }
    uint8_t *out = a.out + (uint64_t)c * a.cap;
    if (h.mode != M_BLOCKS) {
        for (uint64_t it = w0; it < h.items; it += W) {
            const uint64_t o = it * kUnit, m = h.nbytes - o < kUnit ? h.nbytes - o : kUnit;
            if (h.mode == M_MEMCPY) {
                wave_copy(out + o, src + h.overhead + o, m);
            } else if (h.special == 3) {   // the value after the header, repeated
                for (uint64_t i = lane; i < m; i += 64) out[o + i] = gld<uint8_t>(src + 32 + (o + i) % h.vts);
            } else if (h.special == 2) {   // quiet NaN of typesize 4 / 8 (little-endian bytes)
                for (uint64_t i = lane; i < m; i += 64) {
                    const uint32_t r = (uint32_t)((o + i) % h.ts);
                    out[o + i] = h.ts == 4 ? (r == 2 ? 0xc0 : r == 3 ? 0x7f : 0) : (r == 6 ? 0xf8 : r == 7 ? 0x7f : 0);
                }
            } else {   // zeros / uninitialised
                wave_fill(out + o, m, 0);
            }
        }
        return;
    }
    uint8_t *dbase = (h.nfilt ? a.scratch : a.out) + (uint64_t)c * a.cap;
    const uint64_t nfull = h.nbytes / h.bs, bt = h.overhead + 4 * h.nblocks;
    for (uint64_t it = w0; it < h.items; it += W) {
        uint64_t j, k, neblock;
        if (it < nfull * h.nstreams) {
            j = it / h.nstreams;
            k = it % h.nstreams;
            neblock = h.bs / h.nstreams;
        } else {
            j = nfull;
            k = 0;
            neblock = h.leftover;
        }
        const int32_t b0 = ld_i32(src + h.overhead + 4 * j);
        if (b0 < (int32_t)bt || (uint64_t)b0 >= h.cbytes) { fail(err, RDX_BLOSC2_FAILED); return; }
        uint64_t pos = (uint64_t)b0;
        int32_t cb = 0;
        for (uint64_t q = 0;; ++q) {   // walk the csize prefixes of this block's earlier streams
            if (pos + 4 > h.cbytes) { fail(err, RDX_BLOSC2_FAILED); return; }
            cb = ld_i32(src + pos);
            pos += 4;
            if (cb < 0) {
                if (pos + 1 > h.cbytes) { fail(err, RDX_BLOSC2_FAILED); return; }
            } else if (cb > 0 && pos + (uint64_t)cb > h.cbytes) {
                fail(err, RDX_BLOSC2_FAILED);
                return;
            }
            if (q == k) break;
            pos += cb < 0 ? 1 : (uint64_t)cb;
        }
        uint8_t *dst = dbase + j * h.bs + k * neblock;
        if (cb == 0) {
            wave_fill(dst, neblock, 0);
        } else if (cb < 0) {
            const uint32_t token = rfl((uint32_t)gld<uint8_t>(src + pos));
            if (!(token & 1) || cb < -255) { fail(err, RDX_BLOSC2_FAILED); return; }
            wave_fill(dst, neblock, (uint8_t)(-cb));
        } else if ((uint64_t)cb == neblock) {
            wave_copy(dst, src + pos, neblock);
        } else if (h.codec == 3 || h.codec == 4) {   // a row of the stream table: k_inflate (zlib, rows
            // [0, z_capacity)) or k_blosc2_zstd (zstd, rows [z_capacity, 2 z_capacity)) decodes it next
            const uint32_t which = h.codec == 4 ? 1u : 0u;
            uint32_t slot = 0;
            if (lane == 0) slot = atomicAdd(a.z_count + which, 1u);
            slot = rfl((uint32_t)__shfl((int)slot, 0, 64));
            if (slot >= a.z_capacity) { fail(err, RDX_BLOSC2_UNSUPPORTED); return; }
            slot += which * (uint32_t)a.z_capacity;
            if (lane == 0) {
                a.z_in[slot] = src + pos;
                a.z_len[slot] = (uint64_t)cb;
                a.z_out[slot] = dst;
                a.z_cap[slot] = neblock;
                a.z_chunk[slot] = c;
            }
        } else {
            const uint8_t *s = src + pos;
            const uint32_t skew = (uint32_t)((uintptr_t)s & 3);
            LzStream z{LW[wave], lane};
            z.srcw = reinterpret_cast<const uint32_t *>(s - skew);
            z.end = skew + (uint32_t)cb;
            z.staged = 0;
            z.dst = dst;
            z.n = (uint32_t)neblock;
            z.op = z.flushed = 0;
            z.load_unit(0);
            z.stage();
            const bool ok = h.codec == 0 ? z.blosclz(skew) : h.codec == 1 ? z.lz4(skew) : z.snappy(skew);
            if (!ok || z.op != neblock) { fail(err, RDX_BLOSC2_FAILED); return; }
            z.finish();
        }
    }
}

// Filters of one block, backwards (pipeline_backward): from the decode scratch into the output.
__global__ __launch_bounds__(256) void k_blosc2_filter(const KBlosc2Args a) {
    const uint32_t c = blockIdx.x / a.wg_per_chunk;
    if (c >= a.n) return;
    if (gld<uint32_t>(a.err + c)) return;   // written by the decode launch before this one
    const uint8_t *src = reinterpret_cast<const uint8_t *>(gld<const uint8_t *>(a.in + c));
    const uint64_t len = gld<uint64_t>(a.in_len + c);
    const Hdr h = parse(src, len, a.cap, a.z_in != nullptr);
    if (h.code || h.mode != M_BLOCKS || !h.nfilt) return;
    uint8_t *outc = a.out + (uint64_t)c * a.cap, *scr = a.scratch + (uint64_t)c * a.cap;
    const uint32_t ts = h.ts;
    for (uint64_t j = blockIdx.x % a.wg_per_chunk; j < h.nblocks; j += a.wg_per_chunk) {
        const uint64_t bsize = (h.leftover && j == h.nblocks - 1) ? h.leftover : h.bs;
        uint8_t *A = scr + j * h.bs, *B = outc + j * h.bs;
        for (uint32_t f = 0; f < h.nfilt; ++f) {
            const uint32_t kind = (h.filt >> (2 * f)) & 3u;
            const bool coherent = f > 0;   // this workgroup's own earlier stores: read them from L2
            auto rd = [&](const uint8_t *p) -> uint8_t {
                if (!coherent) return gld<uint8_t>(p);
                const uintptr_t q = (uintptr_t)p;
                const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t *>(q & ~(uintptr_t)3),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return (uint8_t)(w >> (8 * (q & 3)));
            };
            if (kind == 1) {
                const uint64_t ne = bsize / ts;
                for (uint64_t i = threadIdx.x; i < ne; i += blockDim.x) {
                    uint8_t *o = B + i * ts;
                    if (ts == 4 && ((uintptr_t)o & 3) == 0) {
                        const uint32_t v = (uint32_t)rd(A + i) | (uint32_t)rd(A + ne + i) << 8 |
                                           (uint32_t)rd(A + 2 * ne + i) << 16 | (uint32_t)rd(A + 3 * ne + i) << 24;
                        gst<uint32_t>(o, v);
                    } else if (ts == 8 && ((uintptr_t)o & 7) == 0) {
                        uint64_t v = 0;
#pragma unroll
                        for (uint32_t k = 0; k < 8; ++k) v |= (uint64_t)rd(A + k * ne + i) << (8 * k);
                        gst<uint64_t>(o, v);
                    } else {
                        for (uint32_t k = 0; k < ts; ++k) o[k] = rd(A + k * ne + i);
                    }
                }
                for (uint64_t i = ne * ts + threadIdx.x; i < bsize; i += blockDim.x) B[i] = rd(A + i);
            } else {
                // elements rounded down to a multiple of 8, the rest copied; a version-2 chunk's block
                // whose element count is not a multiple of 8 was stored unshuffled and is copied whole
                // (c-blosc2 bitunshuffle(..., format_version); oracle_blosc2.cpp bitunshuffle)
                uint64_t size = bsize / ts;
                size = (h.version == 2 && size % 8) ? 0 : size - size % 8;
                const uint64_t rowb = size / 8;
                for (uint64_t g = threadIdx.x; g < rowb; g += blockDim.x) {
                    for (uint32_t k = 0; k < ts; ++k) {
                        uint64_t x = 0;   // byte b = row (8k + b)'s byte g
#pragma unroll
                        for (uint32_t b = 0; b < 8; ++b) x |= (uint64_t)rd(A + (uint64_t)(8 * k + b) * rowb + g) << (8 * b);
                        // 8x8 bit transpose: byte e of the result = bit e of every byte
                        uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
                        x = x ^ t ^ (t << 7);
                        t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
                        x = x ^ t ^ (t << 14);
                        t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
                        x = x ^ t ^ (t << 28);
#pragma unroll
                        for (uint32_t e = 0; e < 8; ++e) B[(8 * g + e) * ts + k] = (uint8_t)(x >> (8 * e));
                    }
                }
                for (uint64_t i = size * ts + threadIdx.x; i < bsize; i += blockDim.x) B[i] = rd(A + i);
            }
            __syncthreads();
            uint8_t *t = A;
            A = B;
            B = t;
        }
        if (h.nfilt % 2 == 0) {   // the result is in the scratch block: move it to the output
            for (uint64_t i = threadIdx.x; i < bsize; i += blockDim.x) {
                const uintptr_t q = (uintptr_t)(A + i);
                const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t *>(q & ~(uintptr_t)3),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                B[i] = (uint8_t)(w >> (8 * (q & 3)));
            }
            __syncthreads();
        }
    }
}

// Results of the zlib-coded streams (k_inflate over the table): a stream that failed or did not produce
// exactly its block share fails its chunk, as blosc_d's size check.
__global__ __launch_bounds__(256) void k_blosc2_zcheck(const KBlosc2Args a) {
    for (uint32_t which = 0; which < 2; ++which) {
        const uint32_t n = __hip_atomic_load(a.z_count + which, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n && j < a.z_capacity;
             j += (uint64_t)gridDim.x * blockDim.x) {
            const uint64_t i = j + which * a.z_capacity;
            const uint32_t code = a.z_err[i] == RDX_BLOSC2_UNSUPPORTED ? (uint32_t)RDX_BLOSC2_UNSUPPORTED
                                                                      : (uint32_t)RDX_BLOSC2_FAILED;
            if (a.z_err[i] != 0 || a.z_out_len[i] != a.z_cap[i]) atomicCAS(a.err + a.z_chunk[i], 0u, code);
        }
    }
}

// zstd rows of the stream table: one wavefront per row, looping over the rows registered by k_blosc2_decode
__global__ __launch_bounds__(64 * kZWaves) __attribute__((amdgpu_waves_per_eu(RDX_ZWPE))) void k_blosc2_zstd(
    const KBlosc2Args a) {
    __shared__ ZLds LZ[kZWaves];
    const uint32_t wave = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t cnt = rfl(__hip_atomic_load(a.z_count + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint64_t n = cnt < a.z_capacity ? cnt : a.z_capacity;
    for (uint64_t r = (uint64_t)blockIdx.x * kZWaves + wave; r < n; r += (uint64_t)gridDim.x * kZWaves) {
        const uint64_t row = a.z_capacity + r;
        const uint8_t *src = reinterpret_cast<const uint8_t *>(rfl64((uint64_t)gld<const uint8_t *>(a.z_in + row)));
        const uint64_t len = rfl64(gld<uint64_t>(a.z_len + row));
        uint8_t *dst = reinterpret_cast<uint8_t *>(rfl64((uint64_t)gld<uint8_t *>(a.z_out + row)));
        const uint64_t cap = rfl64(gld<uint64_t>(a.z_cap + row));
        ZDec zd{LZ[wave], LzStreamT<kZRing>{LZ[wave].w, lane}, lane};
        zd.z.dst = dst;
        zd.z.n = (uint32_t)cap;
        zd.z.op = zd.z.flushed = 0;
        ZP_T(t_row);
        const uint32_t e = zd.stream(src, len);
        if (e == 0) zd.z.finish();
        if (lane == 0) {
            a.z_out_len[row] = e == 0 ? zd.z.op : 0;
            a.z_err[row] = e;
        }
#if RDX_PROBES
        zd.prof[0] += __builtin_amdgcn_s_memtime() - t_row;
        zd.prof[10] = zd.z.flushed / (kZRing / 4);
        if (lane == 0 && r < kZProfRows)
            for (uint32_t k = 0; k < kZProfK; ++k) g_zprof[r * kZProfK + k] = zd.prof[k];
#endif
    }
}

#if RDX_PROBES
}  // namespace rdx
// probe builds: k_blosc2_zstd's per-row phase cycles and counts of the last launch (g_zprof above)
extern "C" int rdx_probe_zprof_read(uint64_t *host, uint32_t n) {
    if (n > rdx::kZProfRows * rdx::kZProfK) n = rdx::kZProfRows * rdx::kZProfK;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rdx::g_zprof), n * sizeof(uint64_t)) == hipSuccess ? 0 : 1;
}
namespace rdx {
#endif

hipError_t launch_blosc2_zstd(const KBlosc2Args &a, hipStream_t s) {
    if (!a.z_capacity) return hipSuccess;
    const uint64_t wgs = std::min<uint64_t>((a.z_capacity + kZWaves - 1) / kZWaves, 2048);   // workgroups loop over rows
    hipLaunchKernelGGL(k_blosc2_zstd, dim3((uint32_t)wgs), dim3(64 * kZWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_blosc2_zcheck(const KBlosc2Args &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    if (a.z_in) {
        hipLaunchKernelGGL(k_blosc2_zcheck, dim3(256), dim3(256), 0, s, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_blosc2_filter, dim3(a.n * a.wg_per_chunk), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_blosc2(const KBlosc2Args &a, bool filters, hipStream_t s) {
    if (!a.n) return hipSuccess;
    const uint32_t blocks = a.n * a.wg_per_chunk;
    hipLaunchKernelGGL(k_blosc2_decode, dim3(blocks), dim3(64 * kWaves), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !filters) return e;
    hipLaunchKernelGGL(k_blosc2_filter, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace rdx
