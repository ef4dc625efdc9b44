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
// Unsupported here (RDX_BLOSC2_UNSUPPORTED, as the oracle): zstd, dictionaries, delta,
// user-defined codecs / filters (and more than 512 zlib-coded streams per chunk of a batch).
#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

constexpr uint32_t kWaves = 4;
constexpr uint32_t kRing = 8192, kRingMask = kRing - 1, kFlush = kRing / 4;
constexpr uint32_t kInBytes = 2048, kInWords = kInBytes / 4, kStage = 1024;
constexpr uint32_t kUnit = 4096;   // memcpy'ed / special chunks: bytes per work item

struct __attribute__((aligned(16))) WaveLds {
    uint8_t win[kRing];
    uint32_t in[kInWords];
};

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
    if (h.codec == 4 || h.codec == 6 || (h.codec == 3 && !zlib)) {
        h.code = RDX_BLOSC2_UNSUPPORTED;
        return h;
    }
    if (h.codec > 3) { h.code = RDX_BLOSC2_FAILED; return h; }
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
__device__ void wave_copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
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
__device__ void wave_fill(uint8_t *dst, uint64_t n, uint8_t v) {
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

struct LzStream {
    WaveLds &L;
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

    // write [flushed, flushed + m) of the ring to HBM (m <= kFlush)
    __device__ void flush(uint32_t m) {
        constexpr uint32_t kSl = kFlush / 64;
        wave_sync();
        const uint32_t base = (uint32_t)(flushed & kRingMask);
        const uint32_t lo = lane * kSl;
        const uint32_t cnt = lo >= m ? 0 : (m - lo < kSl ? m - lo : kSl);
        uint8_t *d = dst + flushed + lo;
        if (cnt == kSl && ((uintptr_t)d & 15) == 0) {
#pragma unroll
            for (uint32_t k = 0; k < kSl / 16; ++k)
                gst<uint4>(d + 16 * k, *reinterpret_cast<const uint4 *>(&L.win[base + lo + 16 * k]));
        } else {
            for (uint32_t k = 0; k < cnt; ++k) d[k] = L.win[(base + lo + k) & kRingMask];
        }
        flushed += m;
        // far match sources read these bytes back: their stores must be in L2 first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_sync();
    }
    __device__ __forceinline__ void room() {
        if (op - flushed > kRing - 64) flush(kFlush);
    }
    __device__ __forceinline__ uint8_t far_byte(uint32_t q) const {
        const uintptr_t a = (uintptr_t)(dst + q);
        const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return (uint8_t)(w >> (8 * (a & 3)));
    }
    // literal run of `run` bytes from input position ip
    __device__ void literals(uint32_t ip, uint32_t run) {
        for (uint32_t s = 0; s < run; s += 64) {
            ensure(ip + s + 64);
            room();
            const uint32_t k = run - s < 64 ? run - s : 64;
            if (lane < k) L.win[(op + lane) & kRingMask] = in_byte(ip + s + lane);
            op += k;
            asm volatile("" ::: "memory");
        }
    }
    // match of len bytes at distance dist (1 <= dist <= op)
    __device__ void match(uint32_t len, uint32_t dist) {
        for (uint32_t s = 0; s < len; s += 64) {
            room();
            const uint32_t k = len - s < 64 ? len - s : 64;
            if (lane < k) {
                const uint32_t m = dist < 64 ? lane % (uint32_t)dist : lane;
                const uint32_t back = dist - m, q = op - back;
                const uint8_t v = back <= kRing - 64 ? L.win[q & kRingMask] : far_byte(q);
                L.win[(op + lane) & kRingMask] = v;
            }
            op += k;
            asm volatile("" ::: "memory");
        }
    }
    __device__ void finish() {
        while (op > flushed) flush(op - flushed < kFlush ? (uint32_t)(op - flushed) : kFlush);
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

}  // namespace

__global__ __launch_bounds__(64 * kWaves) void k_blosc2_decode(const KBlosc2Args a) {
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
        } else if (h.codec == 3) {   // zlib: a row of the stream table, inflated by k_inflate next
            uint32_t slot = 0;
            if (lane == 0) slot = atomicAdd(a.z_count, 1u);
            slot = rfl((uint32_t)__shfl((int)slot, 0, 64));
            if (slot >= a.z_capacity) { fail(err, RDX_BLOSC2_UNSUPPORTED); return; }
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
    const uint32_t n = __hip_atomic_load(a.z_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n && i < a.z_capacity;
         i += (uint64_t)gridDim.x * blockDim.x)
        if (a.z_err[i] != 0 || a.z_out_len[i] != a.z_cap[i]) atomicCAS(a.err + a.z_chunk[i], 0u, (uint32_t)RDX_BLOSC2_FAILED);
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
