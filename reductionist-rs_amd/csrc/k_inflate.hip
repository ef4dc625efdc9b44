// k_inflate — the decompression stage of the filter pipeline (src/filter_pipeline.rs:23-25 ->
// src/compression.rs:18-82) on gfx950: gzip (flate2 GzDecoder: RFC 1952 member, CRC-32 + ISIZE
// checked, trailing bytes ignored) and zlib (zune-inflate decode_zlib: RFC 1950, Adler-32 checked),
// both RFC 1951 DEFLATE.
//
// A DEFLATE stream is one serial bit stream (block boundaries and symbol positions are only known
// after decoding everything before them), so the device parallelism is ACROSS streams: one
// wavefront per compressed chunk, a batch of chunks per launch.  Inside a wave:
//   * the symbol decode is wave-uniform serial code (GCN assembly, symbol_run): every lane holds
//     the same bit buffer and walks the same symbols in SGPRs (no divergence);
//   * the compressed bytes are staged 1 KiB at a time into a 2 KiB LDS input ring by all 64 lanes,
//     the next unit's loads in flight while the current one decodes;
//   * Huffman codes decode through LDS root tables (10 bits literal/length, with literal pairs; 8 bits
//     distance; the rare longer codes by the canonical bit-serial walk), rebuilt per block by all
//     lanes with ballot/popcount ranking instead of zlib's serial table construction;
//   * the output goes through an 8 KiB LDS ring holding the recent window: a back-reference copies
//     up to 64 bytes per step, one byte per lane (src = out - dist + (j mod dist) keeps every source
//     in already-written history, so overlapping matches need no serial byte loop); sources farther
//     back read the output already flushed to HBM; full 2 KiB units are flushed with 16-byte stores;
//   * the CRC-32 / Adler-32 of each flushed unit is computed by all lanes over 32-byte slices and
//     combined (CRC-32: each slice CRC shifted past the bytes after it by one GF(2) multiplication
//     and XOR-reduced, the running CRC folded into lane 0's slice; Adler-32: weighted sums).
// LDS per wave ≈ ring + 8.5 KiB; ring and streams per workgroup chosen per launch (InflateLds).
#include <algorithm>
#include <cstdlib>

#include "rdx_device.hpp"
#include "rdx_kernels.hpp"

namespace rdx {
namespace {

constexpr uint32_t kInBytes = 2048, kInWords = kInBytes / 4;  // input ring
constexpr uint32_t kStage = 1024;                             // bytes staged per refill of the ring
constexpr uint32_t kLitRoot = 10, kDistRoot = 8, kClRoot = 7;

// Per-stream LDS (one per wave).  The DEFLATE window is 32 KiB; the ring keeps the last RING bytes and
// a back-reference farther than that reads the already-flushed output in HBM (L2-hot).  The ring size
// trades residency against far copies, so it is picked per launch from the batch size
// (launch_inflate): a 32 KiB ring (the whole window, never a far copy) and 2 streams per workgroup up
// to 512 streams, 16 KiB x 4 up to 1024 (one wave per SIMD), 8 KiB x 4 beyond (two per SIMD, whose
// serial decode chains hide each other's LDS latency).
template <uint32_t RING>
struct __attribute__((aligned(16))) InflateLds {
    uint8_t win[RING];
    uint32_t in[kInWords];
    uint32_t lit[1u << kLitRoot];
    uint32_t dist[1u << kDistRoot];
    uint32_t cl[1u << kClRoot];
    uint16_t lsym[288], dsym[32], clsym[20];
    uint16_t lcount[16], dcount[16], clcount[16];
    uint16_t offs[16], next[16];
    uint8_t lens[320];
};

// Read-only tables shared by the workgroup's streams.
struct InflateShared {
    uint32_t crc_tab[4][256];    // slicing-by-4 CRC-32 tables (crc_tab[0] = the byte table)
    uint32_t x_after[64];        // x^(8 * 32 * (63 - l)) mod P: shifts lane l's slice CRC to the unit end
    uint32_t x2n[32];            // x^(2^k) mod P (CRC-32 combine)
    uint32_t lbase[29];          // base | extra << 16
    uint32_t dbase[30];
};

// The decode state is wave-uniform: values read from LDS by every lane are made scalar with
// readfirstlane, so the bit buffer, positions and symbol dispatch live in SGPRs and branch on SCC
// (no exec-mask juggling on the serial path).
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return (uint64_t)rfl((uint32_t)(x >> 32)) << 32 | rfl((uint32_t)x);
}
// LDS byte address of a __shared__ object (the address operand of ds_* instructions)
template <class P>
__device__ __forceinline__ uint32_t lds_addr(P *p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void *)p;
}

// Decode-table entry: value (literal byte / length or distance base) in bits 0-15, code length in
// 16-19 (0 = code longer than the root: bit-serial walk), extra bits in 20-23, type in 24-25
// (0 literal or distance, 1 length, 2 end of block, 3 invalid symbol).  Literals have no extra bits:
// their bits 20-21 hold the literal count instead, 1, or 2 for a literal/length root entry holding
// TWO literals whose codes together fit the root (bytes in bits 0-7 and 8-15, the summed length in
// 16-19).
constexpr uint32_t kTypeLen = 1u << 24, kTypeEob = 2u << 24, kTypeBad = 3u << 24, kOneLit = 1u << 20, kPair = 2u << 20;

// Phase counters for tools/probe_inflate.hip (RDX_INFLATE_PROF); compiled out of the product.
#ifdef RDX_INFLATE_PROF
enum { P_LIT, P_MATCH, P_MATCH_BYTES, P_FAR, P_SLOW, P_BLOCKS, P_STAGE, P_FLUSH, P_T_COPY, P_T_FLUSH, P_T_TABLES,
       P_T_STORED, P_T_GENERAL, P_T_TOTAL, P_N };
__device__ unsigned long long g_prof[P_N];
#define PROF_ADD(k, v) (prof[k] += (v))
#define PROF_T0() const uint64_t _t0 = __builtin_readcyclecounter()
#define PROF_T1(k) (prof[k] += __builtin_readcyclecounter() - _t0)
#else
#define PROF_ADD(k, v) ((void)0)
#define PROF_T0() ((void)0)
#define PROF_T1(k) ((void)0)
#endif

// LDS ordering inside ONE wavefront: its LDS instructions execute in order, so a compiler barrier is
// all a lane needs to read what another lane of the same wave wrote (the workgroup's other waves
// decode other streams and never touch this wave's LDS).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- CRC-32 (reflected 0xEDB88320) algebra, as in zlib's crc32_combine ---------------------------
// multmodp restates zlib's crc32.c function of that name (zlib 1.2.12+, (C) Jean-loup Gailly and Mark Adler,
// zlib license): a(x) * b(x) modulo the CRC-32 polynomial, a's bits taken from the top.
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = b & 1 ? (b >> 1) ^ 0xedb88320u : b >> 1;
    }
    return p;
}

// a(x) * b(x) mod P for a lane-varying a: all 32 terms, no data-dependent branches
__device__ __forceinline__ uint32_t mulp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        p ^= (a >> i) & 1 ? b : 0u;
        b = (b >> 1) ^ (b & 1 ? 0xedb88320u : 0u);
    }
    return p;
}

// x^(8n) mod P
__device__ __forceinline__ uint32_t x8n(const InflateShared &L, uint64_t n) {
    uint32_t p = 1u << 31;
    uint32_t k = 3;
    while (n) {
        if (n & 1) p = multmodp(L.x2n[k & 31], p);
        n >>= 1;
        ++k;
    }
    return p;
}

constexpr uint32_t kAdlerMod = 65521;

struct KInflateArgs {
    const uint8_t *const *in;  // device array of stream pointers
    const uint64_t *in_len;    // device array of stream lengths
    uint8_t *out;              // stream i -> out + i * cap
    uint64_t cap;
    uint64_t *out_len;
    uint32_t *err;
    uint32_t format;           // RDX_COMPRESSION_GZIP / ZLIB
    uint32_t n;                // streams (the grid's capacity when n_dev is set)
    // stream tables filled on the device (blosc2 chunks with zlib-coded streams, k_blosc2.hip): the
    // stream count in device memory, and per stream its own output pointer and capacity
    const uint32_t *n_dev;
    uint8_t *const *out_ptrs;
    const uint64_t *caps;
};

template <uint32_t RING>
struct Inflater {
    static constexpr uint32_t kWin = RING, kWinMask = RING - 1;  // LDS ring: the recent window
    static constexpr uint32_t kFlush = RING / 4;                  // output unit written to HBM
    static_assert(kFlush + 516 <= kWin, "the unflushed tail plus one copy (or stored step) must fit the ring");
    InflateLds<RING> &L;
    const InflateShared &S;
    const uint32_t lane;
    // input: the stream as dwords from its 4-byte aligned base; byte q of that aligned stream is
    // byte q - skew of the chunk
    const uint32_t *srcw;
    uint64_t end;     // skew + length: first byte past the stream (aligned-stream coordinates)
    uint64_t staged;  // aligned-stream bytes [.., staged) are in the ring
    uint64_t pf_start;             // the unit whose words are in flight into pf (~0: none)
    uint32_t pf[kStage / 4 / 64];  // this lane's words of that unit
    uint64_t pos;     // next byte to move into the bit buffer
    uint64_t bb;      // bit buffer (LSB first)
    uint32_t bc;      // valid bits in bb
    // output
    uint8_t *dst;
    uint64_t cap, out, flushed;
    // checksums of the flushed output
    uint32_t crc, s1, s2;
    bool gzip;
    uint32_t err;
#ifdef RDX_INFLATE_PROF
    uint64_t prof[P_N];
#endif

    // ---- input -----------------------------------------------------------------------------------
    // One kStage unit of the input as this lane's words (lane-contiguous), bytes past the stream zeroed.
    __device__ __forceinline__ void load_unit(uint64_t start, uint32_t (&v)[kStage / 4 / 64]) const {
        const uint64_t w0 = start / 4 + (uint64_t)lane * (kStage / 4 / 64);
#pragma unroll
        for (int k = 0; k < (int)(kStage / 4 / 64); ++k) {
            const uint64_t w = w0 + k;
            v[k] = 0;
            if (w * 4 < end) {
                v[k] = gld<uint32_t>(srcw + w);
                const uint64_t valid = end - w * 4;  // zero the bytes past the stream
                if (valid < 4) v[k] &= (1u << (8 * valid)) - 1;
            }
        }
    }
    // Stage [start, start + kStage) with start >= pos rounded down into the input ring, then start
    // loading the unit after it: the next stage finds it in registers instead of waiting a full
    // memory round trip (1-2 us per KiB of input otherwise, a third of the decode time at ratio 1).
    __device__ __forceinline__ void stage() {
        PROF_ADD(P_STAGE, 1);
        uint64_t start = pos & ~(uint64_t)(kStage - 1);
        if (start < staged) start = staged;
        if (start != pf_start) load_unit(start, pf);
        const uint32_t i0 = (uint32_t)(start / 4 + (uint64_t)lane * (kStage / 4 / 64));
#pragma unroll
        for (int k = 0; k < (int)(kStage / 4 / 64); ++k) L.in[(i0 + k) & (kInWords - 1)] = pf[k];
        staged = start + kStage;
        pf_start = staged;
        load_unit(pf_start, pf);
        wave_sync();
    }
    __device__ __forceinline__ uint32_t word_at(uint64_t p) const {
        const uint32_t i = (uint32_t)(p >> 2) & (kInWords - 1), sh = (uint32_t)(p & 3) * 8;
        const uint32_t lo = rfl(L.in[i]), hi = rfl(L.in[(i + 1) & (kInWords - 1)]);
        return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
    }
    __device__ __forceinline__ uint32_t byte_at(uint64_t p) const {
        return (L.in[(p >> 2) & (kInWords - 1)] >> ((p & 3) * 8)) & 0xffu;
    }
    // at least 33 valid bits afterwards (unless the input is exhausted -> err)
    __device__ __forceinline__ void refill() {
        if (bc <= 32) {
            if (pos + 8 > staged) stage();
            const uint32_t w = (pos & 3) ? word_at(pos) : rfl(L.in[(uint32_t)(pos >> 2) & (kInWords - 1)]);
            bb |= (uint64_t)w << bc;
            pos += 4;
            bc += 32;
            if (pos > end + 8 && !err) err = RDX_INFLATE_TRUNCATED;  // decoding the zero padding
        }
    }
    __device__ __forceinline__ uint32_t bits(uint32_t n) {  // n <= 32, bc >= n
        const uint32_t v = (uint32_t)(bb & ((1ull << n) - 1));
        bb >>= n;
        bc -= n;
        return v;
    }
    __device__ __forceinline__ uint32_t need(uint32_t n) {  // n <= 32
        if (bc < n) refill();
        return bits(n);
    }
    // bytes consumed so far (aligned-stream coordinates)
    __device__ __forceinline__ uint64_t consumed() const { return pos - bc / 8; }
    __device__ __forceinline__ void align() {
        const uint32_t r = bc & 7;
        bb >>= r;
        bc -= r;
    }
    __device__ __forceinline__ uint32_t byte() {  // byte-aligned read
        const uint32_t v = need(8);
        if (consumed() > end && !err) err = RDX_INFLATE_TRUNCATED;
        return v;
    }

    // ---- output ----------------------------------------------------------------------------------
    // Write [flushed, flushed + n) of the ring to HBM (n <= kFlush) and fold it into the checksum.
    __device__ __forceinline__ void flush(uint32_t n) {
        constexpr uint32_t kSl = kFlush / 64;  // bytes per lane slice
        PROF_ADD(P_FLUSH, 1);
        PROF_T0();
        wave_sync();
        const uint32_t base = (uint32_t)(flushed & kWinMask);
        const uint32_t lo = lane * kSl;
        const uint32_t cnt = lo >= n ? 0 : (n - lo < kSl ? n - lo : kSl);
        uint8_t *d = dst + flushed + lo;
        uint32_t c = 0, a = 0, b = 0;  // slice crc, s1, s2
        if (cnt == kSl && ((uintptr_t)d & 15) == 0) {
#pragma unroll
            for (uint32_t k = 0; k < kSl / 16; ++k) {
                const uint4 v = *reinterpret_cast<const uint4 *>(&L.win[base + lo + 16 * k]);
                gst<uint4>(d + 16 * k, v);
            }
        } else {
            for (uint32_t k = 0; k < cnt; ++k) d[k] = L.win[(base + lo + k) & kWinMask];
        }
        if (gzip) {
            // CRC-32 is linear: crc(state, unit) = XOR over lanes of lane l's slice CRC shifted past the
            // bytes after it (x^(8 * after) mod P), with the running state folded into lane 0's start.
            // `crc` is the raw register (no final inversion).  Full slices: slicing-by-4 over dwords
            // and a per-lane constant shift; a short final unit: bytes and a computed shift.
            c = lane == 0 ? crc : 0u;
            uint32_t xa;
            if (cnt == kSl) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(&L.win[base + lo]);
#pragma unroll
                for (uint32_t k = 0; k < kSl / 4; ++k) {
                    c ^= w[k];
                    c = S.crc_tab[3][c & 0xff] ^ S.crc_tab[2][(c >> 8) & 0xff] ^ S.crc_tab[1][(c >> 16) & 0xff] ^
                        S.crc_tab[0][c >> 24];
                }
                xa = n == kFlush ? S.x_after[lane] : x8n(S, n - (lo + cnt));
            } else {
                for (uint32_t k = 0; k < cnt; ++k) c = S.crc_tab[0][(c ^ L.win[(base + lo + k) & kWinMask]) & 0xff] ^ (c >> 8);
                xa = x8n(S, lo + cnt < n ? n - (lo + cnt) : 0);
            }
            c = mulp(xa, c);
#pragma unroll
            for (int m = 1; m < 64; m <<= 1) c ^= (uint32_t)__shfl_xor((int)c, m, 64);
            crc = rfl(c);
        } else {
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t v = L.win[(base + lo + k) & kWinMask];
                a += v;
                b += (cnt - k) * v;
            }
            // s2(unit) = sum over slices of s2_l + (bytes after slice l) * s1_l
            const uint64_t after = n - (lo + cnt > n ? n : lo + cnt);
            uint64_t t1 = a % kAdlerMod, t2 = (b + (after % kAdlerMod) * (a % kAdlerMod)) % kAdlerMod;
#pragma unroll
            for (int m = 1; m < 64; m <<= 1) {
                t1 += (uint64_t)__shfl_xor((long long)t1, m, 64);
                t2 += (uint64_t)__shfl_xor((long long)t2, m, 64);
            }
            t1 = rfl((uint32_t)(t1 % kAdlerMod));
            t2 = rfl((uint32_t)(t2 % kAdlerMod));
            t2 %= kAdlerMod;
            s2 = (uint32_t)((s2 + (uint64_t)(n % kAdlerMod) * s1 + t2) % kAdlerMod);
            s1 = (uint32_t)((s1 + t1) % kAdlerMod);
        }
        flushed += n;
        // the flushed bytes are read back by back-references farther than the ring (copy()): their
        // stores must have completed in L2 before any such load issues
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_sync();
        PROF_T1(P_T_FLUSH);
    }
    // Flushing happens at ONE place per loop (general() / the stored-copy loop), so the flush code is
    // inlined once there instead of behind every literal and copy.  The unflushed tail stays below
    // kWin: hot() stops at kWin - 258 (one match of room), general() and stored() add at most one
    // copy (<= 258 bytes) after a flush_full(); so no write reaches a ring slot still unflushed, and
    // a source farther back than the ring is always already in HBM.
    __device__ __forceinline__ void flush_full() {
        while (out - flushed >= kFlush) flush(kFlush);
    }
    __device__ __forceinline__ bool room(uint64_t n) {
        if (out + n > cap) {
            if (!err) err = RDX_INFLATE_OUTPUT_OVERFLOW;
            return false;
        }
        return true;
    }
    __device__ __forceinline__ void literal(uint32_t v) {
        if (!room(1)) return;
        if (lane == 0) L.win[out & kWinMask] = (uint8_t)v;
        ++out;
    }
    __device__ __forceinline__ void copy_at(uint64_t o, uint32_t len, uint32_t dist) {
        PROF_ADD(P_MATCH, 1);
        PROF_ADD(P_MATCH_BYTES, len);
        PROF_ADD(P_FAR, dist > kWin - 258 ? 1 : 0);
        asm volatile("" ::: "memory");  // after lane 0's literal writes (in-order LDS, same wave)
        const uint32_t o32 = (uint32_t)o;  // ring indices need only the low bits
        // j mod dist for overlapping copies by a float reciprocal (exact after one correction)
        const float rd = __builtin_amdgcn_rcpf((float)dist);
        for (uint32_t j0 = 0; j0 < len; j0 += 64) {
            const uint32_t j = j0 + lane;
            if (j < len) {
                uint32_t m = j;
                if (dist < len) {
                    const uint32_t q = (uint32_t)((float)j * rd);
                    int32_t r = (int32_t)(j - q * dist);
                    r = r < 0 ? r + (int32_t)dist : (r >= (int32_t)dist ? r - (int32_t)dist : r);
                    m = (uint32_t)r;
                }
                const uint32_t back = dist - m;  // source = o - back
                // the ring holds [frontier - kWin, frontier), the frontier having advanced by the j0
                // bytes this copy already wrote; anything older is flushed to HBM (o - flushed <=
                // kWin - 258 and j0 <= 256, flush_full())
                uint8_t v;
                if (back + j0 <= kWin) [[likely]] v = L.win[(o32 - back) & kWinMask];
                else v = gld<uint8_t>(dst + (o - back));
                L.win[(o32 + j) & kWinMask] = v;
            }
        }
        asm volatile("" ::: "memory");
    }
    __device__ __forceinline__ void copy(uint32_t len, uint32_t dist) {
        if (!room(len)) return;
        copy_at(out, len, dist);
        out += len;
    }

    // ---- Huffman ---------------------------------------------------------------------------------
    // Canonical code of n lengths -> root table (2^root entries: symbol | length << 16, 0 = longer
    // code) + count[] / sym[] for the bit-serial walk.  Returns 0 complete, > 0 incomplete,
    // < 0 over-subscribed; count[0] = number of unused symbols.
    // table entry of symbol s: kind 0 = code-length code (value = s), 1 = literal/length, 2 = distance
    __device__ __forceinline__ uint32_t entry_of(uint32_t s, uint32_t kind) const {
        if (kind == 1) {
            if (s < 256) return s | kOneLit;
            if (s == 256) return kTypeEob;
            if (s < 286) {
                const uint32_t lb = S.lbase[s - 257];
                return (lb & 0xffff) | (lb >> 16) << 20 | kTypeLen;
            }
            return kTypeBad;
        }
        if (kind == 2) {
            if (s < 30) {
                const uint32_t db = S.dbase[s];
                return (db & 0xffff) | (db >> 16) << 20;
            }
            return kTypeBad;
        }
        return s;
    }
    __device__ __forceinline__ int build(const uint8_t *lens, uint32_t n, uint32_t *tab, uint32_t root, uint16_t *count,
                         uint16_t *sym, uint32_t kind) {
        uint32_t cnt[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) cnt[l] = 0;
        for (uint32_t b0 = 0; b0 < n; b0 += 64) {
            const uint32_t s = b0 + lane;
            const uint32_t l = s < n ? lens[s] : 16;
#pragma unroll
            for (int q = 0; q < 16; ++q) cnt[q] += (uint32_t)__popcll(__ballot(l == (uint32_t)q));
        }
        int left = 1;
        bool over = false;
        uint32_t offs[16], next[16];
        offs[1] = 0;
        next[0] = 0;
        uint32_t code = 0;
#pragma unroll
        for (int l = 1; l < 16; ++l) {
            left <<= 1;
            left -= (int)cnt[l];
            over |= left < 0;
            if (l < 15) offs[l + 1] = offs[l] + cnt[l];
            code = (code + (l == 1 ? 0 : cnt[l - 1])) << 1;
            next[l] = code;
        }
        for (uint32_t i = lane; i < (1u << root); i += 64) tab[i] = 0;
        if (lane == 0) {
#pragma unroll
            for (int l = 0; l < 16; ++l) {
                count[l] = (uint16_t)cnt[l];
                L.offs[l] = (uint16_t)(l ? offs[l] : 0);
                L.next[l] = (uint16_t)(l ? next[l] : 0);
            }
        }
        wave_sync();
        if (cnt[0] == n) return 0;  // no codes at all: complete by convention (puff)
        if (over) return -1;
        uint32_t run[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) run[l] = 0;
        const uint64_t lt = (1ull << lane) - 1;
        for (uint32_t b0 = 0; b0 < n; b0 += 64) {
            const uint32_t s = b0 + lane;
            const uint32_t l = s < n ? lens[s] : 0;
            uint32_t rank = 0;
#pragma unroll
            for (int q = 1; q < 16; ++q) {
                const uint64_t m = __ballot(l == (uint32_t)q);
                if (l == (uint32_t)q) rank = run[q] + (uint32_t)__popcll(m & lt);
                run[q] += (uint32_t)__popcll(m);
            }
            if (l) {
                sym[L.offs[l] + rank] = (uint16_t)s;
                if (l <= root) {
                    const uint32_t c = L.next[l] + rank;
                    const uint32_t r = __builtin_bitreverse32(c) >> (32 - l);
                    const uint32_t e = entry_of(s, kind) | l << 16;
                    for (uint32_t k = r; k < (1u << root); k += 1u << l) tab[k] = e;
                }
            }
        }
        wave_sync();
        if (kind == 1 && root == kLitRoot) {
            // literal pairs: where a root entry is a literal of l1 bits and the next 10 - l1 bits
            // start a literal code of l2 <= 10 - l1 bits (the entry at index >> l1 decodes it: its
            // missing high bits are past that code), one lookup yields both
            constexpr uint32_t kPer = (1u << kLitRoot) / 64;
            uint32_t ent[kPer];
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) {
                const uint32_t i = k * 64 + lane;
                uint32_t e1 = tab[i];
                const uint32_t l1 = (e1 >> 16) & 15;
                if (l1 && (e1 >> 24) == 0) {
                    const uint32_t e2 = tab[i >> l1];
                    const uint32_t l2 = (e2 >> 16) & 15;
                    if (l2 && (e2 >> 24) == 0 && l1 + l2 <= kLitRoot)
                        e1 = (e1 & 0xff) | (e2 & 0xff) << 8 | (l1 + l2) << 16 | kPair;
                }
                ent[k] = e1;
            }
            wave_sync();
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) tab[k * 64 + lane] = ent[k];
            wave_sync();
        }
        return left;
    }
    // ---- blocks ------------------------------------------------------------------------------------
    __device__ __forceinline__ void fixed_tables() {
        for (uint32_t s = lane; s < 288 + 30; s += 64)
            L.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
        wave_sync();
        build(L.lens, 288, L.lit, kLitRoot, L.lcount, L.lsym, 1);
        build(L.lens + 288, 30, L.dist, kDistRoot, L.dcount, L.dsym, 2);
    }

    __device__ __forceinline__ void dynamic_tables() {
        refill();
        const uint32_t nlen = bits(5) + 257, ndist = bits(5) + 1, ncode = bits(4) + 4;
        if (nlen > 286 || ndist > 30) {
            err = RDX_INFLATE_CODE_LENGTHS;
            return;
        }
        // 19 code-length code lengths, 3 bits each, in the permuted order of RFC 1951 §3.2.7
        refill();
        const uint32_t n1 = ncode < 10 ? ncode : 10;
        const uint64_t v1 = bits(3 * n1);
        refill();
        const uint32_t n2 = ncode - n1;
        const uint64_t v2 = n2 ? bits(3 * n2) : 0;
        if (lane < 19) {
            constexpr uint32_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            uint32_t ord = 0;
#pragma unroll
            for (int i = 0; i < 19; ++i)
                if ((uint32_t)i == lane) ord = kOrder[i];
            uint32_t v = 0;
            if (lane < ncode) v = lane < 10 ? (uint32_t)(v1 >> (3 * lane)) & 7 : (uint32_t)(v2 >> (3 * (lane - 10))) & 7;
            L.lens[ord] = (uint8_t)v;
        }
        wave_sync();
        if (build(L.lens, 19, L.cl, kClRoot, L.clcount, L.clsym, 0) != 0) {  // complete code required
            err = RDX_INFLATE_CODE_LENGTHS;
            return;
        }
        // literal/length + distance code lengths (run-length coded)
        const uint32_t total = nlen + ndist;
        uint32_t idx = 0, prev = 0;
        bool has_eob = false;
        while (idx < total && !err) {
            refill();
            const uint32_t e = rfl(L.cl[(uint32_t)bb & ((1u << kClRoot) - 1)]);
            const uint32_t l = (e >> 16) & 15, sym = e & 0xffff;
            bb >>= l;
            bc -= l;
            if (sym < 16) {
                if (lane == 0) L.lens[idx] = (uint8_t)sym;
                if (idx == 256) has_eob = sym != 0;
                prev = sym;
                ++idx;
                continue;
            }
            uint32_t rep, val = 0;
            if (sym == 16) {
                if (idx == 0) {
                    err = RDX_INFLATE_CODE_LENGTHS;
                    break;
                }
                val = prev;
                rep = 3 + bits(2);
            } else if (sym == 17) {
                rep = 3 + bits(3);
            } else {
                rep = 11 + bits(7);
            }
            if (idx + rep > total) {
                err = RDX_INFLATE_CODE_LENGTHS;
                break;
            }
            if (lane < rep) L.lens[idx + lane] = (uint8_t)val;
            if (lane + 64 < rep) L.lens[idx + lane + 64] = (uint8_t)val;
            if (lane + 128 < rep) L.lens[idx + lane + 128] = (uint8_t)val;
            if (idx <= 256 && 256 < idx + rep) has_eob = val != 0;
            prev = val;
            idx += rep;
        }
        wave_sync();
        if (err) return;
        if (!has_eob) {
            err = RDX_INFLATE_CODE_LENGTHS;
            return;
        }
        int r = build(L.lens, nlen, L.lit, kLitRoot, L.lcount, L.lsym, 1);
        if (r < 0 || (r > 0 && nlen != rfl((uint32_t)L.lcount[0] + L.lcount[1]))) {
            err = RDX_INFLATE_CODE_LENGTHS;
            return;
        }
        r = build(L.lens + nlen, ndist, L.dist, kDistRoot, L.dcount, L.dsym, 2);
        if (r < 0 || (r > 0 && ndist != rfl((uint32_t)L.dcount[0] + L.dcount[1]))) err = RDX_INFLATE_CODE_LENGTHS;
    }

    // refill for the Huffman loop: `pos` is always 4-byte aligned there (stored() realigns it)
    __device__ __forceinline__ void refill_fast() {
        if (bc <= 32) {
            if (pos + 8 > staged) [[unlikely]] {
                stage();
                if (pos > end + 8 && !err) err = RDX_INFLATE_TRUNCATED;  // decoding the zero padding
            }
            bb |= (uint64_t)rfl(L.in[(uint32_t)(pos >> 2) & (kInWords - 1)]) << bc;
            pos += 4;
            bc += 32;
        }
    }
    // slow symbol: a code longer than the table root (bit-serial canonical walk), or no code
    __device__ uint32_t decode_slow(const uint16_t *count, const uint16_t *sym, uint32_t kind) {
        PROF_ADD(P_SLOW, 1);
        int code = 0, first = 0, index = 0;
#pragma unroll 1
        for (int len = 1; len < 16; ++len) {
            code |= (int)(bb & 1);
            bb >>= 1;
            --bc;
            const int c = (int)rfl(count[len]);
            if (code - c < first) return entry_of(rfl(sym[index + (code - first)]), kind);
            index += c;
            first += c;
            first <<= 1;
            code <<= 1;
        }
        return kTypeBad;
    }

    // The symbol loop of hot() in GCN assembly.  The compiler's version carried ~47 instructions per
    // literal (phi copies between SGPRs, a spilled exec mask for lane 0's store) and a match went
    // through ~1000 cycles of mixed scalar/vector code; here a literal (pair) is ~30 instructions
    // and a near match ~45 plus its two LDS round trips.  State: the bit buffer pinned to s[80:81]
    // (s[82:83] scratch), valid bits c (>= 33 at the loop top), input / output positions p / o as
    // their low 32 bits (all the ring masks need), countdowns rp / ro (as in hot()).  Per symbol:
    // look the next 10 bits up in the literal/length root table; a literal (pair) is stored to the
    // window ring (lane j writes byte j, exec = the count); a length whose distance code hits the
    // distance root table and whose source lies in the ring (dist <= kWin - 258) is copied ring to
    // ring, 64 bytes per step (source o - dist + (j mod dist), always written history).  Leaves with
    // why = 1 at a limit (ro < 0, or a refill due with rp < 0), why = 0 at a symbol for general()
    // (long code, end of block, invalid, or a distance past the output start), nothing consumed;
    // why = 2 after consuming a far match (len, dist) for copy_at() to take from HBM.
    __device__ __forceinline__ void symbol_run(uint64_t &b, uint32_t &c, uint32_t &p32, uint32_t &o32, int32_t &rp,
                                               int32_t &ro, uint32_t &why, uint32_t &len, uint32_t &dist,
                                               uint32_t o_small, uint32_t v_in, uint32_t v_lit, uint32_t v_dst,
                                               uint32_t v_win, uint32_t v_lane, uint32_t v_sh) {
        static_assert(kInWords * 4 == 0x800 && kLitRoot == 10 && kDistRoot == 8, "masks hard-coded below");
#define RDX_REFILL                             \
    "  s_and_b32 s82, %[p], 0x7fc\n"           \
    "  v_add_u32 %[vr], s82, %[vin]\n"         \
    "  ds_read_b32 %[vr], %[vr]\n"             \
    "  s_waitcnt lgkmcnt(0)\n"                 \
    "  v_readfirstlane_b32 s82, %[vr]\n"       \
    "  s_mov_b32 s83, 0\n"                     \
    "  s_lshl_b64 s[82:83], s[82:83], %[c]\n"  \
    "  s_or_b64 s[80:81], s[80:81], s[82:83]\n" \
    "  s_add_u32 %[p], %[p], 4\n"              \
    "  s_sub_i32 %[rp], %[rp], 4\n"            \
    "  s_add_u32 %[c], %[c], 32\n"
#define RDX_COPY_STEP(L)                        \
    "  v_and_b32 %[vs], %[wm], %[vs]\n"        \
    "  v_add_u32 %[vs], %[vs], %[vwin]\n"       \
    "  v_add_u32 %[va], %[o], %[vj]\n"          \
    "  v_and_b32 %[va], %[wm], %[va]\n"        \
    "  v_add_u32 %[va], %[va], %[vwin]\n"       \
    "  s_sub_u32 %[w], %[len], %[j]\n"          \
    "  s_mov_b64 s[82:83], -1\n"                \
    "  s_cmp_lt_u32 %[w], 64\n"                 \
    "  s_cbranch_scc0 " L "f\n"                 \
    "  s_bfm_b64 s[82:83], %[w], 0\n"           \
    L ":\n"                                     \
    "  s_mov_b64 exec, s[82:83]\n"              \
    "  ds_read_u8 %[vd], %[vs]\n"               \
    "  s_waitcnt lgkmcnt(0)\n"                  \
    "  ds_write_b8 %[va], %[vd]\n"              \
    "  s_mov_b64 exec, %[sav]\n"                \
    "  s_add_u32 %[j], %[j], 64\n"              \
    "  s_cmp_lt_u32 %[j], %[len]\n"
        uint64_t sav, bs;
        uint32_t t0, t1, e, u, w, j, od, rs, va, vv, vj, vq, vs, vr, vd;
        asm volatile(
            "  s_mov_b64 %[sav], exec\n"
            "  s_cmp_gt_u32 %[c], 32\n"
            "  s_cbranch_scc1 1f\n"
            "  s_cmp_lt_i32 %[rp], 0\n"
            "  s_cbranch_scc1 80f\n"
            RDX_REFILL
            "1:\n"  // loop top (c >= 33): look the next symbol up
            "  s_cmp_lt_i32 %[ro], 0\n"
            "  s_cbranch_scc1 80f\n"
            "  s_and_b32 s82, s80, 0x3ff\n"
            "  v_lshl_add_u32 %[va], s82, 2, %[vlit]\n"
            "  ds_read_b32 %[vv], %[va]\n"
            "3:\n"  // the lookup of the symbol at the head of the bit buffer is in flight (c >= 33)
            "  s_waitcnt lgkmcnt(0)\n"
            "  v_readfirstlane_b32 %[e], %[vv]\n"
            "  s_bfe_u32 %[u], %[e], 0x40010\n"
            "  s_sub_u32 %[w], %[e], 0x10000\n"
            "  s_cmp_lt_u32 %[w], 0xff0000\n"
            "  s_cbranch_scc0 20f\n"
            // literal (pair): consume it and issue the next lookup first (>= 23 valid bits remain), then
            // store it and refill while that lookup is in flight
            "  s_bfe_u32 %[w], %[e], 0x20014\n"
            "  s_lshr_b64 s[80:81], s[80:81], %[u]\n"
            "  s_sub_u32 %[c], %[c], %[u]\n"
            "  s_and_b32 s82, s80, 0x3ff\n"
            "  v_lshl_add_u32 %[va], s82, 2, %[vlit]\n"
            "  ds_read_b32 %[vv], %[va]\n"
            "  v_add_u32 %[va], %[o], %[vlane]\n"
            "  v_and_b32 %[va], %[wm], %[va]\n"
            "  v_add_u32 %[va], %[va], %[vwin]\n"
            "  v_lshrrev_b32 %[vj], %[vsh], %[e]\n"
            "  s_bfm_b64 s[82:83], %[w], 0\n"
            "  s_mov_b64 exec, s[82:83]\n"
            "  ds_write_b8 %[va], %[vj]\n"
            "  s_mov_b64 exec, %[sav]\n"
            "  s_add_u32 %[o], %[o], %[w]\n"
            "  s_sub_i32 %[ro], %[ro], %[w]\n"
            "  s_cmp_lt_i32 %[ro], 0\n"
            "  s_cbranch_scc1 80f\n"
            "  s_cmp_gt_u32 %[c], 32\n"
            "  s_cbranch_scc1 3b\n"
            "  s_cmp_lt_i32 %[rp], 0\n"
            "  s_cbranch_scc1 80f\n"
            RDX_REFILL
            "  s_branch 3b\n"
            // length symbol: base + extra bits
            "20:\n"
            "  s_cmp_eq_u32 %[u], 0\n"
            "  s_cbranch_scc1 81f\n"
            "  s_lshr_b32 %[w], %[e], 24\n"
            "  s_cmp_lg_u32 %[w], 1\n"
            "  s_cbranch_scc1 81f\n"
            "  s_mov_b64 %[bs], s[80:81]\n"
            "  s_mov_b32 %[od], %[c]\n"
            "  s_mov_b32 %[j], %[p]\n"
            "  s_mov_b32 %[rs], %[rp]\n"
            "  s_lshr_b64 s[80:81], s[80:81], %[u]\n"
            "  s_sub_u32 %[c], %[c], %[u]\n"
            "  s_bfe_u32 %[u], %[e], 0x40014\n"
            "  s_bfm_b32 %[w], %[u], 0\n"
            "  s_and_b32 %[w], s80, %[w]\n"
            "  s_and_b32 %[len], %[e], 0xffff\n"
            "  s_add_u32 %[len], %[len], %[w]\n"
            "  s_lshr_b64 s[80:81], s[80:81], %[u]\n"
            "  s_sub_u32 %[c], %[c], %[u]\n"
            "  s_cmp_gt_u32 %[c], 32\n"
            "  s_cbranch_scc1 21f\n"
            "  s_cmp_lt_i32 %[rp], 0\n"
            "  s_cbranch_scc1 82f\n"
            RDX_REFILL
            // distance: root table + extra bits
            "21:\n"
            "  s_and_b32 %[w], s80, 0xff\n"
            "  v_lshl_add_u32 %[va], %[w], 2, %[vdst]\n"
            "  ds_read_b32 %[vv], %[va]\n"
            "  s_waitcnt lgkmcnt(0)\n"
            "  v_readfirstlane_b32 %[e], %[vv]\n"
            "  s_bfe_u32 %[u], %[e], 0x40010\n"
            "  s_cmp_eq_u32 %[u], 0\n"
            "  s_cbranch_scc1 83f\n"
            "  s_cmp_gt_u32 %[e], 0xffffff\n"
            "  s_cbranch_scc1 83f\n"
            "  s_lshr_b64 s[80:81], s[80:81], %[u]\n"
            "  s_sub_u32 %[c], %[c], %[u]\n"
            "  s_bfe_u32 %[u], %[e], 0x40014\n"
            "  s_bfm_b32 %[w], %[u], 0\n"
            "  s_and_b32 %[w], s80, %[w]\n"
            "  s_and_b32 %[dist], %[e], 0xffff\n"
            "  s_add_u32 %[dist], %[dist], %[w]\n"
            "  s_lshr_b64 s[80:81], s[80:81], %[u]\n"
            "  s_sub_u32 %[c], %[c], %[u]\n"
            "  s_cmp_eq_u32 %[osm], 0\n"
            "  s_cbranch_scc1 22f\n"
            "  s_cmp_gt_u32 %[dist], %[o]\n"
            "  s_cbranch_scc1 83f\n"
            "22:\n"
            "  s_cmp_gt_u32 %[dist], %[near]\n"
            "  s_cbranch_scc1 84f\n"
            // near copy, ring to ring, with the next symbol's lookup in flight meanwhile (>= 12 valid
            // bits remain after the distance)
            "  s_sub_u32 %[od], %[o], %[dist]\n"
            "  s_mov_b32 %[j], 0\n"
            "  s_and_b32 s82, s80, 0x3ff\n"
            "  v_lshl_add_u32 %[va], s82, 2, %[vlit]\n"
            "  ds_read_b32 %[vv], %[va]\n"
            "  s_cmp_lt_u32 %[dist], %[len]\n"
            "  s_cbranch_scc1 40f\n"
            "30:\n"  // source o - dist + j
            "  v_add_u32 %[vj], %[j], %[vlane]\n"
            "  v_add_u32 %[vs], %[od], %[vj]\n"
            RDX_COPY_STEP("31")
            "  s_cbranch_scc1 30b\n"
            "  s_branch 50f\n"
            "40:\n"  // overlapping (dist < len): source o - dist + (j mod dist), float reciprocal + correction
            "  v_cvt_f32_u32 %[vr], %[dist]\n"
            "  v_rcp_f32 %[vr], %[vr]\n"
            "41:\n"
            "  v_add_u32 %[vj], %[j], %[vlane]\n"
            "  v_cvt_f32_u32 %[vq], %[vj]\n"
            "  v_mul_f32 %[vq], %[vq], %[vr]\n"
            "  v_cvt_u32_f32 %[vq], %[vq]\n"
            "  v_mul_lo_u32 %[vq], %[vq], %[dist]\n"
            "  v_sub_u32 %[vq], %[vj], %[vq]\n"
            "  v_add_u32 %[vs], %[dist], %[vq]\n"
            "  v_cmp_gt_i32 vcc, 0, %[vq]\n"
            "  v_cndmask_b32 %[vq], %[vq], %[vs], vcc\n"
            "  v_subrev_u32 %[vs], %[dist], %[vq]\n"
            "  v_cmp_le_u32 vcc, %[dist], %[vq]\n"
            "  v_cndmask_b32 %[vq], %[vq], %[vs], vcc\n"
            "  v_add_u32 %[vs], %[od], %[vq]\n"
            RDX_COPY_STEP("42")
            "  s_cbranch_scc1 41b\n"
            "50:\n"
            "  s_add_u32 %[o], %[o], %[len]\n"
            "  s_sub_i32 %[ro], %[ro], %[len]\n"
            "  s_cmp_lt_i32 %[ro], 0\n"
            "  s_cbranch_scc1 80f\n"
            "  s_cmp_gt_u32 %[c], 32\n"
            "  s_cbranch_scc1 3b\n"
            "  s_cmp_lt_i32 %[rp], 0\n"
            "  s_cbranch_scc1 80f\n"
            RDX_REFILL
            "  s_branch 3b\n"
            "80:\n"
            "  s_mov_b32 %[why], 1\n"
            "  s_branch 90f\n"
            "81:\n"
            "  s_mov_b32 %[why], 0\n"
            "  s_branch 90f\n"
            "82:\n"
            "  s_mov_b32 %[why], 1\n"
            "  s_branch 85f\n"
            "83:\n"
            "  s_mov_b32 %[why], 0\n"
            "85:\n"  // nothing consumed: restore the state before the length symbol
            "  s_mov_b64 s[80:81], %[bs]\n"
            "  s_mov_b32 %[c], %[od]\n"
            "  s_mov_b32 %[p], %[j]\n"
            "  s_mov_b32 %[rp], %[rs]\n"
            "  s_branch 90f\n"
            "84:\n"
            "  s_mov_b32 %[why], 2\n"
            "90:\n"
            "  s_waitcnt lgkmcnt(0)\n"
            : [b] "+{s[80:81]}"(b), [t0] "={s82}"(t0), [t1] "={s83}"(t1), [c] "+s"(c), [p] "+s"(p32), [o] "+s"(o32),
              [rp] "+s"(rp), [ro] "+s"(ro), [why] "=&s"(why), [len] "=&s"(len), [dist] "=&s"(dist),
              [sav] "=&s"(sav), [bs] "=&s"(bs), [e] "=&s"(e), [u] "=&s"(u), [w] "=&s"(w), [j] "=&s"(j),
              [od] "=&s"(od), [rs] "=&s"(rs), [va] "=&v"(va), [vv] "=&v"(vv),
              [vj] "=&v"(vj), [vq] "=&v"(vq), [vs] "=&v"(vs), [vr] "=&v"(vr), [vd] "=&v"(vd)
            : [osm] "s"(o_small), [vin] "v"(v_in), [vlit] "v"(v_lit), [vdst] "v"(v_dst), [vwin] "v"(v_win),
              [vlane] "v"(v_lane), [vsh] "v"(v_sh), [wm] "n"(kWinMask), [near] "n"(kWin - 258)
            : "memory", "scc", "vcc");
#undef RDX_REFILL
#undef RDX_COPY_STEP
    }

    // The symbol loop of one Huffman block, in two tiers.  A wave issues one instruction per 4 cycles
    // at best, so the serial decode is paid per INSTRUCTION: hot() keeps the whole state in a handful
    // of scalar locals and handles only the common cases (literals, and matches whose codes hit the
    // root tables, with the ring and the input known to have room); anything else (input staging,
    // flushing, codes longer than the root, end of block, capacity, errors) leaves hot() WITHOUT
    // consuming the symbol, and general() decodes that one symbol with every check.
    __device__ __forceinline__ void hot() {
        // loop-carried state uniform from the start: phis of SGPR values stay in SGPRs (re-reading
        // them with readfirstlane at the loop head instead makes the compiler carry VGPR copies)
        uint64_t b = rfl64(bb), p = rfl64(pos), o = rfl64(out);
        uint32_t c = rfl(bc);
        const uint64_t stop_p = rfl64(staged) - 8;  // a dword refill needs p + 8 <= staged
        // the unflushed tail may grow to the whole ring less one match: hot() leaves (and general()
        // flushes every complete unit) once per ~3 units, not at every symbol past the first unit
        const uint64_t fl = rfl64(flushed) + kWin, cp = rfl64(cap);
        const uint64_t lim = fl < cp ? fl : cp;
        const uint64_t stop_o = lim > 258 ? lim - 258 : 0;  // room for one more literal or match
        if (rfl64(o) > stop_o || rfl64(p) > stop_p + 8) return;
        // 32-bit countdowns (SALU has no 64-bit ordered compare): input bytes left before a refill
        // would pass `staged`, output bytes left before the ring / capacity check is due
        const uint64_t dp = stop_p + 8 - p, dout = stop_o - o;
        int32_t rp = (int32_t)rfl((uint32_t)((int32_t)(dp < 0x40000000u ? dp : 0x40000000u) - 8));
        int32_t ro = (int32_t)rfl((uint32_t)(dout < 0x40000000u ? dout : 0x40000000u));
        const uint32_t v_in = lds_addr(L.in), v_lit = lds_addr(L.lit), v_dst = lds_addr(L.dist);
        const uint32_t v_win = lds_addr(L.win), v_lane = lane, v_sh = lane * 8;
        for (;;) {
            asm volatile("; inflate hot loop" ::: "memory");
            // positions travel through the asm as their low 32 bits, advanced here by what it consumed
            uint32_t p32 = (uint32_t)p, o32 = (uint32_t)o, why, len, dist;
            const uint32_t p0 = p32, o0 = o32, o_small = rfl((uint32_t)(o >> 31) == 0 ? 1u : 0u);
            symbol_run(b, c, p32, o32, rp, ro, why, len, dist, o_small, v_in, v_lit, v_dst, v_win, v_lane, v_sh);
            p += p32 - p0;
            o += o32 - o0;
            PROF_ADD(P_LIT, o32 - o0);
            if (why != 2) break;
            len = rfl(len);
            dist = rfl(dist);
            PROF_T0();
            copy_at(o, len, dist);   // a source past the ring: from the flushed output in HBM
            PROF_T1(P_T_COPY);
            // past copy_at's lane-dependent code the compiler no longer proves the loop state uniform
            o = rfl64(o + len);
            ro = (int32_t)rfl((uint32_t)(ro - (int32_t)len));
            b = rfl64(b);
            p = rfl64(p);
            c = rfl(c);
            rp = (int32_t)rfl((uint32_t)rp);
        }
        bb = b;
        bc = c;
        pos = p;
        out = o;
    }

    // One symbol with every check; returns true at the end of the block (or on an error).
    __device__ __forceinline__ bool general() {
        flush_full();
        refill();
        if (err) return true;
        uint32_t e = rfl(L.lit[(uint32_t)bb & ((1u << kLitRoot) - 1)]);
        const uint32_t l = (e >> 16) & 15;
        if (l) {
            bb >>= l;
            bc -= l;
        } else {
            e = decode_slow(L.lcount, L.lsym, 1);
        }
        const uint32_t type = e & (3u << 24);
        if (type == 0) {
            PROF_ADD(P_LIT, 1);
            literal(e & 0xff);
            if (e & kPair) literal((e >> 8) & 0xff);
            return err != 0;
        }
        if (type == kTypeEob) return true;
        if (type != kTypeLen) {
            err = RDX_INFLATE_BAD_SYMBOL;
            return true;
        }
        const uint32_t len = (e & 0xffff) + bits((e >> 20) & 15);
        refill();
        uint32_t d = rfl(L.dist[(uint32_t)bb & ((1u << kDistRoot) - 1)]);
        const uint32_t dl = (d >> 16) & 15;
        if (dl) {
            bb >>= dl;
            bc -= dl;
        } else {
            d = decode_slow(L.dcount, L.dsym, 2);
        }
        if (d & (3u << 24)) {
            err = RDX_INFLATE_BAD_SYMBOL;
            return true;
        }
        const uint32_t dist = (d & 0xffff) + bits((d >> 20) & 15);
        if (dist > out) {
            err = RDX_INFLATE_DISTANCE;
            return true;
        }
        copy(len, dist);
        return err != 0;
    }

    __device__ __forceinline__ void codes() {
        while (!err) {
            hot();
            PROF_T0();
            const bool end = general();
            PROF_T1(P_T_GENERAL);
            if (end) break;
        }
    }

    __device__ __forceinline__ void stored() {
        align();
        const uint32_t len = byte() | byte() << 8;
        const uint32_t nlen = byte() | byte() << 8;
        if (err) return;
        if (len != (~nlen & 0xffff)) {
            err = RDX_INFLATE_STORED_LENGTH;
            return;
        }
        uint32_t left = len;
        while (left && bc >= 8 && !err) {  // whole bytes still in the bit buffer (< 8)
            literal(bits(8));
            --left;
        }
        // the rest straight from the input ring, 256 bytes per step (4 per lane; the unflushed tail
        // stays below kFlush + 256 <= kWin - 258, the input ring keeps >= 1 KiB ahead of pos)
        constexpr uint32_t kStep = 256;
        while (left && !err) {
            flush_full();
            if (pos + kStep > staged) stage();
            const uint32_t m = left < kStep ? left : kStep;
            if (pos + m > end) {
                err = RDX_INFLATE_TRUNCATED;
                break;
            }
            if (!room(m)) break;
            uint32_t v[kStep / 64];
#pragma unroll
            for (uint32_t k = 0; k < kStep / 64; ++k) v[k] = byte_at(pos + lane + 64 * k);
#pragma unroll
            for (uint32_t k = 0; k < kStep / 64; ++k)
                if (lane + 64 * k < m) L.win[(uint32_t)(out + lane + 64 * k) & kWinMask] = (uint8_t)v[k];
            __builtin_amdgcn_wave_barrier();
            out += m;
            pos += m;
            left -= m;
        }
        // keep `pos` 4-byte aligned (the Huffman loop refills whole dwords): move the rest of the
        // current dword into the bit buffer
        if (!err && (pos & 3)) {
            const uint32_t sh = (uint32_t)(pos & 3) * 8;
            bb = rfl(L.in[(uint32_t)(pos >> 2) & (kInWords - 1)]) >> sh;
            bc = 32 - sh;
            pos = (pos | 3) + 1;
        }
    }

    __device__ __forceinline__ void run() {
        bool last = false;
        bool fixed_ready = false;
        while (!last && !err) {
            flush_full();
            refill();
            last = bits(1);
            PROF_ADD(P_BLOCKS, 1);
            const uint32_t type = bits(2);
            if (type == 0) {
                PROF_T0();
                stored();
                PROF_T1(P_T_STORED);
            } else if (type == 1) {
                PROF_T0();
                if (!fixed_ready) fixed_tables();
                PROF_T1(P_T_TABLES);
                fixed_ready = true;
                codes();
            } else if (type == 2) {
                fixed_ready = false;
                PROF_T0();
                dynamic_tables();
                PROF_T1(P_T_TABLES);
                if (!err) codes();
            } else {
                err = RDX_INFLATE_BLOCK_TYPE;
            }
        }
    }
};

template <uint32_t RING, uint32_t WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_inflate(const KInflateArgs a) {
    constexpr uint32_t kThreads = 64 * WAVES;
    // a device-side stream count: workgroups past it leave before building their tables
    uint32_t n = a.n;   // with a device-side count: never past the table (the grid covers a.n rows)
    if (a.n_dev) n = min(n, rfl(__hip_atomic_load(a.n_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    if ((uint64_t)blockIdx.x * WAVES >= n) return;
    __shared__ InflateShared S;
    __shared__ InflateLds<RING> LW[WAVES];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // shared constant tables (once per workgroup; the only workgroup-wide barriers)
    if (t < 29) {
        constexpr uint16_t kB[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
        uint32_t b = 0;
#pragma unroll
        for (int k = 0; k < 29; ++k)
            if ((uint32_t)k == t) b = kB[k];
        const uint32_t e = t < 8 || t == 28 ? 0 : (t - 4) / 4;
        S.lbase[t] = b | e << 16;
    } else if (t >= 32 && t < 62) {
        const uint32_t c = t - 32;
        const uint32_t e = c < 2 ? 0 : c / 2 - 1;
        const uint32_t b = c < 4 ? c + 1 : (1u << e) * (2 + (c & 1)) + 1;
        S.dbase[c] = b | e << 16;
    } else if (t == 63) {
        uint32_t p = 1u << 30;  // x^1
        for (int k = 0; k < 32; ++k) {
            S.x2n[k] = p;
            p = multmodp(p, p);
        }
    }
    for (uint32_t q = t; q < 256; q += kThreads) {
        uint32_t c = q;
        for (int k = 0; k < 8; ++k) c = c & 1 ? 0xedb88320u ^ (c >> 1) : c >> 1;
        S.crc_tab[0][q] = c;
    }
    __syncthreads();
    // slicing tables (each from the byte table) and the per-lane unit shifts (from x2n)
    for (uint32_t q = t; q < 256; q += kThreads) {
        uint32_t c = S.crc_tab[0][q];
        for (int k = 1; k < 4; ++k) {
            c = (c >> 8) ^ S.crc_tab[0][c & 0xff];
            S.crc_tab[k][q] = c;
        }
    }
    if (t < 64) S.x_after[t] = x8n(S, (Inflater<RING>::kFlush / 64) * (63 - t));
    __syncthreads();
    InflateLds<RING> &L = LW[wave];
    // stream i = this wave's index, then every gridDim.x * WAVES further (a stream table's grid is smaller
    // than the table: one workgroup's tables serve several streams)
    const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
    for (uint64_t i = (uint64_t)blockIdx.x * WAVES + wv; i < n; i += (uint64_t)gridDim.x * WAVES) {
    // scalar: every lane reads the same descriptor, and the decode state derived from it must stay
    // wave-uniform (SGPRs) for the serial path to compile to scalar code
    const uint8_t *src = reinterpret_cast<const uint8_t *>(rfl64((uint64_t)gld<const uint8_t *>(a.in + i)));
    const uint64_t len = rfl64(gld<uint64_t>(a.in_len + i));

    const uint32_t skew = (uint32_t)((uintptr_t)src & 3);
    Inflater<RING> f{L, S, lane};
    f.srcw = reinterpret_cast<const uint32_t *>(src - skew);
    f.end = skew + len;
    f.staged = 0;
    f.pf_start = ~0ull;
    f.pos = 0;
    f.bb = 0;
    f.bc = 0;
    f.dst = a.out_ptrs ? reinterpret_cast<uint8_t *>(rfl64((uint64_t)gld<uint8_t *>(a.out_ptrs + i)))
                       : a.out + (uint64_t)i * a.cap;
    f.cap = a.caps ? rfl64(gld<uint64_t>(a.caps + i)) : a.cap;
    f.out = f.flushed = 0;
    f.crc = 0xffffffffu;  // raw CRC-32 register
    f.s1 = 0;
    f.s2 = 0;
    f.gzip = a.format == RDX_COMPRESSION_GZIP;
    f.err = 0;
#ifdef RDX_INFLATE_PROF
    for (int k = 0; k < P_N; ++k) f.prof[k] = 0;
    const uint64_t t_start = __builtin_readcyclecounter();
#endif
    f.stage();
    if (skew) {  // refills stay 4-byte aligned: drop the bytes before the stream from the bit buffer
        f.refill();
        f.bits(8 * skew);
    }

    if (f.gzip) {  // RFC 1952 member header (flate2 GzDecoder)
        if (len < 2 || f.need(8) != 0x1f || f.need(8) != 0x8b) {
            f.err = RDX_INFLATE_GZIP_HEADER;
        } else if (f.byte() != 8) {
            f.err = f.err ? f.err : RDX_INFLATE_GZIP_HEADER;
        } else {
            const uint32_t flg = f.byte();
            for (int k = 0; k < 6; ++k) f.byte();  // MTIME, XFL, OS
            if (flg & 4) {                         // FEXTRA
                uint32_t xlen = f.byte();
                xlen |= f.byte() << 8;
                for (uint32_t k = 0; k < xlen && !f.err; ++k) f.byte();
            }
            if (flg & 8)
                while (!f.err && f.byte() != 0) {}  // FNAME
            if (flg & 16)
                while (!f.err && f.byte() != 0) {}  // FCOMMENT
            if (flg & 2) {                          // FHCRC (not verified, as the oracle)
                f.byte();
                f.byte();
            }
        }
    } else {  // RFC 1950 (zune-inflate decode_zlib)
        if (len < 2) {
            f.err = RDX_INFLATE_TRUNCATED;
        } else {
            const uint32_t cmf = f.need(8), flg = f.need(8);
            if ((cmf & 15) != 8) f.err = RDX_INFLATE_ZLIB_METHOD;
            else if ((cmf >> 4) > 7 || (cmf * 256 + flg) % 31 != 0 || (flg & 0x20)) f.err = RDX_INFLATE_ZLIB_HEADER;
        }
    }
    if (!f.err) {
        f.run();
        // the reference decoders read bit by bit and stop at the first bit past the input: any
        // failure met after the stream's end is "input truncated" there (oracle_inflate.cpp BitIn)
        if (f.err && f.pos * 8 - f.bc > f.end * 8) f.err = RDX_INFLATE_TRUNCATED;
    }
    if (!f.err) {
        f.flush_full();
        if (f.out > f.flushed) f.flush((uint32_t)(f.out - f.flushed));
    }
    if (!f.err) {  // trailer
        f.align();
        if (f.gzip) {
            uint32_t crc = 0, isize = 0;
            for (int k = 0; k < 4; ++k) crc |= f.byte() << (8 * k);
            for (int k = 0; k < 4; ++k) isize |= f.byte() << (8 * k);
            if (!f.err && (crc != ~f.crc || isize != (uint32_t)f.out)) f.err = RDX_INFLATE_CHECKSUM;
        } else {
            uint32_t ad = 0;
            for (int k = 0; k < 4; ++k) ad = ad << 8 | f.byte();
            const uint32_t want = (uint32_t)((f.s2 + f.out % kAdlerMod) % kAdlerMod) << 16 | (f.s1 + 1) % kAdlerMod;
            if (!f.err && ad != want) f.err = RDX_INFLATE_CHECKSUM;
        }
    }
    if (lane == 0) {
        a.out_len[i] = f.out;
        a.err[i] = f.err;
#ifdef RDX_INFLATE_PROF
        f.prof[P_T_TOTAL] = __builtin_readcyclecounter() - t_start;
        for (int k = 0; k < P_N; ++k) atomicAdd(&g_prof[k], (unsigned long long)f.prof[k]);
#endif
    }
    }
}

}  // namespace

hipError_t launch_inflate(uint32_t format, const uint8_t *const *d_in, const uint64_t *d_in_len, uint64_t n,
                          uint8_t *d_out, uint64_t cap, uint64_t *d_out_len, uint32_t *d_err, hipStream_t s) {
    if (n == 0) return hipSuccess;
    KInflateArgs a{d_in, d_in_len, d_out, cap, d_out_len, d_err, format, (uint32_t)n, nullptr, nullptr, nullptr};
    // ring size from the batch size (InflateLds); RDX_INFLATE_RING=8192/16384/32768 forces one (tuning)
    static const int force = [] {
        const char *v = std::getenv("RDX_INFLATE_RING");
        return v ? std::atoi(v) : 0;
    }();
    const uint32_t ring = force ? (uint32_t)force : n <= 512 ? 32768u : n <= 1024 ? 16384u : 8192u;
    if (ring == 32768u) {
        hipLaunchKernelGGL((k_inflate<32768, 2>), dim3((uint32_t)((n + 1) / 2)), dim3(128), 0, s, a);
    } else if (ring == 16384u) {
        hipLaunchKernelGGL((k_inflate<16384, 4>), dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL((k_inflate<8192, 4>), dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

// Streams described by device tables (k_blosc2's zlib-coded block streams): up to max_n, the actual count
// in *d_n; stream i -> d_out_ptrs[i] with capacity d_caps[i].  Many short streams: 8 KiB rings, 4 per
// workgroup, at most 1024 workgroups looping over the rows (an empty table costs one small launch).
hipError_t launch_inflate_table(const uint8_t *const *d_in, const uint64_t *d_in_len, uint8_t *const *d_out_ptrs,
                                const uint64_t *d_caps, const uint32_t *d_n, uint64_t max_n, uint64_t *d_out_len,
                                uint32_t *d_err, hipStream_t s) {
    if (max_n == 0) return hipSuccess;
    KInflateArgs a{d_in, d_in_len, nullptr, 0, d_out_len, d_err, RDX_COMPRESSION_ZLIB, (uint32_t)max_n, d_n, d_out_ptrs,
                   d_caps};
    const uint64_t wgs = std::min<uint64_t>((max_n + 3) / 4, 1024);   // workgroups loop over the rows
    hipLaunchKernelGGL((k_inflate<8192, 4>), dim3((uint32_t)wgs), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace rdx
