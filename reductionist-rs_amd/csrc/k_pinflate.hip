// k_pinflate — ONE gzip / zlib stream decoded by the whole chip: a lone compressed request
// (src/filter_pipeline.rs:23-25 -> src/compression.rs:60-82; the reference's docs name decompression the
// heaviest stage, docs/architecture.md:225-228).  k_inflate decodes a batch of streams one wavefront
// each; on a single stream that leaves one wavefront busy for 100-220 ms per 4 MiB.  Here the DEFLATE
// blocks of the stream, and the symbols inside each block, are decoded in parallel:
//
//  1. k_pinf_find   every bit offset is tested for a dynamic-Huffman block header as a zlib encoder writes
//                   it (BTYPE 2, HLIT / HDIST in range, a complete code-length code, a complete literal /
//                   length code with an end-of-block code, a complete or one-code distance code) and every
//                   byte offset for a stored block (LEN = ~NLEN, zero bits before it): the candidates
//                   (every such block start, plus rare false ones).
//  2. k_pinf_block  one workgroup per candidate parses its header with the oracle's checks, builds the
//                   decode tables in LDS and decodes the block body with 1024 lanes at once: lane k starts
//                   at an arbitrary bit of the body (Huffman decoding resynchronises within a few
//                   symbols), stops at its first symbol boundary past its range, and is valid once its
//                   start equals the exit of lane k-1; a mismatched lane re-decodes from that exit, in
//                   rounds, then by a sequential walk if the data keeps the parses apart.  Per candidate:
//                   the end-of-block position, the output size, every lane's verified start and bytes.
//  3. k_pinf_chain  from the stream header, each block's end names the next block's start; the chain of
//                   candidates to BFINAL is followed (successors by binary search over the sorted
//                   candidates in LDS) and the output offsets assigned.  A block start that is no
//                   candidate (a fixed-Huffman block, a header the finder does not accept) goes back to
//                   the host, which decodes that candidate alone and chains again.
//  4. k_pinf_emit   one workgroup per chain block re-decodes its lanes from their verified starts and
//                   writes every output byte as a 32-bit SOURCE: a literal (flag | byte) or the position
//                   the byte copies (o - dist; inside an overlapping match, (j mod dist) into the bytes
//                   before it).
//  5. k_pinf_tile   pointer jumping over the sources inside 32 KiB tiles of output in LDS (a link always
//                   points to a byte with the same final value) until each byte is a literal or a link
//                   into the previous tile; k_pinf_xhop then resolves the links between tiles by pointer
//                   jumping over every tile with links at once, and k_pinf_xout writes their bytes.
//  6. k_pinf_finish / k_pinf_check  Adler-32 / CRC-32 over segments combined by weights / GF(2) shifts,
//                   the trailer.
//
// The path only ever ACCEPTS a stream the sequential decoder accepts, with the same bytes: any error on
// the chain, a chain that cannot be followed, an unresolved byte or a checksum mismatch reports "not
// decoded" and the host runs k_inflate on the stream, which gives the exact error (oracle_inflate).
#include <algorithm>

#include "rdx_device.hpp"
#include "rdx_kernels.hpp"
#include "rdx_pinflate.h"

namespace rdx {
namespace {

constexpr uint32_t kLanes = kPinfLanes;    // decode lanes (threads) per block
#ifndef RDX_PINF_MINBITS
#define RDX_PINF_MINBITS 256
#endif
constexpr uint64_t kMinLaneBits = RDX_PINF_MINBITS;   // a lane's share of a block body, at least
constexpr uint32_t kRoot = 11, kDRoot = 9; // LDS root tables: literal/length, distance
constexpr uint32_t kFlag = 0x80000000u;    // a source that is a literal byte
constexpr uint32_t kRounds = 6;            // resync rounds before a sequential walk
#ifndef RDX_PINF_WARMBITS
#define RDX_PINF_WARMBITS 256
#endif
constexpr uint64_t kWarmBits = RDX_PINF_WARMBITS;   // bits a lane decodes before its range in pass 0
constexpr uint64_t kMaxSpan = 1ull << 21;  // bits a candidate may decode (a zlib block is < 1.6 M bits)
#ifndef RDX_PINF_WIN
#define RDX_PINF_WIN 8192
#endif
// LDS window of the stream per block workgroup: 32 KiB, 256 K bits from the header (past it a lane's refills
// are L2 round trips; an 80 KiB window measured the same on 306 K-bit blocks, r06_pinflate_ab_window.jsonl)
constexpr uint32_t kWinDwords = RDX_PINF_WIN;

// decode-table entry: value in bits 0-15, code length 16-19 (0: longer than the root), extra bits 20-23,
// type 24-25 (0 literal or distance, 1 length, 2 end of block, 3 invalid symbol)
constexpr uint32_t kTyLen = 1u << 24, kTyEob = 2u << 24, kTyBad = 3u << 24;


typedef const __attribute__((address_space(3))) uint32_t *lds_u32p;   // an LDS pointer: ds_read, not flat
typedef __attribute__((address_space(3))) uint64_t *lds_u64p;
// k_pinf_emit: a lane's short matches are recorded (position | (length | distance << 16) << 32) in its LDS
// slots, kEmitRecs of them interleaved with the other lanes' (slot k of thread t at k * kEmitThreads + t),
// and expanded after its decode loop ends: the loop itself writes no match bytes, so a wavefront's symbol
// step no longer runs as long as the longest match any of its 64 lanes copies (an inner loop of up to 31
// per-byte steps per symbol); a lane with more matches than slots writes the rest in the loop
#ifndef RDX_PINF_EMIT_RECS
#define RDX_PINF_EMIT_RECS 24
#endif
constexpr uint32_t kEmitRecs = RDX_PINF_EMIT_RECS;
#ifndef RDX_PINF_EMIT_HALVES
#define RDX_PINF_EMIT_HALVES 1
#endif
constexpr bool kEmitHalves = RDX_PINF_EMIT_HALVES != 0;        // two threads a lane (PinfArgs::lmid)
constexpr uint32_t kEmitLanes = kLanes / kPinfEmitSplit;      // lanes per k_pinf_emit workgroup
constexpr uint32_t kEmitThreads = kEmitHalves ? 2 * kEmitLanes : kEmitLanes;   // k_pinf_emit's workgroup
// its window of the stream: 16 KiB, its lanes of a 1024-lane block up to 1 M bits (past it, L2)
constexpr uint32_t kEmitWin = 8192 * 4 / kPinfEmitSplit;

// ---- the stream as dwords from its 4-byte aligned base (bit positions in those coordinates) ------------
struct Stream {
    const uint32_t *w;
    uint64_t nw;        // dwords holding stream bytes
    uint32_t lmask;     // valid bytes of the last one
    // a window of the stream staged in LDS (dwords [l0, l0 + ln)), read instead of L2 where it covers
    lds_u32p lds;
    uint64_t l0;
    uint32_t ln;
    __device__ __forceinline__ uint32_t ldg(uint64_t i) const {
        if (i >= nw) return 0;
        const uint32_t v = gld<uint32_t>(w + i);
        return i + 1 == nw ? v & lmask : v;
    }
    __device__ __forceinline__ uint32_t ld(uint64_t i) const {
        const uint64_t k = i - l0;
        if (k < ln) return lds[k];
        return ldg(i);
    }
    // all threads of the workgroup: stage up to `cap` dwords from dword i0 into `buf`, then read from it
    __device__ __forceinline__ void stage(uint32_t *buf, uint32_t cap, uint64_t i0, uint64_t i1) {
        const uint32_t n = (uint32_t)min<uint64_t>(cap, i1 > i0 ? i1 - i0 : 0);
        for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) buf[k] = ldg(i0 + k);
        lds = (lds_u32p)buf;
        l0 = i0;
        ln = n;
        __syncthreads();
    }
    // 32 bits from bit position p
    __device__ __forceinline__ uint32_t at(uint64_t p) const {
        const uint64_t i = p >> 5;
        const uint32_t sh = (uint32_t)p & 31;
        const uint64_t v = (uint64_t)ld(i) | (uint64_t)ld(i + 1) << 32;
        return (uint32_t)(v >> sh);
    }
    __device__ __forceinline__ uint32_t byte(uint64_t q) const { return (ld(q >> 2) >> (8 * (q & 3))) & 0xffu; }
};

__device__ __forceinline__ Stream make_stream(const PinfArgs &a) {
    Stream s;
    s.w = a.w;
    s.nw = a.nw;
    s.lmask = a.lmask;
    s.lds = nullptr;
    s.l0 = 0;
    s.ln = 0;
    return s;
}

// A lane's bit reader: 64-bit buffer, refilled one dword at a time.
struct Bits {
    uint64_t bb;
    uint32_t bc;
    uint64_t nxt;
    __device__ __forceinline__ void seek(const Stream &S, uint64_t p) {
        nxt = p >> 5;
        const uint32_t sh = (uint32_t)p & 31;
        const uint64_t v = (uint64_t)S.ld(nxt) | (uint64_t)S.ld(nxt + 1) << 32;
        nxt += 2;
        bb = v >> sh;
        bc = 64 - sh;
    }
    __device__ __forceinline__ uint64_t pos() const { return nxt * 32 - bc; }
    __device__ __forceinline__ void refill(const Stream &S) {
        if (bc <= 32) {
            bb |= (uint64_t)S.ld(nxt++) << bc;
            bc += 32;
        }
    }
    __device__ __forceinline__ void drop(uint32_t n) {
        bb >>= n;
        bc -= n;
    }
};

// ---- Huffman tables in LDS --------------------------------------------------------------------------
// Per code: count[len] (count[0] = unused symbols), first[len] = the first canonical code of that length
// and offs[len] = its first symbol's index in sym[] (puff's running `first` / `index`), the symbols in
// canonical order, and a root table of 2^root entries (codes up to `root` bits in one lookup).
struct alignas(16) Tabs {
    uint32_t lit[1u << kRoot];
    uint32_t dist[1u << kDRoot];
    uint16_t lcount[16], dcount[16], lfirst[16], dfirst[16], loffs[16], doffs[16];
    uint16_t lsym[288], dsym[32];
    uint8_t lens[320];
};
static_assert(sizeof(Tabs) % 16 == 0 && sizeof(Tabs) <= kPinfTabBytes, "PinfArgs::tabs slot");

__device__ __forceinline__ uint32_t entry_of(uint32_t s, bool litlen) {
    if (litlen) {
        if (s < 256) return s;
        if (s == 256) return kTyEob;
        if (s < 286) {   // RFC 1951 3.2.5's length table in closed form (no constant-memory load)
            const uint32_t k = s - 257, x = k < 8 || k == 28 ? 0u : (k - 8) / 4 + 1;
            const uint32_t base = k == 28 ? 258u : k < 8 ? 3 + k : ((4 + (k & 3)) << x) + 3;
            return base | x << 20 | kTyLen;
        }
        return kTyBad;
    }
    if (s < 30) {   // and its distance table
        const uint32_t x = s < 4 ? 0u : s / 2 - 1, base = s < 4 ? 1 + s : ((2 + (s & 1)) << x) + 1;
        return base | x << 20;
    }
    return kTyBad;
}

// Counts, first codes, offsets and canonical symbol order of n lengths, by one wavefront (ballot ranks).
// Returns puff's `left`: 0 complete, > 0 incomplete, < 0 over-subscribed.
__device__ int code_counts(const uint8_t *lens, uint32_t n, uint16_t *count, uint16_t *first, uint16_t *offs,
                           uint16_t *sym, uint32_t lane) {
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
    uint32_t of[16], fi[16];
    of[0] = fi[0] = 0;
    of[1] = fi[1] = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
        left <<= 1;
        left -= (int)cnt[l];
        over |= left < 0;
        if (l < 15) {
            of[l + 1] = of[l] + cnt[l];
            fi[l + 1] = (fi[l] + cnt[l]) << 1;
        }
    }
    if (lane < 16) {
        uint32_t c = 0, f = 0, o = 0;
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            c = lane == (uint32_t)l ? cnt[l] : c;
            f = lane == (uint32_t)l ? fi[l] : f;
            o = lane == (uint32_t)l ? of[l] : o;
        }
        count[lane] = (uint16_t)c;
        first[lane] = (uint16_t)f;
        offs[lane] = (uint16_t)o;
    }
    if (over) return -1;
    uint32_t run[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) run[l] = 0;
    const uint64_t lt = (1ull << lane) - 1;
    for (uint32_t b0 = 0; b0 < n; b0 += 64) {
        const uint32_t s = b0 + lane;
        const uint32_t l = s < n ? lens[s] : 0;
        uint32_t rank = 0, off = 0;
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            const uint64_t m = __ballot(l == (uint32_t)q);
            if (l == (uint32_t)q) {
                rank = run[q] + (uint32_t)__popcll(m & lt);
                off = of[q];
            }
            run[q] += (uint32_t)__popcll(m);
        }
        if (l) sym[off + rank] = (uint16_t)s;
    }
    return left;
}

// The canonical decode of the bits `b` (LSB first) with codes of length lo..hi only: the entry (length in
// bits 16-19), or 0 when no code of those lengths is a prefix of b.
__device__ __forceinline__ uint32_t canon(uint32_t b, const uint16_t *count, const uint16_t *first, const uint16_t *offs,
                                          const uint16_t *sym, bool litlen, int lo, int hi) {
    uint32_t code = 0, e = 0;
#pragma unroll
    for (int len = 1; len < 16; ++len) {
        code = code << 1 | ((b >> (len - 1)) & 1);
        if (len >= lo && len <= hi && e == 0 && code < (uint32_t)first[len] + count[len])
            e = entry_of(sym[offs[len] + code - first[len]], litlen) | (uint32_t)len << 16;
    }
    return e;
}

// Both codes of a block from T.lens, by every thread of the workgroup: counts by wave 0, then the root
// tables filled in parallel, one entry per thread and step.  Returns (the same for all threads) whether
// both codes are acceptable as oracle_inflate's construct() judges them: not over-subscribed, and
// incomplete only with a single code.
__device__ bool build_tabs(Tabs &T, uint32_t nl, uint32_t nd) {
    __shared__ int s_left[2];
    const uint32_t t = threadIdx.x;
    if (t < 64) {
        const int a = code_counts(T.lens, nl, T.lcount, T.lfirst, T.loffs, T.lsym, t);
        const int b = code_counts(T.lens + nl, nd, T.dcount, T.dfirst, T.doffs, T.dsym, t);
        if (t == 0) {
            s_left[0] = a;
            s_left[1] = b;
        }
    }
    __syncthreads();
    const int l0 = s_left[0], l1 = s_left[1];
    const bool ok = !(l0 < 0 || (l0 > 0 && nl != (uint32_t)T.lcount[0] + T.lcount[1])) &&
                    !(l1 < 0 || (l1 > 0 && nd != (uint32_t)T.dcount[0] + T.dcount[1]));
    if (ok) {
        for (uint32_t i = t; i < (1u << kRoot); i += blockDim.x)
            T.lit[i] = canon(i, T.lcount, T.lfirst, T.loffs, T.lsym, true, 1, kRoot);
        for (uint32_t i = t; i < (1u << kDRoot); i += blockDim.x)
            T.dist[i] = canon(i, T.dcount, T.dfirst, T.doffs, T.dsym, false, 1, kDRoot);
    }
    __syncthreads();
    return ok;
}

// A code longer than the root (or no code at all): the lengths root+1..15 from the same bits.
__device__ __forceinline__ uint32_t slow_decode(uint64_t bb, const uint16_t *count, const uint16_t *first,
                                                const uint16_t *offs, const uint16_t *sym, bool litlen, int root) {
    const uint32_t e = canon((uint32_t)bb, count, first, offs, sym, litlen, root + 1, 15);
    return e ? e : kTyBad | 1u << 16;
}

// A lane's sources, written four at a time: entries gather in registers for the aligned quad that holds
// the next position and leave as one 16-byte store once the quad is full (a lane's first and last quads,
// which it may share with its neighbours, go out entry by entry).
struct SrcOut {
    uint32_t *p;
    uint64_t o, o0;                // next position, the lane's first
    uint32_t b0, b1, b2, b3;
    __device__ __forceinline__ void put(uint32_t v) {
        const uint32_t k = (uint32_t)o & 3;
        b0 = k == 0 ? v : b0;
        b1 = k == 1 ? v : b1;
        b2 = k == 2 ? v : b2;
        b3 = k == 3 ? v : b3;
        ++o;
        if ((o & 3) == 0) {
            const uint64_t q = o - 4;
            if (q >= o0) {
                gst<uint4>(p + q, make_uint4(b0, b1, b2, b3));
            } else {
                if (q + 0 >= o0) p[q + 0] = b0;
                if (q + 1 >= o0) p[q + 1] = b1;
                if (q + 2 >= o0) p[q + 2] = b2;
                p[q + 3] = b3;
            }
        }
    }
    __device__ __forceinline__ void finish() {   // the partial last quad
        const uint64_t q = o & ~3ull;
        const uint32_t k = (uint32_t)o & 3;
        if (k > 0 && q + 0 >= o0) p[q + 0] = b0;
        if (k > 1 && q + 1 >= o0) p[q + 1] = b1;
        if (k > 2 && q + 2 >= o0) p[q + 2] = b2;
    }
    // n positions written by someone else (a long match k_pinf_expand fills): flush, restart past them
    __device__ __forceinline__ void skip(uint64_t n) {
        finish();
        o += n;
        o0 = o;
    }
};
constexpr uint32_t kLongMatch = kPinfLongMatch;   // matches at least this long are expanded by k_pinf_expand

// One lane: decode symbols from the reader's position until the first symbol boundary at or past `stop`
// (0), the end-of-block code (1, *exit after it) or an error (2).  *bytes = output bytes of the symbols
// decoded.  EMIT: also write each byte's source at src[o0 + ...] (and check distances against o0).
template <bool EMIT>
__device__ uint32_t run_lane(const Tabs &T, const Stream &S, Bits &br, uint64_t stop, uint64_t end_bits,
                             uint64_t *exit, uint64_t *bytes, uint32_t *src, uint64_t o0, const PinfArgs *pa = nullptr,
                             uint64_t limit = 0, uint32_t *stat = nullptr, lds_u64p rec = nullptr,
                             uint32_t *n_rec = nullptr, uint64_t mid_at = ~0ull, uint64_t *mid = nullptr) {
    // stat (EMIT, RDX_PINF_PROF): symbols, decodes past the root table, refills from L2 instead of LDS
    uint32_t n_sym = 0, n_slow = 0, n_glob = 0;
    SrcOut out;
    if (EMIT) {
        out.p = src;
        out.o = out.o0 = o0;
        out.b0 = out.b1 = out.b2 = out.b3 = 0;
    }
    uint64_t nb = 0;
    uint32_t r = 0;
    // `stop` is used before the loop, as a distance: a value still in flight from a global load at the loop
    // header made the compiler wait for every outstanding memory operation there — with EMIT, for the
    // lane's source stores of the previous symbols, a round trip to memory per symbol
    const uint64_t p0 = br.pos();
    const uint64_t run = stop > p0 ? stop - p0 : 0;
    for (;;) {
        const uint64_t p = br.pos();
        if (p > end_bits) {
            r = 2;
            break;
        }
        if (p - p0 >= run) break;
        if (!EMIT && mid && p >= mid_at && *mid == ~0ull) *mid = p | nb << 40;   // (k_pinf_block: the lane's middle)
        if (EMIT && stat) {
            ++n_sym;
            n_glob += br.bc <= 32 && br.nxt - S.l0 >= S.ln ? 1u : 0u;
        }
        br.refill(S);
        uint32_t e = T.lit[(uint32_t)br.bb & ((1u << kRoot) - 1)];
        if (EMIT && stat) n_slow += ((e >> 16) & 15) == 0 ? 1u : 0u;
        if (((e >> 16) & 15) == 0) e = slow_decode(br.bb, T.lcount, T.lfirst, T.loffs, T.lsym, true, kRoot);
        br.drop((e >> 16) & 15);
        const uint32_t ty = e & (3u << 24);
        if (ty == 0) {
            if (EMIT) {
                if (o0 + nb >= limit) {   // more output than the block decode counted for this lane
                    r = 2;
                    break;
                }
                out.put(kFlag | (e & 0xff));
            }
            ++nb;
            continue;
        }
        if (ty == kTyEob) {
            r = br.pos() > end_bits ? 2 : 1;
            break;
        }
        if (ty == kTyBad) {
            r = 2;
            break;
        }
        const uint32_t lx = (e >> 20) & 15;
        const uint32_t len = (e & 0xffff) + ((uint32_t)br.bb & ((1u << lx) - 1));
        br.drop(lx);
        br.refill(S);
        uint32_t d = T.dist[(uint32_t)br.bb & ((1u << kDRoot) - 1)];
        if (EMIT && stat) n_slow += ((d >> 16) & 15) == 0 ? 1u : 0u;
        if (((d >> 16) & 15) == 0) d = slow_decode(br.bb, T.dcount, T.dfirst, T.doffs, T.dsym, false, kDRoot);
        if ((d & (3u << 24)) == kTyBad) {
            r = 2;
            break;
        }
        br.drop((d >> 16) & 15);
        const uint32_t dx = (d >> 20) & 15;
        const uint32_t dist = (d & 0xffff) + ((uint32_t)br.bb & ((1u << dx) - 1));
        br.drop(dx);
        if (EMIT) {
            const uint64_t q = o0 + nb;
            if (dist > q || q + len > limit) {   // before the start of the output (RDX_INFLATE_DISTANCE), or
                r = 2;                           // more output than the block decode counted for this lane
                break;
            }
            const uint32_t base = (uint32_t)(q - dist);
            uint32_t slot = ~0u;
            if (len >= kLongMatch) {   // a wavefront of k_pinf_expand writes it, 64 entries per store
                slot = atomicAdd(&pa->state->n_match, 1u);
                if (slot < pa->mcap) pa->mlist[slot] = make_uint4((uint32_t)q, len, dist, 0);
            }
            if (slot < pa->mcap) {
                out.skip(len);
            } else if (rec && *n_rec < kEmitRecs) {
                rec[*n_rec * kEmitThreads] = q | (uint64_t)(len | dist << 16) << 32;
                ++*n_rec;
                out.skip(len);
            } else if (dist >= len) {
                for (uint32_t j = 0; j < len; ++j) out.put(base + j);
            } else {   // overlapping: byte j repeats byte (j mod dist) of the dist bytes before the match
                uint32_t m = 0;
                for (uint32_t j = 0; j < len; ++j) {
                    out.put(base + m);
                    m = m + 1 == dist ? 0 : m + 1;
                }
            }
        }
        nb += len;
    }
    if (EMIT) out.finish();
    if (EMIT && stat) {
        stat[0] = n_sym;
        stat[1] = n_slow;
        stat[2] = n_glob;
    }
    *exit = br.pos();
    *bytes = nb;
    return r;
}

// The finder's strict dynamic-header test at bit p (a zlib encoder's header: complete codes), in
// registers only (one thread per bit offset; no per-lane arrays, so no scratch): the code-length code as
// per-length counts and its symbols packed 5 bits each in (len, symbol) order; the literal / length and
// distance code lengths are never stored, only summed into their Kraft sums as they are decoded.
template <class SRC>
__device__ bool dyn_candidate(const SRC &S, uint64_t p, uint64_t end_bits) {
    const uint32_t h = S.at(p);
    if (((h >> 1) & 3) != 2 || ((h >> 3) & 31) > 29 || ((h >> 8) & 31) > 29) return false;
    const uint32_t nc = ((h >> 13) & 15) + 4;
    uint64_t cb = (uint64_t)S.at(p + 17) | (uint64_t)S.at(p + 49) << 32;
    cb &= (1ull << (3 * nc)) - 1;   // fields past HCLEN + 4 are zero lengths
    return dyn_candidate_rest(S, p, end_bits, h, cb);
}

// The finder only (never the block parse, which accepts whatever oracle_inflate accepts): code-length
// sequences that zlib's encoder (scan_tree / send_tree in trees.c, and GNU gzip's and miniz's, which run-length
// code the same way) never writes.  A run of equal lengths is coded as few symbols as its rules allow, so a
// run of zeros is 17 (3-10) or 18 (11-138) and only a remainder below 3 (at most 2 zeros, after an 18 or
// alone) is written out; 16 repeats only a nonzero length; after a 17 the run has ended, so a nonzero length
// follows; a run of a nonzero length is written out only up to three times (longer ones become 16s).  A false survivor in random bits breaks one of these within a few symbols, where its Kraft sums
// could only reject it after ~300 (the finder's slowest workgroup decoded one of those per lane).  A real
// block whose encoder codes runs otherwise is not listed: the chain then reaches it as a miss, which the host
// decodes (k_pinf_chain, pinflate_stream).
#ifndef RDX_PINF_FIND_RLE
#define RDX_PINF_FIND_RLE 1
#endif
constexpr bool kFindRle = RDX_PINF_FIND_RLE != 0;
// `same`: explicit repeats of the previous nonzero length so far (counted within one code: zlib sends the
// literal / length and distance lengths as two sequences, so three explicit L may end one and a fourth
// start the other); `first_dist`: this symbol starts the distance lengths.
__device__ __forceinline__ bool rle_impossible(uint32_t sym, uint32_t psym, uint32_t z0, uint32_t prev, uint32_t same,
                                               bool first_dist) {
    const bool zero_after_zero = sym == 0 && psym == 0 && z0 >= 2;    // a third explicit zero
    const bool after17 = psym == 17 && (sym == 0 || sym >= 16);       // a zero run continued after a 17
    const bool after0 = psym == 0 && sym >= 17;                       // 17 / 18 after explicit zeros
    const bool rep_zero = sym == 16 && prev == 0;                     // 16 repeating a zero length
    const bool fourth = sym - 1u < 15u && sym == psym && same >= 2 && !first_dist;   // a fourth explicit L
    return zero_after_zero || after17 || after0 || rep_zero || fourth;
}
__device__ __forceinline__ uint32_t rle_same(uint32_t sym, uint32_t psym, uint32_t same, bool first_dist) {
    return sym - 1u < 15u && sym == psym && !first_dist ? same + 1 : 0u;
}

// A dynamic header's code lengths (STORE: into lens[]) with oracle_inflate's rules — a complete
// code-length code, no repeat (16) first, no run past HLIT + HDIST, no over-subscribed literal / length or
// distance code — and their Kraft sums (kl, kd: x 2^15), the distance codes used, whether the end-of-block
// code has a length.  Written for one header per lane of a wave (the finder's survivors; thread 0 of
// k_pinf_block's parse): the code-length code as packed registers — per-length region starts S_l and symbol
// offsets O_l in the space of the 7 peeked bits read MSB first (canonical codes of one length are one
// contiguous region, lengths in increasing order), the symbols 5 bits each in canonical order — so a
// symbol is one bit reversal, six compares and two packed lookups; every step is branch-free (one
// exec mask for the lanes still decoding), where the per-length walk with early returns compiled to
// ~170 instructions of exec-mask branches per symbol.
template <bool STORE, class SRC>
__device__ __forceinline__ bool header_lengths(const SRC &S, uint64_t &pos, uint64_t end_bits, uint64_t cb, uint32_t nl,
                                               uint32_t nd, uint8_t *lens, uint32_t &kl, uint32_t &kd, uint32_t &used_d,
                                               bool &eob) {
    constexpr int kField[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};   // symbol -> field
    uint64_t cnt = 0;   // byte l: codes of length l
#pragma unroll
    for (int i = 0; i < 19; ++i) cnt += 1ull << (8 * ((cb >> (3 * i)) & 7));
    int left = 1;
    uint64_t Sp = 0, Op = 0;   // byte l: S_l, O_l
    uint32_t st = 0, of = 0;
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        const uint32_t c = (uint32_t)(cnt >> (8 * l)) & 0xff;
        left = (left << 1) - (int)c;
        Sp |= (uint64_t)st << (8 * l);
        Op |= (uint64_t)of << (8 * l);
        st += c << (7 - l);
        of += c;
    }
    if (left != 0) return false;   // over-subscribed or incomplete (construct() != 0)
    uint64_t pk0 = 0, pk1 = 0, run = 0;
#pragma unroll
    for (int sy = 0; sy < 19; ++sy) {
        const uint32_t l = (uint32_t)(cb >> (3 * kField[sy])) & 7;
        const uint32_t r = (uint32_t)((Op + run) >> (8 * l)) & 0xff;   // (bytes <= 38: no carries)
        run += l ? 1ull << (8 * l) : 0;
        pk0 |= l && r < 12 ? (uint64_t)sy << (5 * r) : 0;
        pk1 |= l && r >= 12 ? (uint64_t)sy << (5 * (r - 12)) : 0;
    }
    const uint64_t E = Sp >> 16;   // byte l-1: S_{l+1}, the end of length l's region (l = 1..6)
    const uint32_t total = nl + nd;
    uint64_t nxt = pos >> 5;
    uint64_t bb = ((uint64_t)S.ld(nxt) | (uint64_t)S.ld(nxt + 1) << 32) >> (pos & 31);
    uint32_t bc = 64 - (uint32_t)(pos & 31);
    nxt += 2;
    uint32_t idx = 0, prev = 0, psym = 19, z0 = 0, same = 0;
    kl = kd = used_d = 0;
    eob = false;
    bool bad = false, live = true;
    uint32_t w = S.ld(nxt);   // the next dword, loaded one refill ahead (off the symbol's dependency chain)
    while (__builtin_amdgcn_ballot_w64(live)) {
        if (live) {
            const bool need = bc < 32;
            bb |= need ? (uint64_t)w << (bc & 63) : 0;
            bc += need ? 32 : 0;
            nxt += need ? 1 : 0;
            if (need) w = S.ld(nxt);
            const uint32_t j = __builtin_bitreverse32((uint32_t)bb) >> 25;
            uint32_t len = 1;
#pragma unroll
            for (int l = 0; l < 6; ++l) len += ((uint32_t)(E >> (8 * l)) & 0xff) <= j ? 1u : 0u;
            const uint32_t Sl = (uint32_t)(Sp >> (8 * len)) & 0xff, Ol = (uint32_t)(Op >> (8 * len)) & 0xff;
            const uint32_t si = Ol + ((j - Sl) >> (7 - len));
            const uint32_t sym = (uint32_t)(si < 12 ? pk0 >> (5 * si) : pk1 >> (5 * (si - 12))) & 31;
            const uint32_t x = (uint32_t)(bb >> len);
            const bool s16 = sym == 16, s17 = sym == 17, s18 = sym == 18;
            const uint32_t rep = s16 ? 3 + (x & 3) : s17 ? 3 + (x & 7) : s18 ? 11 + (x & 127) : 1;
            const uint32_t used = len + (s16 ? 2 : s17 ? 3 : s18 ? 7 : 0);
            const uint32_t val = s16 ? prev : (s17 || s18) ? 0 : sym;
            bad |= (s16 && idx == 0) || idx + rep > total;
            if (!STORE && kFindRle) {
                bad |= rle_impossible(sym, psym, z0, prev, same, idx == nl);
                same = rle_same(sym, psym, same, idx == nl);
                z0 = sym == 0 ? z0 + 1 : 0;
                psym = sym;
            }
            if (STORE && !bad && val)   // (lens[] is zeroed by the caller: runs of zeros write nothing)
                for (uint32_t r = 0; r < rep; ++r) lens[idx + r] = (uint8_t)val;
            const uint32_t nlit = idx < nl ? min(rep, nl - idx) : 0u, ndst = rep - nlit;
            eob |= idx <= 256 && 256 < idx + nlit && val != 0;
            const uint32_t sh = 15 - val;
            kl += val ? nlit << sh : 0u;
            kd += val ? ndst << sh : 0u;
            used_d += val ? ndst : 0u;
            bad |= kl > (1u << 15) || kd > (1u << 15);
            pos += used;
            bb >>= used;
            bc -= used;
            idx += rep;
            prev = val;
            bad |= pos > end_bits;
            live = !bad && idx < total;
        }
    }
    return !bad;
}

// The same by the 64 lanes of one wave together (k_pinf_block's parse, k_pinf_find's open survivors: one
// lane decoding ~300 symbols took 70-120 us, every step waiting on the previous one's latency).  Per 64-bit
// window: lane k decodes the symbol that would start at bit pos + k (all 64 candidates at once); the chain
// of actual symbols is followed with uniform lane reads, a few instructions a symbol; then every symbol's
// effect at once on its lane — its table index by a prefix of the repeat counts, the value a 16 repeats,
// the stores of its run, the Kraft sums by reductions (they only grow, so a sum past 1 at the window's end
// is one past 1 at some symbol).  Same rules and results as header_lengths<true>; every lane returns the
// same values.
template <class SRC>
__device__ bool header_lengths_wave(const SRC &S, uint64_t &pos_io, uint64_t end_bits, uint64_t cb, uint32_t nl,
                                    uint32_t nd, uint8_t *lens, uint32_t &kl_o, uint32_t &kd_o, uint32_t &used_d_o,
                                    bool &eob_o) {
    constexpr int kField[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};
    const uint32_t lane = threadIdx.x & 63;
    uint64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < 19; ++i) cnt += 1ull << (8 * ((cb >> (3 * i)) & 7));
    int left = 1;
    uint64_t Sp = 0, Op = 0;
    uint32_t st = 0, of = 0;
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        const uint32_t c = (uint32_t)(cnt >> (8 * l)) & 0xff;
        left = (left << 1) - (int)c;
        Sp |= (uint64_t)st << (8 * l);
        Op |= (uint64_t)of << (8 * l);
        st += c << (7 - l);
        of += c;
    }
    if (left != 0) return false;
    uint64_t pk0 = 0, pk1 = 0, run = 0;
#pragma unroll
    for (int sy = 0; sy < 19; ++sy) {
        const uint32_t l = (uint32_t)(cb >> (3 * kField[sy])) & 7;
        const uint32_t r = (uint32_t)((Op + run) >> (8 * l)) & 0xff;
        run += l ? 1ull << (8 * l) : 0;
        pk0 |= l && r < 12 ? (uint64_t)sy << (5 * r) : 0;
        pk1 |= l && r >= 12 ? (uint64_t)sy << (5 * (r - 12)) : 0;
    }
    const uint64_t E = Sp >> 16;
    const uint32_t total = nl + nd;
    const uint64_t below = (1ull << lane) - 1;
    uint64_t pos = pos_io;
    uint32_t idx = 0, prev = 0, kl = 0, kd = 0, used_d = 0;
    bool eob = false, bad = false;
    while (!bad && idx < total) {
        // this window: lane k decodes the symbol that would start at bit pos + k
        const uint32_t v = S.at(pos + lane);
        const uint32_t j = __builtin_bitreverse32(v) >> 25;
        uint32_t len = 1;
#pragma unroll
        for (int l = 0; l < 6; ++l) len += ((uint32_t)(E >> (8 * l)) & 0xff) <= j ? 1u : 0u;
        const uint32_t Sl = (uint32_t)(Sp >> (8 * len)) & 0xff, Ol = (uint32_t)(Op >> (8 * len)) & 0xff;
        const uint32_t si = Ol + ((j - Sl) >> (7 - len));
        const uint32_t sym = (uint32_t)(si < 12 ? pk0 >> (5 * si) : pk1 >> (5 * (si - 12))) & 31;
        const uint32_t x = v >> len;
        const uint32_t rep = sym == 16 ? 3 + (x & 3) : sym == 17 ? 3 + (x & 7) : sym == 18 ? 11 + (x & 127) : 1;
        const uint32_t used = len + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
        // the actual symbols: the chain from lane 0 (uniform lane reads, a few instructions a symbol)
        uint64_t M = 0;
        uint32_t c = 0;
        while (c < 64) {
            M |= 1ull << c;
            c += (uint32_t)__builtin_amdgcn_readlane((int)used, (int)c);
        }
        const bool member = (M >> lane) & 1;
        // their table indices: an exclusive prefix of the repeat counts over the chain
        uint32_t incl = member ? rep : 0u;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= (uint32_t)d) incl += o;
        }
        const uint32_t at = idx + incl - (member ? rep : 0u);
        const bool valid = member && at < total;   // (chain symbols past the header are body bits)
        // 16 repeats the value of the last symbol before it that is not a 16 (or the previous window's)
        const uint32_t own = sym < 16 ? sym : 0u;
        const uint64_t src = __ballot(member && sym != 16) & below;
        const int sl = src ? 63 - __builtin_clzll(src) : 0;
        const uint32_t from = (uint32_t)__shfl((int)own, sl, 64);
        const uint32_t val = sym == 16 ? (src ? from : prev) : own;
        const uint32_t nlit = at < nl ? min(rep, nl - at) : 0u, ndst = rep - nlit;
        const bool fault = valid && ((sym == 16 && at == 0) || at + rep > total || pos + lane + used > end_bits);
        if (valid && val && at + rep <= total)   // (lens[] is zeroed by the caller)
            for (uint32_t r = 0; r < rep; ++r) lens[at + r] = (uint8_t)val;
        uint32_t skl = valid && val ? nlit << (15 - val) : 0u, skd = valid && val ? ndst << (15 - val) : 0u;
        uint32_t sud = valid && val ? ndst : 0u;
#pragma unroll
        for (int d = 32; d; d >>= 1) {
            skl += (uint32_t)__shfl_xor((int)skl, d, 64);
            skd += (uint32_t)__shfl_xor((int)skd, d, 64);
            sud += (uint32_t)__shfl_xor((int)sud, d, 64);
        }
        kl += skl;
        kd += skd;
        used_d += sud;
        eob |= __ballot(valid && at <= 256 && 256 < at + nlit && val != 0) != 0;
        bad = __ballot(fault) != 0 || kl > (1u << 15) || kd > (1u << 15);
        // on past the last valid symbol
        const uint64_t vm = __ballot(valid);
        const int last = 63 - __builtin_clzll(vm);
        pos += (uint32_t)__builtin_amdgcn_readlane((int)(lane + used), last);
        idx = (uint32_t)__builtin_amdgcn_readlane((int)(at + rep), last);
        prev = (uint32_t)__builtin_amdgcn_readlane((int)val, last);
    }
    pos_io = pos;
    kl_o = kl;
    kd_o = kd;
    used_d_o = used_d;
    eob_o = eob;
    return !bad;
}

// A block header at bit p (its BFINAL bit) parsed the way oracle_inflate does, by the 64 lanes of wave 0
// (k_pinf_block).  type 1: fixed lengths, 2: dynamic (code lengths into T.lens).  Returns false on any
// error; *body = first bit of the body, *nlen / *ndist the code counts; the same results in every lane.
__device__ bool parse_header_wave(const Stream &S, uint64_t p, uint32_t type, uint64_t end_bits, Tabs &T, uint64_t *body,
                                  uint32_t *nlen, uint32_t *ndist) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t pos = p + 3;
    if (type == 1) {
        for (uint32_t s = lane; s < 320; s += 64) T.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : s < 318 ? 5 : 0;
        *nlen = 288;
        *ndist = 30;
        *body = pos;
        return pos <= end_bits;
    }
    const uint32_t h = S.at(pos);
    const uint32_t nl = (h & 31) + 257, nd = ((h >> 5) & 31) + 1, nc = ((h >> 10) & 15) + 4;
    pos += 14;
    if (nl > 286 || nd > 30) return false;
    for (uint32_t i = lane; i < 320; i += 64) T.lens[i] = 0;
    const uint64_t cb = ((uint64_t)S.at(pos) | (uint64_t)S.at(pos + 32) << 32) & ((1ull << (3 * nc)) - 1);
    pos += 3 * nc;
    uint32_t kl, kd, used_d;
    bool eob;
    // (the codes' completeness is judged by build(), as construct() does in the oracle)
    if (!header_lengths_wave(S, pos, end_bits, cb, nl, nd, T.lens, kl, kd, used_d, eob) || !eob) return false;
    *nlen = nl;
    *ndist = nd;
    *body = pos;
    return true;
}

template <class SRC>
__device__ bool dyn_candidate_rest(const SRC &S, uint64_t p, uint64_t end_bits, uint32_t h, uint64_t cb) {
    const uint32_t nl = ((h >> 3) & 31) + 257, nd = ((h >> 8) & 31) + 1, nc = ((h >> 13) & 15) + 4;
    uint64_t pos = p + 17 + 3 * nc;
    uint32_t kl, kd, used_d;
    bool eob;
    if (!header_lengths<false>(S, pos, end_bits, cb, nl, nd, nullptr, kl, kd, used_d, eob)) return false;
    return eob && kl == (1u << 15) && (kd == (1u << 15) || used_d <= 1);
}

// ---- 1. candidates ------------------------------------------------------------------------------------
// A workgroup tests the bit offsets of kFindBytes bytes and each of those bytes as the LEN of a stored
// block.  The bytes and the longest header behind them (<= 4500 bits) are staged in LDS first and read from
// there only (a surviving offset decodes its header symbol by symbol: each dependent read from L2 would
// cost the lane a round trip).  Rounds of 1024 bytes, 4 per thread: the 32 offsets of a thread are screened
// without branches (BTYPE, HLIT, HDIST, then the code-length code's Kraft sum), and the survivors (about
// one offset in a thousand) go to a list in LDS; the list's headers are then decoded one per lane, so that
// no lane waits on another's survivors.  No global atomics but the rare candidates' (one counter shared
// by every workgroup serialises in L2: a per-wave atomic cost 150 us on a 3.5 MB stream, profiles/r04_*).
constexpr uint32_t kFindBytes = 8192, kFindLook = 640;
constexpr uint32_t kFindWin = (kFindBytes + kFindLook) / 4 + 4;
constexpr uint32_t kFindList = 8192 + 256;   // a round adds at most 8192; decoded once it holds 256
#ifndef RDX_PINF_FIND_LANESYMS
#define RDX_PINF_FIND_LANESYMS 32   // code-length symbols a lane decodes before a wave takes over (0: all)
#endif
constexpr uint32_t kFindLaneSyms = RDX_PINF_FIND_LANESYMS;

struct WinStream {   // bit reads from the staged window only (positions inside it by construction)
    lds_u32p lds;
    uint64_t l0;
    __device__ __forceinline__ uint32_t ld(uint64_t i) const { return lds[min((uint32_t)(i - l0), kFindWin - 1)]; }
    __device__ __forceinline__ uint32_t at(uint64_t p) const {
        const uint32_t i = min((uint32_t)((p >> 5) - l0), kFindWin - 2);
        const uint64_t v = (uint64_t)lds[i] | (uint64_t)lds[i + 1] << 32;
        return (uint32_t)(v >> (p & 31));
    }
};

// The survivors' header test with the code-length code expanded first into a 128-entry table (one byte per
// 7-bit MSB-first peek: symbol | length << 5) in the lane's own LDS slot, so a code-length symbol is one
// table read instead of header_lengths' compares and packed lookups (~170 instructions per symbol with the
// exec-mask bookkeeping, and the workgroup holding a real header walks ~250 of them).  Same rules and
// result as dyn_candidate_rest.
#ifndef RDX_PINF_FIND_LUT
#define RDX_PINF_FIND_LUT 1
#endif
typedef __attribute__((address_space(3))) uint8_t *lds_u8p;
typedef __attribute__((address_space(3))) uint32_t *lds_u32w;
constexpr uint32_t kFindLutStride = 132;   // bytes per lane's table: 33 dwords, lanes in different banks
static_assert(kFindList * 4 >= 256 * kFindLutStride, "the survivor list's memory holds 256 tables");

// Returns kCandNo / kCandYes, or kCandOpen when the header is still consistent after `cap` code-length symbols
// (a real header, almost always, once the run-length rules have thrown out false ones: a whole wave then
// decides it, header_lengths_wave — one lane walking a real header's ~300 symbols was the finder's slowest
// step).
enum : uint32_t { kCandNo = 0, kCandYes = 1, kCandOpen = 2 };
__device__ uint32_t dyn_candidate_lut(const WinStream &S, uint64_t p, uint64_t end_bits, uint32_t h, uint64_t cb,
                                      lds_u8p lut, uint32_t cap) {
    constexpr int kField[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};   // symbol -> field
    const uint32_t nl = ((h >> 3) & 31) + 257, nd = ((h >> 8) & 31) + 1, nc = ((h >> 13) & 15) + 4;
    uint64_t pos = p + 17 + 3 * nc;
    uint64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < 19; ++i) cnt += 1ull << (8 * ((cb >> (3 * i)) & 7));
    int left = 1;
    uint64_t Sp = 0, Op = 0;
    uint32_t st = 0, of = 0;
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        const uint32_t c = (uint32_t)(cnt >> (8 * l)) & 0xff;
        left = (left << 1) - (int)c;
        Sp |= (uint64_t)st << (8 * l);
        Op |= (uint64_t)of << (8 * l);
        st += c << (7 - l);
        of += c;
    }
    if (left != 0) return kCandNo;
    uint64_t pk0 = 0, pk1 = 0, run = 0;
#pragma unroll
    for (int sy = 0; sy < 19; ++sy) {
        const uint32_t l = (uint32_t)(cb >> (3 * kField[sy])) & 7;
        const uint32_t r = (uint32_t)((Op + run) >> (8 * l)) & 0xff;
        run += l ? 1ull << (8 * l) : 0;
        pk0 |= l && r < 12 ? (uint64_t)sy << (5 * r) : 0;
        pk1 |= l && r >= 12 ? (uint64_t)sy << (5 * (r - 12)) : 0;
    }
    // the table by runs: a code of length l is one run of 2^(7-l) entries of the 7-bit space, the codes of one
    // length consecutive from S_l (a complete code fills all 128), runs of 4 or more as dword stores
#pragma unroll
    for (uint32_t l = 1; l < 8; ++l) {
        const uint32_t c = (uint32_t)(cnt >> (8 * l)) & 0xff;
        const uint32_t S0 = (uint32_t)(Sp >> (8 * l)) & 0xff, O0 = (uint32_t)(Op >> (8 * l)) & 0xff;
        constexpr uint32_t kSpan[8] = {0, 64, 32, 16, 8, 4, 2, 1};
        const uint32_t span = kSpan[l];
        for (uint32_t k = 0; k < c; ++k) {
            const uint32_t si = O0 + k;
            const uint32_t v = ((uint32_t)(si < 12 ? pk0 >> (5 * si) : pk1 >> (5 * (si - 12))) & 31) | l << 5;
            const uint32_t st = S0 + k * span;
            if (span >= 4) {
                for (uint32_t q = 0; q < span; q += 4) ((lds_u32w)lut)[(st + q) >> 2] = v * 0x01010101u;
            } else {
                for (uint32_t q = 0; q < span; ++q) lut[st + q] = (uint8_t)v;
            }
        }
    }
    const uint32_t total = nl + nd;
    uint64_t nxt = pos >> 5;
    uint64_t bb = ((uint64_t)S.ld(nxt) | (uint64_t)S.ld(nxt + 1) << 32) >> (pos & 31);
    uint32_t bc = 64 - (uint32_t)(pos & 31);
    nxt += 2;
    uint32_t idx = 0, prev = 0, kl = 0, kd = 0, used_d = 0, psym = 19, z0 = 0, nsym = 0, same = 0;
    bool eob = false, bad = false;
    uint32_t w = S.ld(nxt);
    while (!bad && idx < total && nsym++ < cap) {
        const bool need = bc < 32;
        bb |= need ? (uint64_t)w << (bc & 63) : 0;
        bc += need ? 32 : 0;
        nxt += need ? 1 : 0;
        if (need) w = S.ld(nxt);
        const uint32_t e = lut[__builtin_bitreverse32((uint32_t)bb) >> 25];
        const uint32_t len = e >> 5, sym = e & 31;
        const uint32_t x = (uint32_t)(bb >> len);
        const bool s16 = sym == 16, s17 = sym == 17, s18 = sym == 18;
        const uint32_t rep = s16 ? 3 + (x & 3) : s17 ? 3 + (x & 7) : s18 ? 11 + (x & 127) : 1;
        const uint32_t used = len + (s16 ? 2 : s17 ? 3 : s18 ? 7 : 0);
        const uint32_t val = s16 ? prev : (s17 || s18) ? 0 : sym;
        bad |= (s16 && idx == 0) || idx + rep > total;
        if (kFindRle) {
            bad |= rle_impossible(sym, psym, z0, prev, same, idx == nl);
            same = rle_same(sym, psym, same, idx == nl);
            z0 = sym == 0 ? z0 + 1 : 0;
            psym = sym;
        }
        const uint32_t nlit = idx < nl ? min(rep, nl - idx) : 0u, ndst = rep - nlit;
        eob |= idx <= 256 && 256 < idx + nlit && val != 0;
        const uint32_t sh = 15 - val;
        kl += val ? nlit << sh : 0u;
        kd += val ? ndst << sh : 0u;
        used_d += val ? ndst : 0u;
        bad |= kl > (1u << 15) || kd > (1u << 15);
        pos += used;
        bb >>= used;
        bc -= used;
        idx += rep;
        prev = val;
        bad |= pos > end_bits;
    }
    if (bad) return kCandNo;
    if (idx < total) return kCandOpen;
    return eob && kl == (1u << 15) && (kd == (1u << 15) || used_d <= 1) ? kCandYes : kCandNo;
}

__global__ __launch_bounds__(256) void k_pinf_find(PinfArgs a) {
    __shared__ uint32_t win[kFindWin];
    __shared__ uint32_t list[kFindList];   // survivors: bit offsets from 8 * q0
    __shared__ uint32_t n_list;
    __shared__ uint16_t kraft4[4096];      // Kraft sum (x128) of four 3-bit code-length fields
    __shared__ uint32_t open[256];         // survivors still consistent after kFindLaneSyms symbols
    __shared__ uint32_t n_open;
    __shared__ uint8_t wlens[4 * 320];     // a wave's code lengths while it decides one of them
    const uint32_t t = threadIdx.x, lane = t & 63;
    // RDX_PINF_PROF: (start, staged, last header pass, end, survivors) per workgroup, after k_pinf_emit's
    uint64_t *const prof = a.prof && blockIdx.x < kPinfMaxCand ? a.prof + 16ull * kPinfMaxCand + 8ull * blockIdx.x : nullptr;
    const uint64_t ts0 = prof ? wall_clock64() : 0;
    const Stream G = make_stream(a);
    const uint64_t q0 = a.first_byte + (uint64_t)blockIdx.x * kFindBytes;
    const uint64_t l0 = q0 >= 4 ? (q0 >> 2) - 1 : 0;
    for (uint32_t k = t; k < kFindWin; k += 256) win[k] = G.ldg(l0 + k);
    for (uint32_t e = t; e < 4096; e += 256) {
        uint32_t k = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t l = (e >> (3 * i)) & 7;
            k += l ? 128u >> l : 0u;
        }
        kraft4[e] = (uint16_t)k;
    }
    if (t == 0) n_list = 0;
    __syncthreads();
    WinStream S;
    S.lds = (lds_u32p)win;
    S.l0 = l0;
    PinfState *st = a.state;
    auto push = [&](uint64_t key) -> uint32_t {
        const uint32_t i = atomicAdd(&st->n_cand, 1u);
        if (i < kPinfMaxCand) a.cand[i] = key;
        else atomicOr(&st->overflow, 1u);
        return i;
    };
    const uint64_t ts1 = prof ? wall_clock64() : 0;
    uint64_t ts2 = 0;
    uint32_t survivors = 0;   // (thread 0: this workgroup's, for the tuning counter)
    uint64_t ts_open = 0;     // (RDX_PINF_PROF) the last pass's lane phase ended
    uint32_t opens = 0;       // survivors handed to whole waves
    for (uint32_t r = 0; r < kFindBytes / 1024; ++r) {
        // this thread's 4 bytes: consecutive, so their 32 offsets' bits come from one 64-bit window
        const uint64_t qt = q0 + 1024 * r + 4 * t;
        const uint64_t w64 = (uint64_t)S.at(8 * qt) | (uint64_t)S.at(8 * qt + 32) << 32;
        // all 32 offsets at once, bit b for offset b: BTYPE = 2 (bit b+1 clear, b+2 set), HLIT <= 29 (not bits
        // b+4..b+7 all set), HDIST <= 29 (not bits b+9..b+12 all set), inside the stream
        const uint64_t hl = (w64 >> 4) & (w64 >> 5) & (w64 >> 6) & (w64 >> 7);
        const uint64_t hd = (w64 >> 9) & (w64 >> 10) & (w64 >> 11) & (w64 >> 12);
        const uint64_t in = qt >= a.end_byte ? 0u : qt + 4 <= a.end_byte ? 0xffffffffu : (1u << (8 * (a.end_byte - qt))) - 1;
        uint32_t cheap = (uint32_t)(~(w64 >> 1) & (w64 >> 2) & ~hl & ~hd & in);
        // the code-length code's Kraft sum (about a fifth of the offsets get here)
        uint32_t mask = 0;
        while (cheap) {
            const uint32_t b = __builtin_ctz(cheap);
            cheap &= cheap - 1;
            const uint64_t p = 8 * qt + b;
            const uint32_t h = (uint32_t)(w64 >> b);
            const uint64_t cb = ((uint64_t)S.at(p + 17) | (uint64_t)S.at(p + 49) << 32) &
                                ((1ull << (3 * (((h >> 13) & 15) + 4))) - 1);
            const uint32_t kr = kraft4[cb & 0xfff] + kraft4[(cb >> 12) & 0xfff] + kraft4[(cb >> 24) & 0xfff] +
                                kraft4[(cb >> 36) & 0xfff] + kraft4[(cb >> 48) & 0xfff];
            mask |= kr == 128 ? 1u << b : 0u;
        }
        // append: one LDS atomic per wave
        const uint32_t cnt = __builtin_popcount(mask);
        uint32_t incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= (uint32_t)d) incl += o;
        }
        const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
        uint32_t base = 0;
        if (lane == 63 && tot) base = atomicAdd(&n_list, tot);
        base = (uint32_t)__shfl((int)base, 63, 64);
        uint32_t k = base + incl - cnt;
        while (mask) {
            const uint32_t b = __builtin_ctz(mask);
            mask &= mask - 1;
            list[k++] = (uint32_t)(8 * (qt - q0) + b);
        }
        // stored: LEN, NLEN at q, q+2; the two bits before q are zero (padding or BTYPE 00); the data fits
        for (uint32_t j = 0; j < 4; ++j) {
            const uint64_t q = qt + j;
            if (q >= a.first_byte + 1 && q + 4 <= a.end_byte) {
                const uint32_t v = S.at(8 * q - 8);   // byte q-1, LEN, NLEN (low 8 bits first)
                const uint32_t len = (v >> 8) & 0xffff;
                const uint32_t nlen = S.at(8 * q + 16) & 0xffff;
                if (len == (~nlen & 0xffff) && ((v >> 6) & 3) == 0 && q + 4 + len <= a.end_byte) push((8 * q) << 2 | 0);
            }
        }
        __syncthreads();
        const uint32_t n = n_list;
        if (n >= 256 || r + 1 == kFindBytes / 1024) {
            // the survivors' full header test, one per lane
            if (prof) ts2 = wall_clock64();
#ifndef RDX_PINF_FIND_HDR
#define RDX_PINF_FIND_HDR 1   // tuning probes: 0 skips the survivors' header decode (tools/probe_pinf_find)
#endif
#ifndef RDX_PINF_FIND_SPREAD
#define RDX_PINF_FIND_SPREAD 0   // tuning probes: 1 deals the survivors to the 4 waves round-robin
#endif
            if (RDX_PINF_FIND_LUT && RDX_PINF_FIND_HDR && n <= 256) {
                // one survivor per thread; the list's memory becomes the threads' tables once each has its
                // position
                const uint32_t mine = t < n ? list[t] : 0u;
                if (t == 0) n_open = 0;
                __syncthreads();
                if (t < n) {
                    const uint64_t p = 8 * q0 + mine;
                    const uint32_t h = S.at(p);
                    const uint64_t cb = ((uint64_t)S.at(p + 17) | (uint64_t)S.at(p + 49) << 32) &
                                        ((1ull << (3 * (((h >> 13) & 15) + 4))) - 1);
                    const uint32_t v = dyn_candidate_lut(S, p, a.end_bits, h, cb, (lds_u8p)list + t * kFindLutStride,
                                                         kFindLaneSyms ? kFindLaneSyms : ~0u);
                    if (v == kCandYes) push(p << 2 | 2);
                    if (v == kCandOpen) open[atomicAdd(&n_open, 1u)] = mine;
                }
                __syncthreads();
                if (prof) ts_open = wall_clock64();
                opens += n_open;
                // the still-open headers, one per wave at a time, all 64 lanes on it
                for (uint32_t i = t >> 6; i < n_open; i += 4) {
                    const uint64_t p = 8 * q0 + open[i];
                    const uint32_t h = S.at(p);
                    const uint32_t nl = ((h >> 3) & 31) + 257, nd = ((h >> 8) & 31) + 1, nc = ((h >> 13) & 15) + 4;
                    const uint64_t cb = ((uint64_t)S.at(p + 17) | (uint64_t)S.at(p + 49) << 32) & ((1ull << (3 * nc)) - 1);
                    uint8_t *const lens = wlens + 320 * (t >> 6);
                    for (uint32_t k = lane; k < 320; k += 64) lens[k] = 0;
                    uint64_t pos = p + 17 + 3 * nc;
                    uint32_t kl, kd, used_d;
                    bool eob;
                    const bool ok = header_lengths_wave(S, pos, a.end_bits, cb, nl, nd, lens, kl, kd, used_d, eob) && eob &&
                                    kl == (1u << 15) && (kd == (1u << 15) || used_d <= 1);
                    if (ok) {
                        // listed as parsed (type 3): its code lengths and body start for k_pinf_block, which
                        // then skips the header parse
                        uint32_t ci = lane == 0 ? push(p << 2 | 3) : 0u;
                        ci = (uint32_t)__shfl((int)ci, 0, 64);
                        if (ci < kPinfMaxCand) {
                            for (uint32_t k = lane; k < 320; k += 64) a.lens[(uint64_t)ci * 320 + k] = lens[k];
                            if (lane == 0) {
                                a.blk[ci].body = pos;
                                a.blk[ci].nlen = nl;
                                a.blk[ci].ndist = nd;
                            }
                        }
                    }
                }
            } else
            for (uint32_t i0 = t; RDX_PINF_FIND_HDR && i0 < n + 255; i0 += 256) {
                const uint32_t i = RDX_PINF_FIND_SPREAD ? (i0 - t) + (t & 63) * 4 + (t >> 6) : i0;
                if (i >= n) continue;
                const uint64_t p = 8 * q0 + list[i];
                const uint32_t h = S.at(p);
                const uint64_t cb = ((uint64_t)S.at(p + 17) | (uint64_t)S.at(p + 49) << 32) &
                                    ((1ull << (3 * (((h >> 13) & 15) + 4))) - 1);
                if (dyn_candidate_rest(S, p, a.end_bits, h, cb)) push(p << 2 | 2);
            }
            survivors += n;
            __syncthreads();
            if (t == 0) n_list = 0;
            __syncthreads();
        }
    }
    if (t == 0 && survivors) atomicAdd(&st->n_surv, survivors);
    if (prof) {
        __syncthreads();
        if (t == 0) {
            prof[0] = ts0;
            prof[1] = ts1;
            prof[2] = ts2;
            prof[3] = wall_clock64();
            prof[4] = survivors;
            prof[5] = ts_open;
            prof[6] = opens;
        }
    }
}

// Smallest candidate position strictly after `after` (the end bound of a block's body), or end_bits.
__device__ uint64_t next_cand(const PinfArgs &a, uint32_t n, uint64_t after, uint64_t *red) {
    uint64_t best = ~0ull;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t b = a.cand[i] >> 2;
        if (b > after && b < best) best = b;
    }
    // block-wide min
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint64_t o = (uint64_t)__shfl_xor((long long)best, m, 64);
        best = o < best ? o : best;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = best;
    __syncthreads();
    best = red[0];
    for (uint32_t k = 1; k < blockDim.x / 64; ++k) best = red[k] < best ? red[k] : best;
    __syncthreads();
    return best == ~0ull ? a.end_bits : best;
}

// RDX_PINF_PROF: per workgroup 8 words — [0] start, [1] tables built, [2] first decode pass, [3] lanes
// agree, [4] end (wall clock), [5] resync rounds, [6] sequential walks, [7] body extensions
#define PINF_STAMP(slot, v)                                                                     \
    do {                                                                                        \
        if (prof && threadIdx.x == 0) prof[slot] = (v);                                         \
    } while (0)

// ---- 2. one candidate block per workgroup -------------------------------------------------------------
__device__ void block_body(const PinfArgs &a, uint32_t first, uint32_t count) {
    uint64_t *const prof = a.prof && blockIdx.x < count ? a.prof + 8ull * (first + blockIdx.x) : nullptr;
    uint64_t rounds = 0, walks = 0, exts = 0;
    __shared__ Tabs T;
    __shared__ uint64_t s_st[kLanes], s_x[kLanes], s_red[kLanes / 64];
    static_assert(kLanes % 64 == 0 && kLanes <= 1024, "lanes per block");
    __shared__ uint32_t s_nb[kLanes];
    __shared__ uint64_t s_mid[kLanes];   // the lane's first boundary at or past its middle | bytes before it << 40
    __shared__ uint8_t s_ed[kLanes];
    __shared__ uint32_t s_wm[kLanes / 64];
    __shared__ uint64_t s_body;
    __shared__ uint32_t s_ok, s_nlen, s_ndist, s_first;
    // the tabulated walk: lane exits from each of the kOff starts their predecessor can hand them
    constexpr uint32_t kOff = 48, kG = kLanes / kOff, kWalk = 4;
    __shared__ uint64_t s_tx[kG * kOff];
    __shared__ uint32_t s_tnb[kG * kOff];
    __shared__ uint8_t s_ted[kG * kOff];
    __shared__ uint32_t win[kWinDwords];
    const uint32_t n = min(a.state->n_cand, kPinfMaxCand);
    const uint32_t ci = first + blockIdx.x;
    if (blockIdx.x >= count || ci >= n) return;
    Stream S = make_stream(a);
    const uint32_t t = threadIdx.x;
    const uint64_t key = a.cand[ci];
    const uint64_t bit = key >> 2;
    const uint32_t type = (uint32_t)(key & 3);
    PinfBlk &B = a.blk[ci];
    if (type == 0) {   // stored: LEN / NLEN at the byte `bit / 8`
        if (t == 0) {
            const uint64_t q = bit / 8;
            const uint32_t len = S.byte(q) | S.byte(q + 1) << 8, nlen = S.byte(q + 2) | S.byte(q + 3) << 8;
            const bool ok = len == (~nlen & 0xffff) && q + 4 + len <= a.end_byte;
            B.end = 8 * (q + 4 + len);
            B.bytes = len;
            B.body = 8 * (q + 4);
            B.nlanes = 0;
            B.status = ok ? 0 : 1;
        }
        return;
    }
    // the header and (where it fits) the body from LDS: the window starts at the header's dword
    S.stage(win, kWinDwords, bit >> 5, a.nw);
    if (t < 64) {
        uint64_t body = 0;
        uint32_t nl = 0, nd = 0;
        bool ok = true;
        if (type == 3) {   // parsed by k_pinf_find (the same rules): its code lengths and body start
            for (uint32_t i = t; i < 320; i += 64) T.lens[i] = a.lens[(uint64_t)ci * 320 + i];
            body = B.body;
            nl = B.nlen;
            nd = B.ndist;
        } else {
            ok = parse_header_wave(S, bit, type, a.end_bits, T, &body, &nl, &nd);
        }
        if (t == 0) {
            s_ok = ok ? 1 : 0;
            s_body = body;
            s_nlen = nl;
            s_ndist = nd;
        }
    }
    __syncthreads();
    PINF_STAMP(6, wall_clock64());   // staged and parsed
    const bool hdr_ok = s_ok != 0;
    const bool tabs_ok = hdr_ok && build_tabs(T, s_nlen, s_ndist);
    if (!tabs_ok) {
        if (t == 0) B.status = 1;
        return;
    }
    PINF_STAMP(1, wall_clock64());
    // keep the built tables: k_pinf_emit's workgroups copy them instead of building them again
    {
        const uint4 *from = reinterpret_cast<const uint4 *>(&T);
        uint4 *to = reinterpret_cast<uint4 *>(a.tabs + (uint64_t)ci * sizeof(Tabs));
        for (uint32_t i = t; i < sizeof(Tabs) / 16; i += kLanes) to[i] = from[i];
    }
    const uint64_t body = s_body;
    uint64_t E = next_cand(a, n, bit, s_red);
    for (uint32_t ext = 0; ext < 8; ++ext) {
        if (E <= body) E = body + 1;
        const uint64_t span = E - body;
        if (span > kMaxSpan) break;
        const uint32_t L = (uint32_t)max<uint64_t>(1, min<uint64_t>(kLanes, span / kMinLaneBits));
        auto lo = [&](uint32_t k) -> uint64_t { return k >= L ? E : body + span * k / L; };
        auto run = [&](uint32_t k, uint64_t from) {
            Bits br;
            br.seek(S, from);
            uint64_t x, nb, md = ~0ull;
            const uint64_t m = lo(k) + (lo(k + 1) - lo(k)) / 2;
            const uint32_t r = run_lane<false>(T, S, br, lo(k + 1), a.end_bits, &x, &nb, nullptr, 0, nullptr, 0, nullptr,
                                               nullptr, nullptr, kEmitHalves && from < m ? m : ~0ull, &md);
            s_st[k] = from;
            s_x[k] = x;
            s_nb[k] = (uint32_t)nb;
            s_ed[k] = (uint8_t)r;
            s_mid[k] = md;
        };
        // pass 0: lane k > 0 first decodes kWarmBits before its range and starts at its first symbol
        // boundary at or past lo(k) — by then its parse has almost always resynchronised with the true one,
        // so few lanes need resync rounds (each round costs a whole pass)
        if (t < L) {
            uint64_t from = lo(t);
            if (t > 0 && from - body > kWarmBits) {
                Bits br;
                br.seek(S, from - kWarmBits);
                uint64_t x, nb;
                if (run_lane<false>(T, S, br, from, a.end_bits, &x, &nb, nullptr, 0) == 0) from = x;
            }
            run(t, from);
        }
        __syncthreads();
        PINF_STAMP(2, wall_clock64());
        for (;;) {
            // resync rounds: lane k re-decodes from lane k-1's exit when its start differs.  Lanes up to
            // the first break of the chain from lane 0 are verified; the rounds end once a verified lane
            // has ended the block (lanes past it decode bits after the block and do not matter) or every
            // lane is verified
            bool done = false;
            for (uint32_t round = 0; round < kRounds; ++round) {
                const bool brk = t >= 1 && t < L && (s_ed[t - 1] != 0 || s_st[t] != s_x[t - 1]);
                const uint64_t bw = __ballot(brk);
                if ((t & 63) == 0) s_wm[t >> 6] = bw ? (t & ~63u) + (uint32_t)__builtin_ctzll(bw) : L;
                __syncthreads();
                uint32_t m = L;
                for (uint32_t w = 0; w < kLanes / 64; ++w) m = s_wm[w] < m ? s_wm[w] : m;
                if (m >= L || s_ed[m - 1] != 0) {
                    done = true;
                    break;
                }
                uint64_t px = 0;
                bool redo = false;
                if (t >= m && t < L) {
                    px = s_x[t - 1];
                    redo = s_ed[t - 1] == 0 && s_st[t] != px;
                }
                __syncthreads();
                if (redo) run(t, px);
                ++rounds;
                __syncthreads();
            }
            if (done) break;
            // the data keeps the parses apart (periodic data: a parse that starts out of phase stays out of
            // phase, so rounds verify one lane each).  The true start of lane j is the first symbol boundary
            // at or past lo(j): one of the kOff bit offsets after it (a symbol — length, distance and their
            // extra bits — is at most 48 bits).  So lane j's exit is tabulated for every one of those starts,
            // kG lanes per pass with all threads, and thread 0 composes the true chain through the tables:
            // a pass verifies kG lanes in the time of one lane's decode (the walk it replaces verified one)
            ++walks;
            // first the cheap form: thread 0 walks on from the first break, lane by lane, for up to kWalk
            // lanes (most breaks heal within a lane or two); only parses still apart after that are tabulated
            if (t == 0) {
                uint32_t m = 1;
                while (m < L && (s_ed[m - 1] != 0 || s_st[m] == s_x[m - 1])) ++m;
                uint32_t j = m;
                for (uint32_t w = 0; j < L && w < kWalk; ++w, ++j) {
                    if (j > m && (s_ed[j - 1] != 0 || s_st[j] == s_x[j - 1])) break;
                    run(j, s_x[j - 1]);
                }
                // the next break, if the walk did not heal it
                while (j < L && s_ed[j - 1] == 0 && s_st[j] == s_x[j - 1]) ++j;
                s_first = j < L && s_ed[j - 1] == 0 && j < m + kWalk + 1 ? j : L;
            }
            __syncthreads();
            if (s_first >= L) continue;   // healed (or the block ended): back to the rounds
            // each pass tabulates the kG lanes from the first break; thread 0 composes them, then skips to
            // the next lane whose start disagrees with its predecessor's exit (lanes whose parses agree need
            // no table), so data with few breaks costs one pass and periodic data one pass per kG lanes
            uint32_t base = s_first;
            for (;;) {
                const uint32_t k = base + t / kOff, o = t % kOff;
                if (t < kG * kOff && k < L) {
                    Bits br;
                    br.seek(S, lo(k) + o);
                    uint64_t x, nb;
                    const uint32_t r = run_lane<false>(T, S, br, lo(k + 1), a.end_bits, &x, &nb, nullptr, 0);
                    s_tx[t] = x;
                    s_tnb[t] = (uint32_t)nb;
                    s_ted[t] = (uint8_t)r;
                }
                __syncthreads();
                if (t == 0) {
                    uint32_t next = L;
                    const uint32_t hi = base + kG < L ? base + kG : L;
                    uint32_t j = base;
                    for (; j < hi; ++j) {
                        if (s_ed[j - 1] != 0) break;   // the block ended before lane j
                        const uint64_t st = s_x[j - 1];
                        if (s_st[j] == st) continue;   // already decoded from its true start
                        const uint64_t off = st - lo(j);
                        if (off < kOff) {
                            const uint32_t q = (j - base) * kOff + (uint32_t)off;
                            s_st[j] = st;
                            s_x[j] = s_tx[q];
                            s_nb[j] = s_tnb[q];
                            s_mid[j] = ~0ull;   // (not recorded by the tabulation)
                            s_ed[j] = s_ted[q];
                        } else {
                            run(j, st);   // (a symbol longer than kOff bits cannot occur)
                        }
                    }
                    if (j == hi) {   // the next break past the pass, if the block goes on
                        while (j < L && s_ed[j - 1] == 0 && s_st[j] == s_x[j - 1]) ++j;
                        if (j < L && s_ed[j - 1] == 0) next = j;
                    }
                    s_wm[0] = next;
                }
                __syncthreads();
                if (s_wm[0] >= L) break;
                base = s_wm[0];
                __syncthreads();
            }
            __syncthreads();
        }
        // the first lane that ended (end of block or error) closes the block
        if (t == 0) {
            uint32_t j = 0;
            while (j < L && s_ed[j] == 0) ++j;
            s_first = j;
        }
        __syncthreads();
        const uint32_t j = s_first;
        PINF_STAMP(3, wall_clock64());
        if (j == L) {   // no end of block before E (a false candidate inside the body): extend the body
            // to the next candidate, and at least to a whole pass of lanes (the lanes' time does not grow
            // with the span up to kLanes x kMinLaneBits; each extension costs a pass)
            if (E >= a.end_bits) break;
            E = max(next_cand(a, n, E, s_red), min(body + (uint64_t)kLanes * kMinLaneBits, a.end_bits));
            ++exts;
            continue;
        }
        PINF_STAMP(5, rounds);
        PINF_STAMP(7, exts | walks << 32);
        if (t == 0) {
            uint64_t bytes = 0;
            for (uint32_t k = 0; k <= j; ++k) bytes += s_nb[k];
            B.end = s_x[j];
            B.bytes = bytes;
            B.body = body;
            B.nlanes = j + 1;
            B.nlen = s_nlen;
            B.ndist = s_ndist;
            B.status = s_ed[j] == 1 ? 0 : 1;
        }
        if (t <= j) {
            a.lst[(uint64_t)ci * kLanes + t] = s_st[t];
            a.lnb[(uint64_t)ci * kLanes + t] = s_nb[t];
            a.lmid[(uint64_t)ci * kLanes + t] = s_mid[t];
        }
        return;
    }
    if (t == 0) B.status = 1;   // no end of block within kMaxSpan / the stream
}

// RDX_PINF_PROF: every workgroup's start / end (wall clock) in a.prof, for tools/probe_pinflate.py
__global__ __launch_bounds__(kLanes) void k_pinf_block(PinfArgs a, uint32_t first, uint32_t count) {
    const uint64_t t0 = a.prof ? wall_clock64() : 0;
    block_body(a, first, count);
    if (a.prof) {
        __syncthreads();
        if (threadIdx.x == 0 && blockIdx.x < count) {
            a.prof[8 * (first + blockIdx.x)] = t0;
            a.prof[8 * (first + blockIdx.x) + 4] = wall_clock64();
        }
    }
}

// ---- 3. the chain ---------------------------------------------------------------------------------------
constexpr uint32_t kChainThreads = 1024;

__global__ __launch_bounds__(kChainThreads) void k_pinf_chain(PinfArgs a) {
    __shared__ uint64_t sk[kPinfMaxCand];      // (key << 12 | index), sorted
    __shared__ int32_t succ[kPinfMaxCand];     // sorted index of the next block, or < 0
    __shared__ uint16_t order[kPinfMaxCand];   // the chain: sorted indices in stream order
    __shared__ uint8_t fin[kPinfMaxCand];      // BFINAL of that next block
    __shared__ uint64_t s_scan[kChainThreads / 64];
    __shared__ int32_t s_head;
    __shared__ uint32_t s_headfin, s_nc, s_status;
    __shared__ uint64_t s_p0, s_miss;
    __shared__ uint32_t s_hok;
    PinfState *st = a.state;
    const uint32_t t = threadIdx.x;
    const Stream S = make_stream(a);
    if (st->overflow) {
        if (t == 0) st->status = kPinfFallback;
        return;
    }
    const uint32_t n = min(st->n_cand, kPinfMaxCand);
    for (uint32_t i = t; i < kPinfMaxCand; i += kChainThreads) sk[i] = i < n ? (a.cand[i] << 12 | i) : ~0ull;
    // the stream header (thread 0): zlib RFC 1950 / gzip RFC 1952, as oracle_inflate unzlib / gunzip
    if (t == 0) {
        uint64_t q = a.first_byte;
        bool ok = true;
        if (a.format == RDX_COMPRESSION_ZLIB) {
            ok = a.end_byte >= q + 2;
            const uint32_t cmf = S.byte(q), flg = S.byte(q + 1);
            ok = ok && (cmf & 15) == 8 && (cmf >> 4) <= 7 && (cmf * 256 + flg) % 31 == 0 && !(flg & 0x20);
            q += 2;
        } else {
            ok = a.end_byte >= q + 10 && S.byte(q) == 0x1f && S.byte(q + 1) == 0x8b && S.byte(q + 2) == 8;
            const uint32_t flg = S.byte(q + 3);
            q += 10;
            if (ok && (flg & 4)) {
                const uint32_t xlen = S.byte(q) | S.byte(q + 1) << 8;
                q += 2 + xlen;
            }
            if (ok && (flg & 8)) {
                while (q < a.end_byte && S.byte(q) != 0) ++q;
                ++q;
            }
            if (ok && (flg & 16)) {
                while (q < a.end_byte && S.byte(q) != 0) ++q;
                ++q;
            }
            if (ok && (flg & 2)) q += 2;
            ok = ok && q < a.end_byte;
        }
        s_hok = ok ? 1 : 0;
        s_p0 = 8 * q;
    }
    __syncthreads();
    // sort the candidate keys (unique: the index is in the low bits).  Up to one per thread: each key's rank
    // by counting the smaller ones (uniform LDS reads, no barrier per stage); more: a bitonic sort of as many
    // as there are, rounded up to a power of two
    uint32_t m = 2;
    while (m < n) m <<= 1;
    if (n <= kChainThreads) {
        uint64_t key = 0;
        uint32_t rank = 0;
        if (t < n) {
            key = sk[t];
            for (uint32_t j = 0; j < n; ++j) rank += sk[j] < key ? 1u : 0u;
        }
        __syncthreads();
        if (t < n) sk[rank] = key;
        __syncthreads();
        m = 0;   // (no bitonic stages)
    }
    for (uint32_t k = 2; k <= m; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < m; i += kChainThreads) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t x = sk[i], y = sk[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) {
                        sk[i] = y;
                        sk[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    // successor of a block ending at e: the candidate the header at e names (-1: none, a miss; -3: the
    // stream ends or BTYPE 3)
    auto find = [&](uint64_t e, uint8_t *f) -> int32_t {
        if (e + 3 > a.end_bits) return -3;
        const uint32_t h = S.at(e) & 7;
        *f = (uint8_t)(h & 1);
        const uint32_t ty = (h >> 1) & 3;
        if (ty == 3) return -3;
        uint64_t k = ty == 0 ? (8 * ((e + 3 + 7) / 8)) << 2 | 0 : e << 2 | ty;
        uint32_t lo = 0, hi = n;   // first sorted key >= k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if ((sk[mid] >> 12) < k) lo = mid + 1;
            else hi = mid;
        }
        // (a dynamic block's candidate is type 2, or 3 when k_pinf_find parsed its header: the next key)
        if (lo < n && ((sk[lo] >> 12) == k || (ty == 2 && (sk[lo] >> 12) == (k | 1)))) return (int32_t)lo;
        return -1;
    };
    for (uint32_t i = t; i < n; i += kChainThreads) {
        const uint32_t c = (uint32_t)(sk[i] & 4095);
        const PinfBlk &B = a.blk[c];
        uint8_t f = 0;
        succ[i] = B.status ? -2 : find(B.end, &f);
        fin[i] = f;
    }
    if (t == 0) {
        uint8_t f = 0;
        s_head = s_hok ? find(s_p0, &f) : -3;
        s_headfin = f;
    }
    __syncthreads();
    // the walk (thread 0, LDS only): sorted indices in stream order up to the BFINAL block
    if (t == 0) {
        int32_t cur = s_head;
        uint32_t f = s_headfin, nc = 0, status = kPinfFallback;
        int32_t last = -1;
        for (;;) {
            if (cur == -1) {   // a block start that is no candidate: the host decodes it and chains again
                status = kPinfMiss;
                break;
            }
            if (cur < 0 || nc >= kPinfMaxCand) break;   // an error: the sequential decoder reports it
            order[nc++] = (uint16_t)cur;
            if (f) {
                status = kPinfOk;
                break;
            }
            f = fin[cur];
            last = cur;
            cur = succ[cur];
        }
        // the position where the walk stopped: a miss's block start
        s_miss = status == kPinfMiss ? (last < 0 ? s_p0 : a.blk[sk[last] & 4095].end) : 0;
        s_nc = nc;
        s_status = status;
    }
    __syncthreads();
    const uint32_t nc = s_nc;
    // output offsets: an exclusive scan of the chain blocks' bytes, 4 per thread
    uint64_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t k = 4 * t + q;
        v[q] = k < nc ? a.blk[sk[order[k]] & 4095].bytes : 0;
        sum += v[q];
    }
    uint64_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = (uint64_t)__shfl_up((long long)incl, d, 64);
        if ((t & 63) >= (uint32_t)d) incl += o;
    }
    if ((t & 63) == 63) s_scan[t / 64] = incl;
    __syncthreads();
    uint64_t base = 0;
    for (uint32_t w = 0; w < t / 64; ++w) base += s_scan[w];
    uint64_t run = base + incl - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t k = 4 * t + q;
        if (k < nc) {
            a.chain[k] = (uint32_t)(sk[order[k]] & 4095);
            a.coff[k] = run;
        }
        run += v[q];
    }
    if (t == kChainThreads - 1) {
        const uint64_t total = run;   // the last thread's running sum: every chain block's bytes
        uint32_t status = s_status;
        if (status == kPinfOk) {   // BFINAL: the trailer follows at the next byte boundary
            const uint64_t e = a.blk[sk[order[nc - 1]] & 4095].end;
            const uint64_t tb = (e + 7) / 8;
            const uint64_t need = a.format == RDX_COMPRESSION_ZLIB ? 4 : 8;
            if (tb + need > a.end_byte || total >= (1ull << 31)) status = kPinfFallback;
            st->trailer_byte = tb;
        }
        if (status == kPinfMiss) {
            const uint64_t e = s_miss;
            st->miss_bit = e;
            st->miss_type = (S.at(e) >> 1) & 3;
        }
        st->n_chain = nc;
        st->total = total;
        st->status = status;
        if (a.hslot) {   // the host's copy, polled (system-scope vector stores into page-locked memory)
            const uint64_t T = (uint64_t)a.tag << 48;
            const uint64_t mb = status == kPinfMiss ? s_miss : 0;
            const uint64_t mt = status == kPinfMiss ? (S.at(mb) >> 1) & 3 : 0;
            const uint64_t g0 = status | mt << 2 | (uint64_t)nc << 4 | (uint64_t)min(st->n_cand, 8191u) << 17;
            __hip_atomic_store(a.hslot + 1, (total & kPinfPayload) | T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.hslot + 2, (mb & kPinfPayload) | T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.hslot + 0, g0 | T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---- 4. sources of every output byte ----------------------------------------------------------------------
// kPinfEmitSplit workgroups per chain block (consecutive blockIdx), workgroup g with lanes
// [g * kEmitThreads, (g + 1) * kEmitThreads): its own window of the stream and its own tables
__device__ void emit_body(const PinfArgs &a) {
    __shared__ Tabs T;
    __shared__ uint64_t s_off[kEmitThreads];
    __shared__ uint64_t s_red[kEmitThreads / 64];
    __shared__ uint32_t win[kEmitWin];
    __shared__ uint64_t s_rec[(kEmitRecs ? kEmitRecs : 1) * kEmitThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t bi = blockIdx.x / kPinfEmitSplit, g = blockIdx.x % kPinfEmitSplit;
    const uint32_t lane = g * kEmitLanes + (kEmitHalves ? t / 2 : t), half = kEmitHalves ? t & 1 : 0u;
    const uint32_t c = a.chain[bi];
    const uint64_t o = a.coff[bi];
    const PinfBlk B = a.blk[c];
    Stream S = make_stream(a);
    uint32_t *src = a.src;
    const uint32_t type = (uint32_t)(a.cand[c] & 3);
    if (type == 0) {   // stored: four bytes per thread and step, 16-byte stores where the quad is aligned
        const uint64_t q0 = B.body / 8;
        for (uint64_t j = 4 * ((uint64_t)g * kEmitThreads + t); j < B.bytes; j += 4ull * kEmitThreads * kPinfEmitSplit) {
            const uint32_t w = S.at(8 * (q0 + j));
            const uint64_t d = o + j;
            const uint32_t k = (uint32_t)min<uint64_t>(4, B.bytes - j);
            if (k == 4 && (d & 3) == 0) {
                gst<uint4>(src + d, make_uint4(kFlag | (w & 0xff), kFlag | ((w >> 8) & 0xff), kFlag | ((w >> 16) & 0xff),
                                               kFlag | (w >> 24)));
            } else {
                for (uint32_t i = 0; i < k; ++i) src[d + i] = kFlag | ((w >> (8 * i)) & 0xff);
            }
        }
        return;
    }
    const uint32_t L = B.nlanes;
    const uint32_t g0 = g * kEmitLanes;
    if (g0 >= L) return;   // (the whole workgroup)
    const uint64_t *const lst = a.lst + (uint64_t)c * kLanes;
    const uint32_t *const lnb = a.lnb + (uint64_t)c * kLanes;
    const uint32_t g1 = min(L, g0 + kEmitLanes);
    S.stage(win, kEmitWin, lst[g0] >> 5, ((g1 < L ? lst[g1] : B.end) >> 5) + 2);
    {   // the block's tables, as k_pinf_block built them
        const uint4 *from = reinterpret_cast<const uint4 *>(a.tabs + (uint64_t)c * sizeof(Tabs));
        uint4 *to = reinterpret_cast<uint4 *>(&T);
        for (uint32_t i = t; i < sizeof(Tabs) / 16; i += kEmitThreads) to[i] = from[i];
    }
    // the output bytes of the block's lanes before this workgroup's (a block's bytes fit 32 bits)
    uint32_t before = 0;
    for (uint32_t k = t; k < g0; k += kEmitThreads) before += lnb[k];
#pragma unroll
    for (int d = 32; d; d >>= 1) before += (uint32_t)__shfl_xor((int)before, d, 64);
    if ((t & 63) == 0) s_red[t >> 6] = before;
    __syncthreads();
    before = 0;
    for (uint32_t w = 0; w < kEmitThreads / 64; ++w) before += (uint32_t)s_red[w];
    uint64_t *const prof = a.prof && blockIdx.x < kPinfMaxCand ? a.prof + 8ull * (kPinfMaxCand + blockIdx.x) : nullptr;
    const uint32_t nb = lane < L ? lnb[lane] : 0;
    const uint64_t mid = kEmitHalves && lane < L ? a.lmid[(uint64_t)c * kLanes + lane] : ~0ull;
    // exclusive prefix of the lanes' bytes (a lane's bytes counted once, on its first half)
    s_off[t] = half ? 0u : nb;
    __syncthreads();
    for (uint32_t d = 1; d < kEmitThreads; d <<= 1) {
        const uint64_t v = t >= d ? s_off[t - d] : 0;
        __syncthreads();
        s_off[t] += v;
        __syncthreads();
    }
    PINF_STAMP(1, wall_clock64());
    if (lane >= L) return;
    // this thread's part of the lane: all of it, or the half before / from its recorded middle boundary
    const bool split = mid != ~0ull;
    if (half && !split) return;
    const uint64_t mpos = mid & ((1ull << 40) - 1), mnb = mid >> 40;
    const uint64_t my = o + before + s_off[t] - nb + (half ? mnb : 0);
    const uint64_t want_nb = split ? (half ? nb - mnb : mnb) : nb;
    Bits br;
    br.seek(S, half ? mpos : lst[lane]);
    const uint64_t stop = split && !half ? mpos : lane + 1 < L ? lst[lane + 1] : ~0ull;
    uint64_t x, got;
#ifndef RDX_PINF_LANESTAT
#define RDX_PINF_LANESTAT 0   // tuning builds: RDX_PINF_PROF also reports emit's slowest lane (costs scratch)
#endif
#if RDX_PINF_LANESTAT
    uint32_t stat[3] = {0, 0, 0};
    const uint64_t tl = prof ? wall_clock64() : 0;
    const uint32_t r = run_lane<true>(T, S, br, stop, a.end_bits, &x, &got, src, my, &a, my + want_nb, prof ? stat : nullptr);
#else
    uint32_t n_rec = 0;
    const uint32_t r = run_lane<true>(T, S, br, stop, a.end_bits, &x, &got, src, my, &a, my + want_nb, nullptr,
                                      (lds_u64p)s_rec + t, &n_rec);
    // the recorded matches (checked against the output bounds when they were decoded)
    for (uint32_t k = 0; k < n_rec; ++k) {
        const uint64_t m = s_rec[k * kEmitThreads + t];
        const uint32_t q = (uint32_t)m, len = (uint32_t)(m >> 32) & 0xffff, dist = (uint32_t)(m >> 48), base = q - dist;
        if (dist >= len) {
            for (uint32_t j = 0; j < len; ++j) src[q + j] = base + j;
        } else {
            uint32_t mm = 0;
            for (uint32_t j = 0; j < len; ++j) {
                src[q + j] = base + mm;
                mm = mm + 1 == dist ? 0 : mm + 1;
            }
        }
    }
#endif
    const uint32_t want = lane + 1 < L || (split && !half) ? 0u : 1u;
    if (r != want || got != want_nb) atomicOr(&a.state->emit_err, 1u);
#if RDX_PINF_LANESTAT
    if (prof) {   // the slowest lane: [2] its decode time (ticks), [5] symbols, [6] past the root, [7] L2 refills
        const uint64_t dt = wall_clock64() - tl;
        const uint64_t mine = dt << 32 | (uint64_t)stat[0] << 16 | min(stat[1], 255u) << 8 | min(stat[2], 255u);
        atomicMax((unsigned long long *)&prof[2], (unsigned long long)mine);
    }
#endif
}

__global__ __launch_bounds__(kEmitThreads) void k_pinf_emit(PinfArgs a) {
    const uint64_t t0 = a.prof ? wall_clock64() : 0;
    emit_body(a);
    if (a.prof && blockIdx.x < kPinfMaxCand) {
        __syncthreads();
        if (threadIdx.x == 0) {
            a.prof[8 * (kPinfMaxCand + blockIdx.x)] = t0;
            a.prof[8 * (kPinfMaxCand + blockIdx.x) + 4] = wall_clock64();
        }
    }
}

// ---- 4b. long matches: one wavefront per match record ------------------------------------------------
// (the grid is capped — launch_pinf_rest — and each wavefront loops over the records: near the 2^31-byte
// limit one wavefront per record would exceed a launch's 2^32 work-items)
constexpr uint32_t kExpandMaxBlocks = 65536;

__global__ __launch_bounds__(256) void k_pinf_expand(PinfArgs a) {
    const uint32_t n = min(a.state->n_match, a.mcap);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t *src = a.src;
    for (uint32_t r = blockIdx.x * 4 + threadIdx.x / 64; r < n; r += gridDim.x * 4) {
        const uint4 m = a.mlist[r];
        const uint32_t o = m.x, len = m.y, dist = m.z;
        if ((uint64_t)o + len > a.state->total || dist > o || dist == 0) {   // (k_pinf_emit checked it: never)
            if (lane == 0) atomicOr(&a.state->emit_err, 8u);
            continue;
        }
        if (dist >= len) {
            for (uint32_t j = lane; j < len; j += 64) src[o + j] = o + j - dist;
        } else {   // overlapping: (j mod dist) into the dist bytes before the match (a float quotient, corrected)
            const float rd = __builtin_amdgcn_rcpf((float)dist);
            for (uint32_t j = lane; j < len; j += 64) {
                const uint32_t q = (uint32_t)((float)j * rd);
                int32_t rem = (int32_t)(j - q * dist);
                rem = rem < 0 ? rem + (int32_t)dist : (rem >= (int32_t)dist ? rem - (int32_t)dist : rem);
                src[o + j] = o - dist + (uint32_t)rem;
            }
        }
    }
}

// ---- 5. sources -> bytes -------------------------------------------------------------------------------
// Tiles of 32 KiB of output, the DEFLATE window: a link from a tile leads into the same tile or the one
// before it.  k_pinf_tile (one workgroup per tile, its sources in 128 KiB of LDS) follows every link that
// stays in the tile, at LDS latency, until each byte is a literal or a link into the previous tile, and
// writes the tile back over its sources (a literal, or a link into the previous tile); a tile of literals
// also writes its bytes.  k_pinf_xhop / k_pinf_xout (below) resolve the links between tiles.  Links always
// point back (a copy source precedes its byte); one that does not, or a link further back than the window,
// is an inconsistency (stale sources after a failed emit): the check rejects the stream.
constexpr uint32_t kTile = kPinfTile, kTileThreads = 1024, kWindow = 32768;
#ifndef RDX_PINF_TILE_HOPS
#define RDX_PINF_TILE_HOPS 4
#endif
constexpr uint32_t kTileHops = RDX_PINF_TILE_HOPS;

__global__ __launch_bounds__(kTileThreads) void k_pinf_tile(PinfArgs a) {
    __shared__ uint32_t tl[kTile];
    PinfState *st = a.state;
    const uint64_t N = st->total;
    const uint64_t T0 = (uint64_t)blockIdx.x * kTile;
    if (T0 >= N) return;
    const uint32_t n = (uint32_t)min<uint64_t>(kTile, N - T0), t = threadIdx.x;
    uint32_t *src = a.src + T0;   // (16-byte aligned: the buffer is, and T0 is a multiple of 32 KiB)
    for (uint32_t i = 4 * t; i < n; i += 4 * kTileThreads) {
        if (i + 4 <= n) {
            const uint4 v = gld<uint4>(src + i);
            tl[i] = v.x;
            tl[i + 1] = v.y;
            tl[i + 2] = v.z;
            tl[i + 3] = v.w;
        } else {
            for (uint32_t k = i; k < n; ++k) tl[k] = src[k];
        }
    }
    __syncthreads();
    bool err = false, more = true;
    for (uint32_t it = 0; it < 48 && more; ++it) {   // (chains halve per pass: 15 passes cover a tile)
        bool m = false;
        for (uint32_t i = t; i < n; i += kTileThreads) {
            const uint32_t v = tl[i];
            if ((v & kFlag) || v < T0) continue;   // a literal, or a link out of the tile
            if (v >= T0 + i) {
                err = true;
                tl[i] = kFlag;
                continue;
            }
            // up to kTileHops links per pass (each read may already see other entries' progress)
            uint32_t w = tl[v - T0];
#pragma unroll
            for (uint32_t h = 1; h < kTileHops; ++h) {
                if ((w & kFlag) || w < T0) break;
                w = tl[w - T0];
            }
            tl[i] = w;
            m |= !(w & kFlag) && w >= T0;
        }
        more = __syncthreads_or(m);
    }
    err |= more;
    bool lit = true;
    for (uint32_t i = t; i < n; i += kTileThreads) lit &= (tl[i] & kFlag) != 0;
    const bool all_lit = __syncthreads_and(lit);
    if (all_lit) {   // the bytes themselves (out is 16-byte aligned), and the literals over the sources for
                     // k_pinf_xhop, whose links into this tile then resolve with one read
        for (uint32_t i = 4 * t; i < n; i += 4 * kTileThreads) {
            if (i + 4 <= n) {
                gst<uint32_t>(a.out + T0 + i, (tl[i] & 0xff) | (tl[i + 1] & 0xff) << 8 | (tl[i + 2] & 0xff) << 16 | tl[i + 3] << 24);
                gst<uint4>(reinterpret_cast<uint4 *>(src + i), make_uint4(tl[i], tl[i + 1], tl[i + 2], tl[i + 3]));
            } else {
                for (uint32_t k = i; k < n; ++k) {
                    a.out[T0 + k] = (uint8_t)tl[k];
                    src[k] = tl[k];
                }
            }
        }
    } else {         // the entries themselves, back over the tile's sources: literals, or links into the previous tile
        const uint64_t base = T0 >= kWindow ? T0 - kWindow : 0;   // (T0 > 0 here: tile 0 has no links out)
        auto chk = [&](uint32_t v) -> uint32_t {
            if (!(v & kFlag) && (T0 == 0 || v < base || v >= T0)) {
                err = true;
                return kFlag;
            }
            return v;
        };
        for (uint32_t i = 4 * t; i < n; i += 4 * kTileThreads) {
            if (i + 4 <= n) {
                gst<uint4>(reinterpret_cast<uint4 *>(src + i), make_uint4(chk(tl[i]), chk(tl[i + 1]), chk(tl[i + 2]), chk(tl[i + 3])));
            } else {
                for (uint32_t k = i; k < n; ++k) src[k] = chk(tl[k]);
            }
        }
    }
    if (t == 0) a.tflag[blockIdx.x] = all_lit ? 1u : 0u;
    if (__syncthreads_or(err) && t == 0) atomicOr(&st->emit_err, 4u);
}

// Cross-tile links, resolved in parallel by pointer jumping over every tile with links at once: round r
// replaces each link by its target's own entry (a literal tile's entries are its literals), so a chain of h
// tiles needs ceil(log2 h) + 1 rounds and every tile advances in every round; a round whose predecessor
// left nothing unresolved returns at once.  Entries are read and written in place while other workgroups
// advance them: every such access is a relaxed agent-scope atomic (single-copy atomic 32-bit entries, no
// data race in the HIP memory model), and any value read is an ancestor on the same chain — an older entry
// or one another workgroup already advanced — so the rounds only converge faster.  No ordering between
// entries is needed: each entry is self-contained (a literal, or a position whose entry is still valid).
#ifndef RDX_PINF_XHOPS
#define RDX_PINF_XHOPS 2
#endif
#ifndef RDX_PINF_XPER
#define RDX_PINF_XPER 8
#endif
constexpr uint32_t kXThreads = 256, kXPer = RDX_PINF_XPER, kXPerTile = kTile / (kXThreads * kXPer);
constexpr uint32_t kXHops = RDX_PINF_XHOPS;   // links followed per entry and round

__device__ __forceinline__ uint32_t xld(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kXThreads) void k_pinf_xhop(PinfArgs a, uint32_t r) {
    PinfState *st = a.state;
    if (r && !st->xmore[r - 1]) return;
    const uint64_t N = st->total;
    const uint32_t tile = blockIdx.x / kXPerTile;
    if (a.tflag[tile]) return;
    // entry j of a thread is base + t + 256 j: each load instruction reads 64 consecutive entries, and
    // their targets (the consecutive sources of a match) are consecutive too
    const uint64_t base = (uint64_t)tile * kTile + (blockIdx.x % kXPerTile) * (kXThreads * kXPer) + threadIdx.x;
    bool more = false;
    uint32_t v[kXPer], w[kXPer];
#pragma unroll
    for (uint32_t j = 0; j < kXPer; ++j) {
        const uint64_t i = base + kXThreads * j;
        v[j] = i < N ? xld(a.src + i) : kFlag;
    }
    // the targets' entries as independent loads (a literal reads its own slot; past the end, the first)
#pragma unroll
    for (uint32_t j = 0; j < kXPer; ++j) {
        const uint64_t i = base + kXThreads * j;
        w[j] = xld(a.src + ((v[j] & kFlag) ? (i < N ? i : 0) : v[j]));
    }
#pragma unroll
    for (uint32_t h = 1; h < kXHops; ++h) {
#pragma unroll
        for (uint32_t j = 0; j < kXPer; ++j)
            if (!(v[j] & kFlag) && !(w[j] & kFlag)) w[j] = xld(a.src + w[j]);
    }
#pragma unroll
    for (uint32_t j = 0; j < kXPer; ++j) {
        const uint64_t i = base + kXThreads * j;
        if (!(v[j] & kFlag)) {
            more |= !(w[j] & kFlag);
            __hip_atomic_store(a.src + i, w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // one plain store per workgroup that left a link (same-address atomics from every wave serialise in
    // L2 and cost a full round's time); every store writes the same 1
    if (__syncthreads_or(more) && threadIdx.x == 0 &&
        !__hip_atomic_load(&st->xmore[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_store(&st->xmore[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the bytes of every tile with links (an entry still a link after the rounds is an inconsistency)
__global__ __launch_bounds__(kXThreads) void k_pinf_xout(PinfArgs a) {
    PinfState *st = a.state;
    const uint64_t N = st->total;
    const uint32_t tile = blockIdx.x / kXPerTile;
    if (a.tflag[tile]) return;
    const uint64_t i0 = (uint64_t)tile * kTile + (blockIdx.x % kXPerTile) * (kXThreads * kXPer) + kXPer * threadIdx.x;
    bool err = false;
    if (i0 + kXPer <= N) {
        const uint4 p = gld<uint4>(reinterpret_cast<const uint4 *>(a.src + i0)), q = gld<uint4>(reinterpret_cast<const uint4 *>(a.src + i0 + 4));
        err = !((p.x & p.y & p.z & p.w & q.x & q.y & q.z & q.w) & kFlag);
        const uint32_t lo = (p.x & 0xff) | (p.y & 0xff) << 8 | (p.z & 0xff) << 16 | (p.w & 0xff) << 24;
        const uint32_t hi = (q.x & 0xff) | (q.y & 0xff) << 8 | (q.z & 0xff) << 16 | (q.w & 0xff) << 24;
        gst<uint64_t>(reinterpret_cast<uint64_t *>(a.out + i0), (uint64_t)hi << 32 | lo);
    } else {
        for (uint64_t i = i0; i < N; ++i) {
            const uint32_t v = a.src[i];
            err |= !(v & kFlag);
            a.out[i] = (uint8_t)v;
        }
    }
    if (__ballot(err) && (threadIdx.x & 63) == 0) atomicOr(&st->emit_err, 4u);
}

// ---- 6. bytes + checksums -----------------------------------------------------------------------------------
constexpr uint32_t kAdler = 65521;

// GF(2) polynomial arithmetic modulo the CRC-32 polynomial (reflected: bit 31 is x^0), the operation of
// zlib's crc32.c multmodp / x2nmodp (zlib 1.2.12+, (C) Jean-loup Gailly and Mark Adler, zlib license): a
// third-party algorithm, not the reference's code.  Branch-free here (32 steps), and the shifts x^(8n)
// come from a compile-time table: x^(8 n) = T0[n & 255] T1[(n >> 8) & 255] T2[..] T3[..], three products
// instead of an exponentiation by squaring per thread (which cost k_pinf_finish 150 us on a 4 MiB gzip).
__host__ __device__ constexpr uint32_t gf2_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int k = 0; k < 32; ++k) {
        p ^= (a & (0x80000000u >> k)) ? b : 0u;
        b = (b & 1u) ? (b >> 1) ^ 0xedb88320u : b >> 1;
    }
    return p;
}
struct X8nTable {
    uint32_t t[4][256];
};
constexpr X8nTable make_x8n_table() {
    X8nTable r{};
    uint32_t e = 0x00800000u;   // x^8 (reflected: bit 31 - 8)
    for (int i = 0; i < 4; ++i) {
        r.t[i][0] = 0x80000000u;   // x^0
        for (int j = 1; j < 256; ++j) r.t[i][j] = gf2_mul(r.t[i][j - 1], e);
        // x^(8 * 256^(i+1)) = (x^(8 * 256^i))^256: eight squarings
        for (int k = 0; k < 8; ++k) e = gf2_mul(e, e);
    }
    return r;
}
__constant__ X8nTable c_x8n = make_x8n_table();

__global__ __launch_bounds__(256) void k_pinf_finish(PinfArgs a) {
    __shared__ uint32_t crc_tab[256];
    __shared__ uint32_t x8[4][256];
    __shared__ uint64_t r1[4], r2[4];
    __shared__ uint32_t rc[4];
    PinfState *st = a.state;
    const uint32_t t = threadIdx.x;
    const uint64_t N = st->total;
    const bool gz = a.format == RDX_COMPRESSION_GZIP;
    if (gz) {
        uint32_t c = t;
        for (int k = 0; k < 8; ++k) c = c & 1 ? (c >> 1) ^ 0xedb88320u : c >> 1;
        crc_tab[t] = c;
        for (int i = 0; i < 4; ++i) x8[i][t] = c_x8n.t[i][t];
    }
    __syncthreads();
    // segment of this workgroup, slice of this thread (multiples of 4 bytes)
    const uint64_t seg = ((N + gridDim.x - 1) / gridDim.x + 1023) / 1024 * 1024;
    const uint64_t s0 = (uint64_t)blockIdx.x * seg;
    const uint64_t sl = seg / 256;
    const uint64_t b0 = min(N, s0 + t * sl), b1 = min(N, s0 + (t + 1) * sl);
    uint64_t sa = 0, sw = 0;
    uint32_t c = 0xffffffffu;
    for (uint64_t o = b0; o < b1; o += 4) {
        const uint32_t k = (uint32_t)min<uint64_t>(4, b1 - o);
        uint32_t word = 0;
        if (k == 4) word = gld<uint32_t>(reinterpret_cast<const uint32_t *>(a.out + o));   // (out: 16-byte aligned)
        else for (uint32_t i = 0; i < k; ++i) word |= (uint32_t)a.out[o + i] << (8 * i);
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t by = (word >> (8 * i)) & 0xff;
            if (gz) c = crc_tab[(c ^ by) & 0xff] ^ (c >> 8);
            sa += by;
            sw += (b1 - (o + i)) * by;   // weight: bytes of the slice from this one to its end
        }
    }
    // fold to the whole stream: Adler s2 gains (bytes after the slice) x s1; CRC shifts by those bytes
    const uint64_t after = N - b1;
    uint64_t p1 = sa % kAdler, p2 = (sw % kAdler + (after % kAdler) * p1) % kAdler;
    uint32_t pc = 0;
    if (gz && b1 > b0) {   // the slice's CRC shifted past the bytes after it (after < 2^31)
        const uint32_t sh = gf2_mul(gf2_mul(x8[0][after & 255], x8[1][(after >> 8) & 255]),
                                    gf2_mul(x8[2][(after >> 16) & 255], x8[3][(after >> 24) & 255]));
        pc = gf2_mul(sh, c ^ 0xffffffffu);
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        p1 += (uint64_t)__shfl_xor((long long)p1, m, 64);
        p2 += (uint64_t)__shfl_xor((long long)p2, m, 64);
        pc ^= (uint32_t)__shfl_xor((int)pc, m, 64);
    }
    if ((t & 63) == 0) {
        r1[t / 64] = p1 % kAdler;
        r2[t / 64] = p2 % kAdler;
        rc[t / 64] = pc;
    }
    __syncthreads();
    if (t == 0) {
        const uint64_t q1 = (r1[0] + r1[1] + r1[2] + r1[3]) % kAdler, q2 = (r2[0] + r2[1] + r2[2] + r2[3]) % kAdler;
        a.partial[3 * blockIdx.x + 0] = q1;
        a.partial[3 * blockIdx.x + 1] = q2;
        a.partial[3 * blockIdx.x + 2] = rc[0] ^ rc[1] ^ rc[2] ^ rc[3];
    }
}

__global__ __launch_bounds__(64) void k_pinf_check(PinfArgs a, uint32_t parts) {
    PinfState *st = a.state;
    const uint32_t t = threadIdx.x;
    const Stream S = make_stream(a);
    uint64_t s1 = 0, s2 = 0;
    uint32_t c = 0;
    for (uint32_t i = t; i < parts; i += 64) {
        s1 += a.partial[3 * i];
        s2 += a.partial[3 * i + 1];
        c ^= (uint32_t)a.partial[3 * i + 2];
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        s1 += (uint64_t)__shfl_xor((long long)s1, m, 64);
        s2 += (uint64_t)__shfl_xor((long long)s2, m, 64);
        c ^= (uint32_t)__shfl_xor((int)c, m, 64);
    }
    if (t) return;
    const uint64_t N = st->total, tb = st->trailer_byte;
    bool ok = st->emit_err == 0;
    if (a.format == RDX_COMPRESSION_ZLIB) {
        // Adler-32: s1 starts at 1, so s2 gains N more
        const uint32_t A1 = (uint32_t)((1 + s1) % kAdler), A2 = (uint32_t)((s2 + N) % kAdler);
        const uint32_t want = S.byte(tb) << 24 | S.byte(tb + 1) << 16 | S.byte(tb + 2) << 8 | S.byte(tb + 3);
        ok = ok && want == (A2 << 16 | A1);
    } else {
        const uint32_t crc = c;   // XOR of the slices' CRC-32s, each shifted past the bytes after it
        const uint32_t want = S.byte(tb) | S.byte(tb + 1) << 8 | S.byte(tb + 2) << 16 | S.byte(tb + 3) << 24;
        const uint32_t isz = S.byte(tb + 4) | S.byte(tb + 5) << 8 | S.byte(tb + 6) << 16 | S.byte(tb + 7) << 24;
        ok = ok && want == crc && isz == (uint32_t)N;
    }
    st->final_ok = ok ? 1 : 0;
    if (a.hslot)
        __hip_atomic_store(a.hslot + 3, (ok ? 1u : 0u) | (uint64_t)min(st->emit_err, 255u) << 8 | (uint64_t)a.tag << 48,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t launch_pinf_find(const PinfArgs &a, hipStream_t s) {
    const uint64_t n = a.end_byte - a.first_byte;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_pinf_find, dim3((uint32_t)((n + kFindBytes - 1) / kFindBytes)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_pinf_block(const PinfArgs &a, uint32_t first, uint32_t count, hipStream_t s) {
    hipLaunchKernelGGL(k_pinf_block, dim3(count), dim3(kLanes), 0, s, a, first, count);
    return hipGetLastError();
}
hipError_t launch_pinf_chain(const PinfArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_pinf_chain, dim3(1), dim3(kChainThreads), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_pinf_rest(const PinfArgs &a, uint32_t n_chain, uint64_t total, int cus, hipStream_t s) {
    if (n_chain) hipLaunchKernelGGL(k_pinf_emit, dim3(n_chain * kPinfEmitSplit), dim3(kEmitThreads), 0, s, a);
    if (a.mcap)
        hipLaunchKernelGGL(k_pinf_expand, dim3(std::min<uint32_t>(kExpandMaxBlocks, (a.mcap + 3) / 4)), dim3(256), 0, s, a);
    if (total) {
        hipLaunchKernelGGL(k_pinf_tile, dim3((uint32_t)((total + kTile - 1) / kTile)), dim3(kTileThreads), 0, s, a);
        const uint32_t tiles = (uint32_t)((total + kTile - 1) / kTile);
        // a round multiplies the tiles every unresolved link has covered by kXHops + 1, and a chain spans
        // at most tiles - 1: one round more than that needs
        uint32_t rounds = 1;
        for (uint64_t cov = 1; cov < tiles; cov *= kXHops + 1) ++rounds;
        for (uint32_t r = 0; r < rounds && tiles > 1; ++r)
            hipLaunchKernelGGL(k_pinf_xhop, dim3(tiles * kXPerTile), dim3(kXThreads), 0, s, a, r);
        if (tiles > 1) hipLaunchKernelGGL(k_pinf_xout, dim3(tiles * kXPerTile), dim3(kXThreads), 0, s, a);
    }
    const uint32_t parts = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kPinfMaxParts, (total + 4095) / 4096));
    hipLaunchKernelGGL(k_pinf_finish, dim3(parts), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pinf_check, dim3(1), dim3(64), 0, s, a, parts);
    return hipGetLastError();
}

}  // namespace rdx
