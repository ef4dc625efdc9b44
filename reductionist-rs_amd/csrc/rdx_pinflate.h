// Launch descriptor of the single-stream parallel inflate (k_pinflate.hip), shared by host and device.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rdx {

constexpr uint32_t kPinfMaxCand = 4096;   // block-start candidates per stream (more: the stream falls back)
#ifndef RDX_PINF_LANES
#define RDX_PINF_LANES 1024
#endif
constexpr uint32_t kPinfLanes = RDX_PINF_LANES;   // decode lanes per block (k_pinf_block / k_pinf_emit)
#ifndef RDX_PINF_EMIT_SPLIT
#define RDX_PINF_EMIT_SPLIT 8
#endif
// k_pinf_emit workgroups per chain block: each re-decodes kPinfLanes / kPinfEmitSplit of its lanes on a CU
// of its own (a block's lanes on one CU share its four SIMDs' issue slots), two threads a lane — each half
// from the symbol boundary k_pinf_block recorded at the lane's middle (PinfArgs::lmid)
constexpr uint32_t kPinfEmitSplit = RDX_PINF_EMIT_SPLIT;
static_assert(kPinfLanes % (32 * kPinfEmitSplit) == 0, "whole waves per emit workgroup");
constexpr uint32_t kPinfMaxParts = 1024;  // checksum segments
constexpr uint64_t kPinfTabBytes = 11392;  // one block's decode tables (k_pinflate.hip Tabs)
#ifndef RDX_PINF_TILE
#define RDX_PINF_TILE 32768
#endif
constexpr uint32_t kPinfTile = RDX_PINF_TILE;   // k_pinf_tile's tile of output entries (<= the 32 KiB window)
static_assert(kPinfTile <= 32768 && (kPinfTile & (kPinfTile - 1)) == 0, "tile size");
#ifndef RDX_PINF_LONG_MATCH
#define RDX_PINF_LONG_MATCH 32
#endif
constexpr uint32_t kPinfLongMatch = RDX_PINF_LONG_MATCH;   // matches this long are expanded by k_pinf_expand

enum : uint32_t { kPinfFallback = 0, kPinfOk = 1, kPinfMiss = 2 };

// one candidate block start, decoded
struct PinfBlk {
    uint64_t end;      // bit after its end-of-block code (stored: after its data)
    uint64_t bytes;    // output bytes
    uint64_t body;     // first bit of the body (stored: of the data)
    uint32_t status;   // 0 decoded, 1 error (on its own path)
    uint32_t nlanes;   // lanes with verified starts (the last one ends the block)
    uint32_t nlen, ndist;
};

struct PinfState {
    uint32_t n_cand, overflow;        // candidates found (k_pinf_find, + the host's forced ones)
    uint32_t n_chain, status;         // k_pinf_chain: blocks on the chain, kPinf*
    uint64_t miss_bit;                // kPinfMiss: the block start no candidate covers
    uint32_t miss_type, emit_err;     // its BTYPE; k_pinf_emit / k_pinf_finish errors
    uint64_t total;                   // output bytes
    uint64_t trailer_byte;            // the checksum trailer (aligned byte position)
    uint32_t final_ok, n_match;       // k_pinf_check's verdict; long-match records of k_pinf_emit
    uint32_t n_surv, pad;             // offsets k_pinf_find's screen passed to the full header test
    uint32_t xmore[32];               // k_pinf_xhop round r left links unresolved
};

struct PinfArgs {
    const uint32_t *w;      // the stream as dwords from its 4-byte aligned base
    uint64_t nw;            // dwords holding stream bytes
    uint32_t lmask;         // valid bytes of the last dword
    uint32_t format;        // RDX_COMPRESSION_GZIP / ZLIB
    uint64_t first_byte;    // the stream's first byte in aligned coordinates (its base's skew)
    uint64_t end_byte;      // first byte past it
    uint64_t end_bits;      // 8 * end_byte
    uint64_t *cand;         // [kPinfMaxCand] bit << 2 | type (0 stored: bit of LEN; 1 fixed; 2 dynamic;
                            //  3 dynamic, its header parsed by k_pinf_find: lens, blk body / nlen / ndist set)
    PinfBlk *blk;           // [kPinfMaxCand]
    uint64_t *lst;          // [kPinfMaxCand][kPinfLanes] lane starts
    uint32_t *lnb;          // [kPinfMaxCand][kPinfLanes] lane output bytes
    uint64_t *lmid;         // [kPinfMaxCand][kPinfLanes] a lane's first symbol boundary at or past its middle
                            //  (bit) | output bytes before it << 40; ~0: none recorded
    uint8_t *lens;          // [kPinfMaxCand][320] code lengths (k_pinf_find -> k_pinf_block)
    uint8_t *tabs;          // [kPinfMaxCand][kPinfTabBytes] decode tables (k_pinf_block -> k_pinf_emit)
    uint32_t *chain;        // [kPinfMaxCand] candidate of each chain block
    uint64_t *coff;         // [kPinfMaxCand] its output offset
    PinfState *state;
    uint32_t *src;          // [total] the source of every output byte
    uint8_t *out;           // [total] (16-byte aligned)
    uint64_t *partial;      // [kPinfMaxParts][3] checksum partials
    uint4 *mlist;           // [mcap] long matches (o, len, dist): written by k_pinf_expand
    uint32_t mcap;
    uint32_t *tflag;        // [ceil(total / 32 KiB)] k_pinf_tile: the tile is literals only
    uint64_t *prof;         // RDX_PINF_PROF: per-workgroup (start, end) of k_pinf_block, then k_pinf_emit; else null
    // page-locked coherent host memory, or null: tagged granules (payload | tag << 48) the host polls instead
    // of copying the state back after a stream synchronise — [0..2] k_pinf_chain's verdict, [3] k_pinf_check's
    uint64_t *hslot;
    uint32_t tag;           // this launch's tag (1..65535)
};
// k_pinf_chain's granules: [0] status | miss_type << 2 | n_chain << 4 | min(n_cand, 8191) << 17, [1] total,
// [2] miss_bit; k_pinf_check's: [3] final_ok | min(emit_err, 255) << 8
constexpr uint64_t kPinfPayload = (1ull << 48) - 1;

hipError_t launch_pinf_find(const PinfArgs &a, hipStream_t s);
hipError_t launch_pinf_block(const PinfArgs &a, uint32_t first, uint32_t count, hipStream_t s);
hipError_t launch_pinf_chain(const PinfArgs &a, hipStream_t s);
hipError_t launch_pinf_rest(const PinfArgs &a, uint32_t n_chain, uint64_t total, int cus, hipStream_t s);

}  // namespace rdx
