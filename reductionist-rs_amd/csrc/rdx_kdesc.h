// Plain-data descriptors handed from the host planner (rdx_plan.cpp) to the gfx950 kernels
// (rdx_kernels.hip).  Everything here is trivially copyable and passed BY VALUE as kernel
// arguments (< 4 KiB), so a launch needs no descriptor upload.
#pragma once
#include <stdint.h>

namespace rdx {

constexpr int kMaxKDims = 16;        // dims left after canonicalisation (unit dims dropped, merged)
constexpr int kInlineMissing = 16;   // missing_values lists up to this length travel in the args
constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)
constexpr int kPartialWords = 6;     // u64 words per partial record
constexpr int kRecordU64 = 2 * kPartialWords;  // u64 slots per hand-off record (each word = 2 tagged granules)
constexpr uint32_t kTicketShards = 8; // arrival counter shards per chunk
constexpr uint32_t kTicketStride = 64; // u32 words between counters: one 256 B line each
constexpr uint32_t kTicketWords = (1 + kTicketShards) * kTicketStride;

enum OpCode : uint32_t { OP_COUNT = 0, OP_MAX = 1, OP_MIN = 2, OP_SELECT = 3, OP_SUM = 4 };

// u32 index division by a runtime constant: q = umulhi64(n, magic) for n < 2^32, d < 2^32.
struct Div {
    uint64_t magic;  // ceil(2^64 / d); 0 encodes d == 1
    uint32_t d;
    uint32_t pad;
};

// Where the element values come from.  `fused` != 0: the chunk is byte-shuffled with
// element_size == sizeof(T) and element e's byte k lives at base[k * plane + e]
// (src/filters/shuffle.rs:32-83 inverted on the fly).  `bswap`: reverse the byte order of every
// element (src/array.rs:147-177, byte_order == NON_NATIVE).
struct KSrc {
    const uint8_t *base;                // single chunk (or NULL when ptrs is used)
    const uint8_t *const *ptrs;         // batch: device array of chunk base pointers
    uint64_t plane;                     // bytes per byte-plane (= chunk elements) when fused
    uint32_t fused;
    uint32_t bswap;
    uint32_t table;                     // 1: chunk i's base is tbl.p[i] of the kernel's own arguments
    uint32_t pad;
};

// Chunk pointers carried in the kernel arguments (a coalesced group of same-plan requests: no table
// upload between the host call and the kernel).
constexpr int kTableChunks = 64;
struct KChunkTable {
    const uint8_t *p[kTableChunks];
};

// Missing-data predicate (src/types/missing.rs:114-122).  Values are raw T bits.
struct KMissing {
    uint32_t kind;   // rdx_missing_kind
    uint32_t n;      // MISSING_VALUES length
    uint64_t v0, v1; // VALUE / VALID_MIN / VALID_MAX: v0; VALID_RANGE: v0=min, v1=max
    uint64_t inl[kInlineMissing];   // VALUES, n <= kInlineMissing (linear scan, reference order)
    const uint64_t *list;           // VALUES, n > kInlineMissing: sorted, -0.0 folded to +0.0 (binary search)
};

// Per-chunk outputs and the cross-workgroup reduction state.
struct KOut {
    uint8_t *body;            // response body (T or i64 values)
    int64_t *counts;          // response counts
    uint32_t *status;         // per-chunk status word (RDX_E_NAN_UNORDERED), may be NULL
    uint64_t body_stride;     // bytes between consecutive chunks' bodies (batch)
    uint64_t counts_stride;   // elements between consecutive chunks' counts (batch)
    uint64_t *partials;       // [chunk][block] x kPartialWords
    uint32_t *tickets;        // [chunk][kTicketWords] arrival counters, self-resetting
    uint32_t status_any;      // 1: one status word for all chunks (chunks = outputs of an axis
                              // reduction), NaN ORed in; the caller clears it when a NaN can set it
    uint32_t epoch;           // this launch's hand-off tag (never 0): records carry it per granule
    uint32_t fold_last;       // 1: the chunk's LAST block (the last one dispatched) folds the records,
                              // polling them; no arrival counters (rdx_device.hpp arrive_and_fold);
                              // 2: the same, order-free folds through atomics (rdx_device.hpp atomic_fold)
    uint32_t host_slots;      // 1: `body` is a page-locked host slot of 3 tagged granules per chunk
                              // (value lo, value hi, count | status), written with system-scope stores
#if RDX_PROBES
    uint32_t drop_block;      // probe builds: 1 + the grid block that skips publishing (0: none)
    uint32_t pad_probe;
#endif
};

// Reduction over ALL axes of a view whose elements form one ascending contiguous run
// [off, off + n) of the chunk (after flipping negative strides).  rank(e) = r0 + (e - off) * rs
// orders ±0 ties the way ndarray's fold visits them.
struct KAllContig {
    KSrc src;
    KMissing miss;
    KOut out;
    uint64_t off, n;
    int64_t r0, rs;
    uint32_t filter_semantics;  // Count(All) uses missing_filter (operations.rs:25-33)
    uint32_t blocks_per_chunk;
    KChunkTable tbl;            // src.table: chunk pointers (last: only this much is read)
};

// A strided view: dims innermost-first.  offset(e) = base_off + sum idx_k * vstride_k,
// rank(e) = r0 + sum idx_k * rstride_k.
struct KView {
    int32_t ndim;
    int32_t pad;
    int64_t base_off;
    int64_t r0;
    uint64_t n;                       // number of elements (< 2^32)
    uint32_t count[kMaxKDims];
    Div div[kMaxKDims];
    int64_t vstride[kMaxKDims];
    int64_t rstride[kMaxKDims];
};

struct KAllStrided {
    KSrc src;
    KMissing miss;
    KOut out;
    KView view;
    uint32_t filter_semantics;
    uint32_t blocks_per_chunk;
    uint32_t vec;       // elements per 16-byte lane load along the contiguous inner dim (1 = scalar)
    uint32_t pad;
    KChunkTable tbl;    // src.table: chunk pointers
};

// Reduction over a subset of axes.  Output o (C order over kept dims) reduces the elements
// base_off + okept(o) + sum over reduced dims.  Work is split into `slices` slices of the reduced
// index range; with slices > 1 every slice publishes a partial record and the last slice to arrive
// for an output (rows) or output tile (cols) folds them in the same launch.
struct KAxis {
    KSrc src;
    KMissing miss;
    KOut out;
    KView kept;      // kept dims innermost-first in the lane/thread enumeration order;
                     // rstride here = output C-order stride of that dim
    KView red;       // reduced dims innermost-first; rstride = tie rank stride
    uint64_t n_out;
    uint64_t n_red;
    uint32_t slices;
    uint32_t mode;   // 0 = rows (a wave per output), 1 = cols (a lane per output)
    uint32_t vec;    // elements per 16-byte lane load (1 = scalar)
    uint32_t group;  // rows mode: lanes per output (power of two <= 64); 64/group outputs per wave
    uint32_t probe;  // tuning probe only (RDX_AXIS_PROBE): 1 = skip the slice fold, 2 = stop after streaming
    uint32_t fold_sep;  // cols, slices > 1: 0 = the tile's last slice folds (arrival counters); 1 = every
                        // slice only publishes and k_axis_cols_fold folds (a wave per output) next
};

// One request of a heterogeneous batch (k_multi.hip): an all-axes reduction over its own view of at
// most kMultiDims dims, with its own dtype / op / source / missing predicate / outputs.  Compact (152 B)
// so that a whole batch travels in the launch's kernel arguments: no table upload, no copy-engine or
// cross-stream event between the host call and the kernel.
constexpr int kMultiDims = 4;
constexpr int kMultiMaxItems = 24;   // requests per launch (the kernel arguments stay under 4 KiB)
enum : uint8_t {                     // KMultiReq::flags
    kMultiEq0 = 1,                   // x == v0 is missing  (MISSING_VALUE, MISSING_VALUES[0])
    kMultiEq1 = 2,                   // x == v1 is missing  (MISSING_VALUES[1])
    kMultiLo = 4,                    // x < v0 is missing   (VALID_MIN, VALID_RANGE)
    kMultiHi = 8,                    // x > v1 is missing   (VALID_MAX, VALID_RANGE)
    kMultiFilt = 16,                 // Count(All) semantics: NaN excluded under a valid_* predicate
    kMultiBswap = 32,                // non-native byte order
};
struct KMultiReq {
    const uint8_t *base;             // the request's chunk
    uint8_t *body;
    int64_t *counts;
    uint32_t *status;                // may be NULL
    int64_t base_off, r0;            // view origin (elements) and its rank
    uint64_t v0, v1;                 // predicate operands (bit patterns of T)
    uint64_t magic[kMultiDims - 1];  // Div::magic of count[0..2] (the outermost index needs no division)
    int32_t vstride[kMultiDims];     // element strides, innermost first (dims >= ndim: 0)
    int32_t rstride[kMultiDims];     // rank strides
    uint32_t count[kMultiDims - 1];  // dim extents, innermost first
    uint32_t n;                      // elements in the view (< 2^32)
    uint32_t block0;                 // first grid block of this request
    uint32_t bpc;                    // its blocks
    uint8_t dtype, op, vec, ndim;    // rdx_dtype, OpCode, elements per 16-B lane load (1 = scalar), dims
    uint8_t flags, pad8[3];
};
static_assert(sizeof(KMultiReq) == 152, "KMultiReq layout");

enum : uint32_t { kMultiFoldLast = 1, kMultiHostSlots = 2, kMultiAtomicFold = 4 };   // KMultiArgs::flags -> KOut
struct KMultiArgs {
    uint64_t *partials;              // hand-off records: request k's block b at (block0 + b) * kRecordU64
    uint32_t *tickets;               // request k's arrival counters at k * kTicketWords
    uint32_t n_items, epoch;
    uint32_t flags, pad;
    KMultiReq req[kMultiMaxItems];
};
static_assert(sizeof(KMultiArgs) <= 4096, "k_multi arguments exceed 4 KiB");

// Response serialisation (k_cbor.hip): the CBOR body's host-known segments and the count array to encode.
constexpr int kCborFixedMax = 1024;   // segment A (map head, "bytes", body head) + segment B (dtype .. count head)
constexpr int kCborTailMax = 64;      // segment D ("count_as_bytes" + head) + segment F ("byte_order": "little")
struct KCbor {
    uint8_t *out;               // the encoded response (device)
    const int64_t *counts;      // the count array's values (device)
    uint64_t n;                 // counts encoded as the array (0: empty or count_as_bytes)
    uint64_t c_off;             // offset of the array's first integer in out
    uint64_t b_off;             // offset of segment B (after the body)
    uint64_t raw_len;           // bytes of the count_as_bytes payload between D and F (copied by the host)
    uint64_t *out_len;          // device: total encoded length
    uint64_t *records;          // one word per tile: k_cbor_agg's encoded length, k_cbor_scan's offset
                                //   (staged form: n_tiles + 1 words, k_cbor_pack's lengths -> offsets + total)
    uint8_t *stage;             // staged form: tile t's encoded bytes at stage + t * kStageWave (k_cbor.hip)
    uint32_t *arrive;           // staged form: k_cbor_pack's sharded arrival counters (self-resetting)
    uint64_t *tagged;           // staged form: tile t's length as a tagged granule (the hand-off of rdx_device.hpp)
    uint32_t staged, epoch;
    uint32_t tpg, pad_;         // staged form: tiles per k_cbor_pack workgroup (records[n_tiles + 1 + g]: group offsets)
    uint32_t *status;           // staged form: RDX_E_DEVICE when a tile length never arrived (a device fault)
    const uint8_t *body;        // the response body (device), copied in-kernel when copy_body
    uint64_t body_len;
    uint32_t n_tiles, vec;
    uint32_t copy_body, copy_raw;   // in-kernel copies (alignment permitting), else hipMemcpyAsync
    uint32_t a_len, b_len, d_len, f_len;
    uint8_t fixed[kCborFixedMax];   // A then B
    uint8_t tail[kCborTailMax];     // D then F
};

// blosc2 chunks (k_blosc2.hip): chunk i = in[i] (in_len[i] bytes) -> out + i * cap; the decode
// scratch (same layout) holds the filtered blocks until k_blosc2_filter writes them into out.
struct KBlosc2Args {
    const uint8_t *const *in;   // device array of chunk pointers
    const uint64_t *in_len;     // device array of chunk lengths
    uint8_t *out;
    uint8_t *scratch;           // n * cap bytes (may be null when no chunk has an active filter)
    uint64_t cap;
    uint64_t *out_len;          // nbytes (also on RDX_INFLATE_OUTPUT_OVERFLOW, so the caller can resize)
    uint32_t *err;              // rdx_inflate_error; zeroed by the caller before the launch
    uint32_t n;
    uint32_t wg_per_chunk;      // workgroups (4 decoding waves each) per chunk
    // zlib- and zstd-coded block streams are not decoded here but appended to this table (slot = atomic
    // counter: zlib rows [0, z_capacity) counted by z_count[0], inflated by k_inflate afterwards; zstd rows
    // [z_capacity, 2 z_capacity) counted by z_count[1], decoded by k_blosc2_zstd); null: such chunks fail
    // with RDX_BLOSC2_UNSUPPORTED
    const uint8_t **z_in;       // stream start
    uint64_t *z_len;            // csize
    uint8_t **z_out;            // destination (decode scratch or output)
    uint64_t *z_cap;            // expected size (neblock)
    uint32_t *z_chunk;          // chunk index
    uint64_t *z_out_len;        // k_inflate: bytes produced
    uint32_t *z_err;            // k_inflate: rdx_inflate_error
    uint32_t *z_count;          // [2]: zlib / zstd entries used (zeroed by the caller)
    uint64_t z_capacity;        // rows per codec (the arrays hold 2 z_capacity)
};

// Element-wise map in output order: Select (operations.rs:487-526) and axis=[]
// (operations.rs:188-210, :58-67).  out index g -> element offset via `view` (dims
// innermost-first in OUTPUT order).
struct KMap {
    KSrc src;
    KMissing miss;
    KOut out;
    KView view;
    uint32_t kind;    // 0 = select (values + non-missing count), 1 = zero-axes values+0/1 counts,
                      // 2 = zero-axes counts only (Count op: body = counts)
    uint32_t vec;     // elements per 16-byte lane load/store (1 = scalar)
};

}  // namespace rdx
