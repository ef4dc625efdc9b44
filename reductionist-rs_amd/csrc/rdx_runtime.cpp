// C ABI implementation (include/rdx.h): device pool, per-stream workspaces, host-resident and
// device-resident execution.  No CPU fallback exists: without a gfx950 device every execute entry
// point fails with RDX_E_NO_DEVICE / RDX_E_DEVICE.
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <pthread.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <ctime>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <chrono>
#include <cstdio>
#include <deque>
#include <memory>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/rdx.h"
#include "rdx_cbor.hpp"
#include "rdx_kernels.hpp"
#include "rdx_jobsync.hpp"
#include "rdx_pinflate.h"
#include "rdx_plan.hpp"

using namespace rdx;

namespace {

rdx_status map_err(hipError_t e) {
    if (e == hipSuccess) return RDX_OK;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return RDX_E_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RDX_E_NO_DEVICE;
    return RDX_E_DEVICE;
}

#define RDX_HIP(call)                                      \
    do {                                                   \
        hipError_t _e = (call);                            \
        if (_e != hipSuccess) return map_err(_e);          \
    } while (0)

int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

// Tuning knobs, read from the environment once (getenv scans the whole environment: microseconds per
// request if done per launch).
struct Tuning {
    int blocks_per_cu = env_int("RDX_BLOCKS_PER_CU", 1);  // k_all_contig fill target (gpurun_out/bpcu2)
    int min_tiles = env_int("RDX_MIN_TILES_PER_BLOCK", 2);
    int force_bpc = env_int("RDX_FORCE_BPC", 0);   // tuning only
    int no_vec = env_int("RDX_NO_VEC", 0);
    int axis_rows_waves = env_int("RDX_AXIS_ROWS_WAVES_PER_CU", 16);   // sliced-rows fill target
    int axis_cols_wgs = env_int("RDX_AXIS_COLS_WGS_PER_CU", 4);        // sliced-cols fill target
    int axis_cols_vw = env_int("RDX_AXIS_COLS_VW", 0);                 // tuning only: force the cols lane width
    int axis_cols_w = env_int("RDX_AXIS_COLS_W", 32);                  // cap on the lanes per tile row (0: none)
    int axis_fold_kib = env_int("RDX_AXIS_FOLD_KIB", 64);              // cols fold bytes per tile (x2 with >= 8 streams)
    int axis_fold_sep = env_int("RDX_AXIS_FOLD_SEP", -1);              // cols fold launch: -1 auto, 0 off, 1 on
#if RDX_PROBES
    int axis_probe = env_int("RDX_AXIS_PROBE", 0);                     // phase probe (wrong results)
    int drop_block = env_int("RDX_DROP_BLOCK", 0);                     // fault injection: 1 + grid block
    int drop_launches = env_int("RDX_DROP_LAUNCHES", 0);               // ... in this many launches only (0: all)
#else
    int axis_probe = 0;   // product builds: the phase probe is compiled out (make EXTRA=-DRDX_PROBES=1)
#endif
    // few long contiguous rows: reduce each row as a chunk of the batched all-axes kernel
    int axis_rowbatch_kib = env_int("RDX_AXIS_ROWBATCH_KIB", 64);      // min row bytes (0 = off)
    int multi_blocks_per_cu = env_int("RDX_MULTI_BLOCKS_PER_CU", 5);   // k_multi fill target (5 resident per CU)
    int fold_last = env_int("RDX_FOLD_LAST", 2);                       // 2: + atomic folds, 1: records only, 0: arrival counters
    int fold_last_pairs = env_int("RDX_FOLD_LAST_PAIRS", 1);           // fold-last above kFoldLastChunks when bpc <= 2 (r06_fold_pairs_ab)
    int wait_spin = env_int("RDX_WAIT_SPIN", 200);                     // coalesced callers: pause spins, then futex
    int coalesce_depth = env_int("RDX_COALESCE_DEPTH", 1);            // launches in flight per coalescer stream (1-2)
    int direct_max = env_int("RDX_DIRECT_MAX", 1);                     // idle-queue fast path: callers launching at once
    int idle_us = env_int("RDX_DISPATCH_IDLE_US", 30);                 // dispatcher: polling without progress before it naps
    int nap_us = env_int("RDX_DISPATCH_NAP_US", 20);                   // ... and the nap between polls after that
    int host_spin_us = env_int("RDX_HOST_SPIN_US", -1);                // caller's spin before it sleeps (-1: by request size)
    int host_read_kib = env_int("RDX_HOST_READ_KIB", 4096);            // pinned chunks up to this: the kernel reads them over PCIe
    int host_read_wgs = env_int("RDX_HOST_READ_WGS", 8);               // ... with this many workgroups (few: profiles/r05_hread_probe)
    int phases = env_int("RDX_PHASES", 0);                             // phase statistics of the direct path (stderr at destroy)
    int cbor_staged = env_int("RDX_CBOR_STAGED", 1);                   // CBOR count arrays: pack -> place (0: agg / scan / encode)
    int pinflate = env_int("RDX_PINFLATE", 1);                         // a lone gzip / zlib stream: k_pinflate
    int pinflate_min = env_int("RDX_PINFLATE_MIN_BYTES", 1024);        // ... from this many compressed bytes
    int pinflate_prof = env_int("RDX_PINF_PROF", 0);                   // tuning: per-workgroup times to stderr
    int pinflate_forced = env_int("RDX_PINF_MAX_FORCED", 8);           // host-forced block starts before it declines
    int inflate_serial_max = env_int("RDX_INFLATE_SERIAL_MAX", 4096);  // declined streams up to this many bytes: k_inflate
#if RDX_PROBES
    int epoch_start = env_int("RDX_EPOCH_START", 0);                   // tests: start workspaces' tags near the wrap
#endif
};

const Tuning &tuning() {
    static const Tuning t;
    return t;
}

// KOut::fold_last of a fold-last launch: 2 = order-free ops fold through atomics (rdx_device.hpp atomic_fold),
// the rest through records; 1 = records for every op
uint32_t fold_mode() { return tuning().fold_last >= 2 ? 2u : 1u; }

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
};

}  // namespace

struct rdx_workspace {
    int device = 0;
    int cus = 256;
    bool inflate_fallback = false;     // rdx_context_config.inflate_fallback of the context that made it
    hipStream_t own_stream = nullptr;  // host path
    DevBuf<uint64_t> partials;   // hand-off records (tagged granules, rdx_device.hpp publish / collect)
    DevBuf<uint32_t> tickets;
    uint32_t epoch = 0;           // tag of the last launch's records
    DevBuf<uint8_t> scratch[2];
    DevBuf<uint64_t> miss_list;
    DevBuf<const uint8_t *> ptrs;
    // pinned staging for small uploads (missing list, batch pointer tables)
    uint8_t *pinned = nullptr;
    size_t pinned_cap = 0;
    hipEvent_t upload_done = nullptr;
    bool upload_pending = false;
    std::vector<uint8_t> last_list, last_ptrs;
    // host-path device buffers
    DevBuf<uint8_t> chunk;
    DevBuf<uint8_t> body;
    DevBuf<int64_t> counts;
    DevBuf<uint32_t> status;
    // decompression (k_inflate): stream tables, the decompressed chunk of a compressed request, and a
    // pinned readback of its length + error
    DevBuf<const uint8_t *> zptrs;
    DevBuf<uint64_t> zlens;
    DevBuf<uint64_t> zout_len;
    DevBuf<uint32_t> zerr;
    DevBuf<uint8_t> raw;
    DevBuf<uint8_t> zscratch;   // blosc2: decoded blocks before their filters (k_blosc2_filter)
    // blosc2: the table of zlib-coded block streams k_blosc2_decode hands to k_inflate
    DevBuf<const uint8_t *> zt_in;
    DevBuf<uint64_t> zt_len, zt_cap, zt_out_len;
    DevBuf<uint8_t *> zt_out;
    DevBuf<uint32_t> zt_chunk, zt_err, zt_count;
    std::vector<uint8_t> last_zptrs, last_zlens;
    // rdx_execute_cbor: the encoded response and its length
    DevBuf<uint8_t> cbor;
    DevBuf<uint64_t> cbor_len;
    uint64_t *zback = nullptr;  // pinned: [0] = out_len, [1] = err
    // page-locked readback of a host-path request: [0] status, [1] CBOR length, then small responses
    // (a D2H copy into pageable memory — a stack word, a caller's std::vector — is a synchronous, spinning
    // copy in HIP; into this block it is a DMA the caller can sleep through)
    uint64_t *h_back = nullptr;
    // the coalescer's idle-queue fast path: this workspace's own page-locked result slots (a one-request
    // lane launched on the caller's thread; rdx_device.hpp put_host_slot)
    uint64_t *h_slot = nullptr;
    // k_pinflate (one stream decoded by the whole device): its scratch arena, the byte sources, and the
    // page-locked copy of its state
    DevBuf<uint8_t> pinf;
    DevBuf<uint32_t> psrc;
    DevBuf<uint64_t> pprof;
    DevBuf<uint64_t> cbor_rec;   // k_cbor_agg / k_cbor_scan: per-tile lengths, then offsets
    DevBuf<uint8_t> cbor_stage;  // k_cbor_pack: the tiles' encoded bytes (the staged form)
    PinfState *pinf_back = nullptr;
    uint64_t *pinf_slot = nullptr;   // k_pinflate's tagged granules (PinfArgs::hslot), coherent page-locked
    uint32_t pinf_tag = 0;
    // pipelined host path (map_pipelined): a second stream and one event per piece
    hipStream_t aux_stream = nullptr;
    hipEvent_t piece_ev[8] = {};
    // a host chunk's H2D copy (a coalesced launch waits for it on the device), and the end of this
    // workspace's work for a caller that sleeps instead of spinning (wait_event)
    hipEvent_t copy_ev = nullptr, done_ev = nullptr;
    hipEvent_t ph_ev[3] = {};   // RDX_PHASES: timing events around the copy and the kernel
};

namespace {

// One k_multi launch lane of the coalescer: its own workspace (stream, hand-off records), an event, and a
// page-locked result slot per request that the kernel writes directly (no copy-engine round trip).
// Launches with up to this many chunks (folders) use the fold-by-last-block hand-off (KOut::fold_last).
constexpr uint64_t kFoldLastChunks = 64;
constexpr uint64_t kSlotWords = 3;   // rdx_device.hpp put_host_slot: value lo, value hi, count | status
struct Job;
struct Lane {
    rdx_workspace *ws = nullptr;
    bool owns_ws = true;                     // false: the stream / workspace of `twin` (launch-ahead pairs)
    Lane *twin = nullptr;                    // the lane sharing this stream, if any
    uint64_t *h_res = nullptr;               // kTableChunks slots, fine-grained page-locked memory
    Job *batch[kTableChunks] = {};
    bool group = false;                      // the launch: one plan over the batch's chunks (else k_multi)
    uint32_t n = 0;                          // requests of the launch (0: the lane is free)
    uint32_t remaining = 0;                  // of which not yet seen
    uint32_t tag = 0;                        // the launch's epoch (its slots' tag)
    uint32_t polls = 0;
    hipEvent_t done = nullptr;               // recorded behind each launch: its end (the fault fallback's test)
    std::chrono::steady_clock::time_point t0;   // when the launch was issued (dispatch statistics)
};

rdx_context_config effective_config(const rdx_context_config &c);
void destroy_lane(Lane *L);

// A request waiting for (or in) a coalesced launch.  The caller owns it and spins on `done`.
struct Job {
    // one plan over many chunks (a batched k_all_contig / k_all_strided launch): requests with the same
    // plan and launch descriptor (all but the chunk) share one; the descriptor's src.base is null here
    Mode mode = Mode::AllContig;
    uint32_t dtype = 0, op = 0, esz = 0;
    KAllContig contig{};
    KAllStrided strided{};
    const uint8_t *chunk = nullptr;        // device
    hipEvent_t dep = nullptr;              // the chunk's H2D copy (host chunks): the launch waits for it on the device
    bool host_read = false;                // `chunk` is page-locked host memory the kernel reads over PCIe
    // the heterogeneous form (k_multi), when the request fits it
    bool multi_ok = false;
    KMultiReq q{};                 // chunk / view / op; outputs are bound to the lane's slots at launch
    uint64_t body_bytes = 0, n_counts = 0;
    void *h_body = nullptr;        // host destinations
    int64_t *h_counts = nullptr;
    rdx_status st = RDX_OK;
    // futex word (rdx_jobsync.hpp): whoever completes the job writes `st` and the outputs, then exchanges
    // kJobDone in; after that exchange it touches no field of the Job (the caller may already have returned
    // and its stack frame be reused): a wake-up passes only the word's address to the kernel.
    std::atomic<uint32_t> state{kJobPending};
};

// A caller that waits for an event of its own stream without spinning: the entry's dispatcher thread
// polls the event with its lanes and wakes it (wait_event; the same one-word hand-off as a Job).
struct Waiter {
    hipEvent_t ev = nullptr;
    rdx_status st = RDX_OK;
    std::atomic<uint32_t> state{kJobPending};
};

// One entry of the context's device pool.
struct PoolEntry {
    int device = 0;
    std::mutex mu;                               // everything below but `outstanding` / the dispatcher's lanes
    std::condition_variable ws_cv;               // a workspace was released
    std::vector<rdx_workspace *> free_ws;
    std::vector<rdx_workspace *> all_ws;
    uint32_t busy = 0, creating = 0;
    // the coalescer: callers append to `jobs`; one dispatcher thread per entry launches and completes them
    std::condition_variable job_cv;              // the idle dispatcher waits here for work
    std::deque<Job *> jobs;
    std::vector<Waiter *> watch;                 // waiters handed to the dispatcher
    std::thread dispatcher;
    bool dispatcher_idle = false, stop = false;
    std::vector<Lane *> lanes;                   // dispatcher-owned
    // dispatcher timing (RDX_DISPATCH_STATS=1: printed to stderr when the context is destroyed)
    double t_launch = 0, t_flight = 0, t_complete = 0;
    uint64_t n_launch = 0, n_done = 0;
    std::atomic<uint64_t> outstanding{0};        // chunk bytes in flight (placement key)
    uint64_t requests = 0, coalesced = 0, launches = 0, waits = 0;
    uint32_t direct_active = 0;                  // idle-queue fast-path launches in flight (<= RDX_DIRECT_MAX)
    uint64_t direct = 0;                         // requests served by the fast path
    uint64_t placed_bytes = 0;                   // chunk bytes placed here, cumulative
    uint64_t peak_outstanding = 0;               // high-water mark of `outstanding`
    uint64_t host_reads = 0;                     // direct requests whose kernel read the host chunk itself
    std::atomic<uint64_t> sleeps{0};             // callers that slept in wait_event
};

}  // namespace

struct rdx_context {
    std::vector<int> devices;                    // per pool entry
    std::vector<std::unique_ptr<PoolEntry>> entries;
    rdx_context_config cfg{};
    std::mutex mu;                               // the pinned response pool
    std::atomic<uint64_t> rr{0};                 // tie-break start of the placement scan
    std::atomic<bool> served{false};             // a request has been placed: the configuration is frozen
    // page-locked response buffers of rdx_execute_owned (size class -> free blocks; block -> class)
    std::map<uint64_t, std::vector<void *>> pinned_free;
    std::map<void *, uint64_t> pinned_class;
    uint64_t pinned_cached = 0;
};

namespace {

template <class T>
rdx_status ensure(rdx_workspace *ws, DevBuf<T> &b, size_t n, hipStream_t s, bool zero = false) {
    if (b.cap >= n && b.p) return RDX_OK;
    if (b.p) {
        RDX_HIP(hipStreamSynchronize(s));  // in-flight work may still read the old buffer
        RDX_HIP(hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
    }
    size_t want = std::max<size_t>(n, 1);
    want = std::max(want, (size_t)(b.cap * 2));
    void *p = nullptr;
    RDX_HIP(hipMalloc(&p, want * sizeof(T)));
    b.p = static_cast<T *>(p);
    b.cap = want;
    // on the work stream: a null-stream memset is not ordered before kernels on a non-blocking stream
    if (zero) RDX_HIP(hipMemsetAsync(b.p, 0, want * sizeof(T), s));
    (void)ws;
    return RDX_OK;
}

// Stream-ordered upload of a small host array through the workspace's pinned staging buffer;
// identical consecutive uploads are skipped (e.g. a batch re-using the same chunk set).
rdx_status upload(rdx_workspace *ws, void *dst, const void *src, size_t bytes, std::vector<uint8_t> &cache,
                  hipStream_t s) {
    if (cache.size() == bytes && std::memcmp(cache.data(), src, bytes) == 0) return RDX_OK;
    if (ws->upload_pending) {
        RDX_HIP(hipEventSynchronize(ws->upload_done));
        ws->upload_pending = false;
    }
    if (ws->pinned_cap < bytes) {
        if (ws->pinned) RDX_HIP(hipHostFree(ws->pinned));
        ws->pinned = nullptr;
        ws->pinned_cap = 0;
        RDX_HIP(hipHostMalloc((void **)&ws->pinned, bytes, hipHostMallocDefault));
        ws->pinned_cap = bytes;
    }
    std::memcpy(ws->pinned, src, bytes);
    RDX_HIP(hipMemcpyAsync(dst, ws->pinned, bytes, hipMemcpyHostToDevice, s));
    RDX_HIP(hipEventRecord(ws->upload_done, s));
    ws->upload_pending = true;
    cache.assign(static_cast<const uint8_t *>(src), static_cast<const uint8_t *>(src) + bytes);
    return RDX_OK;
}

rdx_status ensure_aux(rdx_workspace *ws) {
    if (!ws->aux_stream) RDX_HIP(hipStreamCreateWithFlags(&ws->aux_stream, hipStreamNonBlocking));
    for (hipEvent_t &e : ws->piece_ev)
        if (!e) RDX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return RDX_OK;
}

uint32_t pick_bpc(uint64_t tiles, uint64_t n_chunks, int cus, int per_cu = 0) {
    const uint64_t target = (uint64_t)cus * (uint64_t)(per_cu > 0 ? per_cu : tuning().blocks_per_cu);
    uint64_t bpc = (target + n_chunks - 1) / n_chunks;
    const uint64_t min_tiles = (uint64_t)tuning().min_tiles;
    uint64_t cap = (tiles + min_tiles - 1) / min_tiles;
    if (bpc > cap) bpc = cap;
    if (bpc < 1) bpc = 1;
    if (bpc > 65536) bpc = 65536;
    const int force = tuning().force_bpc;
    if (force > 0) bpc = (uint64_t)force;
    return (uint32_t)bpc;
}

// The hand-off tag of the next launch on this workspace: never 0 (a cleared record buffer holds 0), and
// when the 16-bit tag wraps the record buffer is cleared on the stream first, so no stale granule
// can carry a current tag (rdx_device.hpp, tagged granules).
rdx_status next_epoch(rdx_workspace *ws, hipStream_t s, uint32_t &epoch) {
    if (++ws->epoch > 0xffffu) {   // 16-bit tags
        if (ws->partials.p) RDX_HIP(hipMemsetAsync(ws->partials.p, 0, ws->partials.cap * sizeof(uint64_t), s));
        ws->epoch = 1;
    }
    epoch = ws->epoch;
    return RDX_OK;
}

// Lanes may move 16 bytes of a view at once when its innermost dim is a contiguous, aligned run.
uint32_t vec_width(const KView &v, uint32_t esz, const uint8_t *base, const uint8_t *const *ptrs, uint64_t n_chunks,
                   bool fused) {
    const uint32_t vw = 16 / esz;
    if (fused || tuning().no_vec) return 1;
    if (v.ndim < 1 || v.vstride[0] != 1 || v.count[0] % vw != 0 || v.base_off % (int64_t)vw != 0) return 1;
    for (int k = 1; k < v.ndim; ++k)
        if (v.vstride[k] % (int64_t)vw != 0) return 1;
    if (ptrs) {
        for (uint64_t i = 0; i < n_chunks; ++i)
            if ((uintptr_t)ptrs[i] % 16) return 1;
    } else if ((uintptr_t)base % 16) {
        return 1;
    }
    return vw;
}

// Everything after planning for n_chunks chunks that share the plan (device pointers only).
rdx_status run_device(rdx_workspace *ws, ExecPlan &p, const uint8_t *d_chunk, const uint8_t *const *h_ptrs,
                      uint64_t n_chunks, uint64_t len, uint8_t *d_body, int64_t *d_counts, uint32_t *d_status,
                      hipStream_t s) {
    rdx_status st;
    const uint64_t body_bytes = p.info.body_bytes, n_counts = p.info.n_counts;
    const bool batchable = (p.mode == Mode::AllContig || p.mode == Mode::AllStrided) && p.unfused_es.empty();
    if (n_chunks > 1 && !batchable) {
        for (uint64_t i = 0; i < n_chunks; ++i) {
            if ((st = run_device(ws, p, h_ptrs[i], nullptr, 1, len, d_body ? d_body + i * body_bytes : nullptr,
                                 d_counts ? d_counts + i * n_counts : nullptr, d_status ? d_status + i : nullptr, s)))
                return st;
        }
        return RDX_OK;
    }
    if (n_chunks == 1 && h_ptrs) d_chunk = h_ptrs[0];

    // 1. filter chain (all but a fused final decode) into scratch
    const uint8_t *src = d_chunk;
    for (size_t i = 0; i < p.unfused_es.size(); ++i) {
        DevBuf<uint8_t> &dst = ws->scratch[i & 1];
        if ((st = ensure(ws, dst, len, s))) return st;
        RDX_HIP(launch_unshuffle(src, dst.p, len, p.unfused_es[i], ws->cus, s));
        src = dst.p;
    }

    // 2. missing list
    KMissing miss = p.miss;
    if (!p.miss_list.empty()) {
        if ((st = ensure(ws, ws->miss_list, p.miss_list.size(), s))) return st;
        if ((st = upload(ws, ws->miss_list.p, p.miss_list.data(), p.miss_list.size() * 8, ws->last_list, s))) return st;
        miss.list = ws->miss_list.p;
    }

    KSrc ksrc{};
    ksrc.base = src;
    ksrc.plane = len / p.esz;
    ksrc.fused = p.fused;
    ksrc.bswap = p.bswap;
    if (n_chunks > 1) {
        if ((st = ensure(ws, ws->ptrs, n_chunks, s))) return st;
        if ((st = upload(ws, (void *)ws->ptrs.p, h_ptrs, n_chunks * sizeof(void *), ws->last_ptrs, s))) return st;
        ksrc.ptrs = ws->ptrs.p;
        ksrc.base = nullptr;
    }
    KOut out{};
    if ((st = next_epoch(ws, s, out.epoch))) return st;
    out.body = d_body;
    out.counts = d_counts;
    out.status = d_status;
    out.body_stride = body_bytes;
    out.counts_stride = n_counts;
    // all-axes launches of few chunks: the last block of each chunk folds (no arrival counters)
    out.fold_last = n_chunks <= kFoldLastChunks && tuning().fold_last ? fold_mode() : 0u;
#if RDX_PROBES
    {
        static std::atomic<int> launches{0};
        const int k = launches.fetch_add(1, std::memory_order_relaxed);
        out.drop_block = tuning().drop_launches <= 0 || k < tuning().drop_launches ? (uint32_t)tuning().drop_block : 0u;
    }
#endif

    switch (p.mode) {
        case Mode::AllContig: {
            KAllContig a = p.all_contig;
            const uint64_t te = p.fused ? 4096 : 16384 / p.esz;
            // unshuffled f64 sums: the compensated arithmetic is exposed at one wave per SIMD, so two
            // workgroups per CU (8 x 64 MiB: 86-88 -> 81-82 us; an i64 sum of the same bytes is slower so,
            // 77 -> 80 us: profiles/r05_f64_variants.jsonl)
            const int per_cu = p.dtype == RDX_DTYPE_FLOAT64 && p.op == RDX_OP_SUM && !p.fused && p.miss.kind == 0 &&
                               tuning().blocks_per_cu == 1 ? 2 : 0;
            a.blocks_per_chunk = pick_bpc((a.n + te - 1) / te, n_chunks, ws->cus, per_cu);
            // many chunks of one or two blocks each: a folder waits at most for its partner, the block just
            // below it in dispatch order, which never waits itself, so fold-last is safe at any chunk count
            if (!out.fold_last && tuning().fold_last && tuning().fold_last_pairs && a.blocks_per_chunk <= 2)
                out.fold_last = fold_mode();
            if ((st = ensure(ws, ws->partials, n_chunks * a.blocks_per_chunk * kRecordU64, s, true))) return st;
            if ((st = ensure(ws, ws->tickets, n_chunks * kTicketWords, s, true))) return st;
            out.partials = ws->partials.p;
            out.tickets = ws->tickets.p;
            a.src = ksrc;
            a.miss = miss;
            a.out = out;
            RDX_HIP(launch_all_contig(p.dtype, p.op, a, (uint32_t)n_chunks, s));
            return RDX_OK;
        }
        case Mode::AllStrided: {
            KAllStrided a = p.all_strided;
            a.vec = vec_width(a.view, p.esz, src, n_chunks > 1 ? h_ptrs : nullptr, n_chunks, p.fused);
            {   // one round trip per lane when possible: kU vectors of `vec` elements per lane
                const uint64_t per_block = (uint64_t)kBlock * (a.vec > 1 ? 4 : 8);
                const uint64_t want = (a.view.n / a.vec + per_block - 1) / per_block;
                uint64_t cap = ((uint64_t)ws->cus * 8 + n_chunks - 1) / n_chunks;
                a.blocks_per_chunk = (uint32_t)std::max<uint64_t>(1, std::min(want, std::max<uint64_t>(cap, 1)));
                const int force = tuning().force_bpc;
                if (force > 0) a.blocks_per_chunk = (uint32_t)force;
            }
            if ((st = ensure(ws, ws->partials, n_chunks * a.blocks_per_chunk * kRecordU64, s, true))) return st;
            if ((st = ensure(ws, ws->tickets, n_chunks * kTicketWords, s, true))) return st;
            out.partials = ws->partials.p;
            out.tickets = ws->tickets.p;
            a.src = ksrc;
            a.miss = miss;
            a.out = out;
            RDX_HIP(launch_all_strided(p.dtype, p.op, a, (uint32_t)n_chunks, s));
            return RDX_OK;
        }
        case Mode::Axis: {
            KAxis a = p.axis;
            // the kernels clear the status word themselves unless a NaN can set it (float min/max)
            const bool can_fail = (p.dtype == RDX_DTYPE_FLOAT32 || p.dtype == RDX_DTYPE_FLOAT64) &&
                                  (p.op == RDX_OP_MIN || p.op == RDX_OP_MAX);
            if (d_status && (can_fail || a.n_out == 0)) RDX_HIP(hipMemsetAsync(d_status, 0, sizeof(uint32_t), s));
            if (a.n_out == 0) return RDX_OK;
            // Few long contiguous rows (the reduced axes form one unit-stride run per output): each
            // row is a chunk of the batched all-axes kernel, which streams at the contiguous read
            // rate and folds through the sharded hand-off instead of one wave per output's slices.
            const uint64_t rb_min = (uint64_t)tuning().axis_rowbatch_kib * 1024;
            if (rb_min && a.mode == 0 && a.red.ndim == 1 && a.red.vstride[0] == 1 && a.n_red * p.esz >= rb_min &&
                a.n_out <= (uint64_t)ws->cus * 4) {
                std::vector<const uint8_t *> rows(a.n_out);
                for (uint64_t t = 0; t < a.n_out; ++t) {
                    int64_t off = a.kept.base_off, oi = 0;
                    uint64_t q = t;
                    for (int k = 0; k < a.kept.ndim; ++k) {
                        const uint64_t idx = q % a.kept.count[k];
                        q /= a.kept.count[k];
                        off += (int64_t)idx * a.kept.vstride[k];
                        oi += (int64_t)idx * a.kept.rstride[k];
                    }
                    rows[(uint64_t)oi] = src + off * (p.fused ? 1 : (int64_t)p.esz);
                }
                KAllContig c{};
                c.off = 0;
                c.n = a.n_red;
                c.r0 = a.red.r0;
                c.rs = a.red.rstride[0];
                c.filter_semantics = 0;   // fold semantics, as k_axis.hip fold_in
                const uint64_t te = p.fused ? 4096 : 16384 / p.esz;
                c.blocks_per_chunk = pick_bpc((c.n + te - 1) / te, a.n_out, ws->cus);
                if ((st = ensure(ws, ws->ptrs, a.n_out, s))) return st;
                if ((st = upload(ws, (void *)ws->ptrs.p, rows.data(), a.n_out * sizeof(void *), ws->last_ptrs, s)))
                    return st;
                if ((st = ensure(ws, ws->partials, a.n_out * c.blocks_per_chunk * kRecordU64, s, true))) return st;
                if ((st = ensure(ws, ws->tickets, a.n_out * kTicketWords, s, true))) return st;
                c.src = ksrc;
                c.src.base = nullptr;
                c.src.ptrs = ws->ptrs.p;
                c.miss = miss;
                c.out = out;
                c.out.body_stride = p.op == RDX_OP_COUNT ? 8 : p.esz;
                c.out.counts_stride = 1;
                c.out.status_any = 1;
                c.out.fold_last = a.n_out <= kFoldLastChunks && tuning().fold_last ? fold_mode() : 0u;
                c.out.partials = ws->partials.p;
                c.out.tickets = ws->tickets.p;
                RDX_HIP(launch_all_contig(p.dtype, p.op, c, (uint32_t)a.n_out, s));
                return RDX_OK;
            }
            uint64_t slices = 1;
            // vw-element lanes when every stride keeps vectors aligned and inside one dim
            auto vec_ok = [&](uint32_t vw) {
                if (vw == 1) return true;
                const KView &inner = a.mode == 0 ? a.red : a.kept;
                bool ok = !p.fused && !tuning().no_vec && inner.ndim >= 1 && inner.vstride[0] == 1 &&
                          inner.count[0] % vw == 0 && a.kept.base_off % (int64_t)vw == 0 &&
                          (uintptr_t)src % (vw * p.esz) == 0;
                for (int k = 0; k < a.kept.ndim; ++k) ok = ok && (a.mode == 1 && k == 0 ? true : a.kept.vstride[k] % (int64_t)vw == 0);
                for (int k = 0; k < a.red.ndim; ++k) ok = ok && (a.mode == 0 && k == 0 ? true : a.red.vstride[k] % (int64_t)vw == 0);
                return ok;
            };
            const uint32_t vmax = 16 / p.esz;
            a.group = 64;
            a.probe = (uint32_t)tuning().axis_probe;
            a.fold_sep = 0;
            if (a.mode == 0) {
                a.vec = vec_ok(vmax) ? vmax : 1;
                const uint64_t target = (uint64_t)ws->cus * tuning().axis_rows_waves;     // waves
                const uint64_t nrv = a.n_red / a.vec;
                // short rows: just enough lanes per output for 4 loads in flight per lane
                const uint64_t want = (nrv + 3) / 4;
                while (a.group > 1 && a.group / 2 >= want) a.group /= 2;
                if (a.group == 64 && a.n_out < target)
                    slices = std::min<uint64_t>((target + a.n_out - 1) / a.n_out, (nrv + 255) / 256);
            } else {
                // Tile width W lanes x vw outputs; slices of the reduced rows fill the chip, bounded so
                // that the last slice's fold (one workgroup, 256/W parallel slice streams) stays short:
                // fold bytes per tile <= 64 KiB (128 KiB with >= 8 streams), <= 16 slices per stream.
                // (A two-level fold over slice groups, measured this round, did not beat this bound.)
                const bool frank = (p.dtype == RDX_DTYPE_FLOAT32 || p.dtype == RDX_DTYPE_FLOAT64) &&
                                   (p.op == RDX_OP_MIN || p.op == RDX_OP_MAX);
                const uint64_t rec = 8 * ((p.op != RDX_OP_COUNT) + (p.op == RDX_OP_SUM && p.dtype == RDX_DTYPE_FLOAT64) +
                                          1 + (frank ? 3 : 0));
                const uint64_t target = (uint64_t)ws->cus * tuning().axis_cols_wgs;      // workgroups
                uint64_t best_wgs = 0;
                // at most 2 outputs per lane: 4-wide f32 lanes stream as fast but double the slice
                // records each lane publishes and folds (axis0 4096^2 f32: 20 vs 32 us, 64x1024x256
                // axis 1: 20 vs 26 us, tools/gpu_foldkib.sh)
                const uint32_t vtop = tuning().axis_cols_vw ? vmax : std::min<uint32_t>(vmax, 2);
                for (uint32_t vw = vtop; vw >= 1; vw /= 2) {
                    if (!vec_ok(vw)) continue;
                    // (tuning: a forced width the dtype cannot take is ignored)
                    if (tuning().axis_cols_vw && (uint32_t)tuning().axis_cols_vw <= vmax &&
                        vw != (uint32_t)tuning().axis_cols_vw)
                        continue;
                    const uint64_t nkv = a.n_out / vw;
                    uint32_t W = 64;
                    while (W > 1 && W / 2 >= nkv) W /= 2;
                    // at most 32 lanes per row of a tile: narrower tiles need fewer slices to fill the chip,
                    // so fewer slice records and a shorter fold ([4096,4096] f32 axis 0: 21.5 -> 18.7 us,
                    // [64,1024,256] axis 1: 18.9 -> 17.9 us; W 16 / 8 / 4 no better or slower:
                    // profiles/r03_axis_cols_sweep.jsonl)
                    if (tuning().axis_cols_w) W = std::min<uint32_t>(W, (uint32_t)tuning().axis_cols_w);
                    const uint64_t tiles = (nkv + W - 1) / W, G = kBlock / W, R = 64 / W;
                    const uint64_t fold = (uint64_t)tuning().axis_fold_kib * 1024;
                    const uint64_t budget = std::min<uint64_t>(fold * std::max<uint64_t>(1, G / 4), 2 * fold);
                    const uint64_t smax = std::max<uint64_t>(
                        1, std::min({budget / (W * vw * rec), 16 * G, a.n_red / (16 * R)}));
                    uint64_t sl = std::max<uint64_t>(1, std::min((target + tiles - 1) / tiles, smax));
                    // few tiles whose fold budget leaves the chip underfilled (tall, narrow): more slices
                    // and the separate fold launch (k_axis_cols_fold, parallel across outputs)
                    bool sep = tuning().axis_fold_sep == 1;
                    // (below a quarter of the target: at 3/8, [4096,4096] f32 axis-0 max, the in-kernel
                    // fold measured 25.7 us vs 33.9 us with the fold launch, tools/gpu_colsmax.sh)
                    if (tuning().axis_fold_sep < 0 && tiles * sl * 4 < target) sep = true;
                    if (sep) {
                        const uint64_t target2 = (uint64_t)ws->cus * 8;
                        sl = std::max<uint64_t>(1, std::min<uint64_t>({(target2 + tiles - 1) / tiles,
                                                                       a.n_red / (16 * R), 4096}));
                    }
                    const uint64_t wgs = tiles * sl;
                    if (wgs > best_wgs) {
                        best_wgs = wgs;
                        a.vec = vw;
                        a.group = W;
                        slices = sl;
                        a.fold_sep = sep ? 1u : 0u;
                    }
                    if (wgs * 2 >= target) break;   // the widest lanes that fill the chip
                }
            }
            slices = std::max<uint64_t>(1, std::min<uint64_t>(slices, 65535));
            a.slices = (uint32_t)slices;
            if (slices > 1) {   // partial records + a self-resetting arrival counter (own L2 line) per output / tile
                const uint64_t tiles = (a.n_out / a.vec + a.group - 1) / a.group;
                const uint64_t recs = a.mode == 0 ? a.n_out : tiles * a.group * a.vec;
                if ((st = ensure(ws, ws->partials, recs * slices * kRecordU64, s, true))) return st;
                if ((st = ensure(ws, ws->tickets, std::max<uint64_t>((a.mode == 0 ? a.n_out : tiles) * kTicketStride, kTicketWords),
                                 s, true)))
                    return st;
                out.partials = ws->partials.p;
                out.tickets = ws->tickets.p;
            }
            a.src = ksrc;
            a.miss = miss;
            a.out = out;
            RDX_HIP(launch_axis(p.dtype, p.op, a, ws->cus, s));
            return RDX_OK;
        }
        case Mode::Map: {
            KMap a = p.map;
            a.vec = vec_width(a.view, p.esz, src, nullptr, 1, p.fused);
            if ((uintptr_t)d_body % 16 || (a.kind != 0 && (uintptr_t)d_counts % 16)) a.vec = 1;
            if (a.view.n == 0) {
                if (d_status) RDX_HIP(hipMemsetAsync(d_status, 0, sizeof(uint32_t), s));
                if (a.kind == 0) RDX_HIP(hipMemsetAsync(d_counts, 0, sizeof(int64_t), s));
                return RDX_OK;
            }
            if (a.kind == 0) {
                if ((st = ensure(ws, ws->partials, (uint64_t)ws->cus * 8 * 2, s, true))) return st;
                if ((st = ensure(ws, ws->tickets, kTicketWords, s, true))) return st;
                out.partials = ws->partials.p;
                out.tickets = ws->tickets.p;
            }
            a.src = ksrc;
            a.miss = miss;
            a.out = out;
            RDX_HIP(launch_map(p.dtype, a, ws->cus, s));
            return RDX_OK;
        }
    }
    return RDX_E_INVALID_ARGUMENT;
}

thread_local uint32_t g_inflate_error = RDX_INFLATE_OK;
thread_local uint32_t g_inflate_path = RDX_INFLATE_PATH_NONE;

// ---- one gzip / zlib stream decoded by the whole device (k_pinflate.hip) ------------------------------
// Returns RDX_OK with the stream's bytes in ws->raw (*raw_len of them), kNotDecoded when the sequential
// decoder must run (an error anywhere, a chain it could not follow), or a device / memory error.
const rdx_status kNotDecoded = static_cast<rdx_status>(254);

// Wait for granules [i0, i1) of the pinflate slot to carry `tag` (a spin with pauses; the stream is asked
// every 256 turns whether it has ended): false when it ended or failed without them — the caller then reads
// the state back through the stream, which reports any device error.
bool pinf_wait(const uint64_t *slot, uint32_t i0, uint32_t i1, uint32_t tag, hipStream_t s) {
    auto fresh = [&] {
        bool f = true;
        for (uint32_t i = i0; i < i1; ++i) f &= (__atomic_load_n(slot + i, __ATOMIC_ACQUIRE) >> 48) == tag;
        return f;
    };
    for (uint32_t it = 1;; ++it) {
        if (fresh()) return true;
        if ((it & 255) == 0) {
            const hipError_t e = hipStreamQuery(s);
            if (e != hipErrorNotReady) {
                (void)hipGetLastError();
                return e == hipSuccess && fresh();
            }
        }
        __builtin_ia32_pause();
    }
}
constexpr uint64_t kPinfKeepSources = 256ull << 20;   // source entries kept between streams (1 GiB)

rdx_status pinflate_stream(rdx_workspace *ws, uint32_t compression, const uint8_t *d_src, uint64_t len, hipStream_t s,
                           uint64_t *raw_len) {
    rdx_status st;
    // arena: state | cand | blk | chain | coff | partial | lens | lnb | lst | tabs | lmid
    constexpr uint64_t oState = 0, oCand = 256, oBlk = oCand + 8ull * kPinfMaxCand,
                       oChain = oBlk + sizeof(PinfBlk) * kPinfMaxCand, oCoff = oChain + 4ull * kPinfMaxCand,
                       oPart = oCoff + 8ull * kPinfMaxCand, oLens = oPart + 24ull * kPinfMaxParts,
                       oLnb = oLens + 320ull * kPinfMaxCand, oLst = oLnb + 4ull * kPinfMaxCand * kPinfLanes,
                       oTabs = oLst + 8ull * kPinfMaxCand * kPinfLanes, oMid = oTabs + kPinfTabBytes * kPinfMaxCand,
                       oEnd = oMid + 8ull * kPinfMaxCand * kPinfLanes;
    static_assert(sizeof(PinfState) <= 256, "state slot");
    if ((st = ensure(ws, ws->pinf, oEnd, s))) return st;
    if (!ws->pinf_back) RDX_HIP(hipHostMalloc((void **)&ws->pinf_back, sizeof(PinfState), hipHostMallocDefault));
    uint8_t *ar = ws->pinf.p;
    PinfArgs a{};
    const uint64_t skew = (uintptr_t)d_src & 3;
    a.w = reinterpret_cast<const uint32_t *>(d_src - skew);
    a.first_byte = skew;
    a.end_byte = skew + len;
    a.end_bits = 8 * a.end_byte;
    a.nw = (a.end_byte + 3) / 4;
    a.lmask = a.end_byte % 4 ? (1u << (8 * (a.end_byte % 4))) - 1 : 0xffffffffu;
    a.format = compression;
    a.state = reinterpret_cast<PinfState *>(ar + oState);
    a.cand = reinterpret_cast<uint64_t *>(ar + oCand);
    a.blk = reinterpret_cast<PinfBlk *>(ar + oBlk);
    a.chain = reinterpret_cast<uint32_t *>(ar + oChain);
    a.coff = reinterpret_cast<uint64_t *>(ar + oCoff);
    a.partial = reinterpret_cast<uint64_t *>(ar + oPart);
    a.lens = ar + oLens;
    a.lnb = reinterpret_cast<uint32_t *>(ar + oLnb);
    a.lst = reinterpret_cast<uint64_t *>(ar + oLst);
    a.tabs = ar + oTabs;
    a.lmid = reinterpret_cast<uint64_t *>(ar + oMid);
    if (tuning().pinflate_prof) {
        if ((st = ensure(ws, ws->pprof, 24ull * kPinfMaxCand, s))) return st;
        RDX_HIP(hipMemsetAsync(ws->pprof.p, 0, 192ull * kPinfMaxCand, s));
        a.prof = ws->pprof.p;
    }
    // the two points where the host needs the device's answer (the chain's verdict and size; the final check)
    // are read from tagged granules the kernels write into page-locked memory, not by copying the state back
    // after a stream synchronise (~20-40 us of idle device each, profiles/r06_pinflate_kernel_stats_final.csv)
    if (!tuning().pinflate_prof) {
        if (!ws->pinf_slot) {
            RDX_HIP(hipHostMalloc((void **)&ws->pinf_slot, 4 * sizeof(uint64_t), hipHostMallocCoherent));
            std::memset(ws->pinf_slot, 0, 4 * sizeof(uint64_t));
        }
        a.hslot = ws->pinf_slot;
    }
    auto next_tag = [&] {
        ws->pinf_tag = ws->pinf_tag % 65535 + 1;
        return ws->pinf_tag;
    };
    RDX_HIP(hipMemsetAsync(a.state, 0, sizeof(PinfState), s));
    RDX_HIP(launch_pinf_find(a, s));
    RDX_HIP(launch_pinf_block(a, 0, kPinfMaxCand, s));
    PinfState &h = *ws->pinf_back;
    for (uint32_t forced = 0;; ++forced) {
        a.tag = next_tag();
        RDX_HIP(launch_pinf_chain(a, s));
        if (a.hslot && pinf_wait(a.hslot, 0, 3, a.tag, s)) {
            const uint64_t g0 = a.hslot[0], g1 = a.hslot[1], g2 = a.hslot[2];
            h.status = (uint32_t)(g0 & 3);
            h.miss_type = (uint32_t)(g0 >> 2) & 3;
            h.n_chain = (uint32_t)(g0 >> 4) & 8191;
            h.n_cand = (uint32_t)(g0 >> 17) & 8191;
            h.total = g1 & kPinfPayload;
            h.miss_bit = g2 & kPinfPayload;
            h.overflow = 0;
        } else {
            RDX_HIP(hipMemcpyAsync(&h, a.state, sizeof(PinfState), hipMemcpyDeviceToHost, s));
            RDX_HIP(hipStreamSynchronize(s));
        }
        if (h.status != kPinfMiss) break;
        // a block start no candidate covers (a fixed-Huffman block, or a header the finder's zlib-encoder
        // rules reject): decode that one block and follow the chain again
        const uint32_t n = h.n_cand;
        // (a stream of many fixed-Huffman blocks, Z_FIXED, would take a host round trip per block: it is
        // declined after a few, so a decline costs little more than the finder and the block decode)
        if (forced >= (uint32_t)std::max(0, tuning().pinflate_forced) || n >= kPinfMaxCand || h.miss_type == 3)
            return kNotDecoded;
        const uint64_t e = h.miss_bit;
        const uint64_t key = h.miss_type == 0 ? (8 * ((e + 3 + 7) / 8)) << 2 : e << 2 | h.miss_type;
        const uint32_t n1 = n + 1;
        RDX_HIP(hipMemcpyAsync(a.cand + n, &key, sizeof key, hipMemcpyHostToDevice, s));
        RDX_HIP(hipMemcpyAsync(&a.state->n_cand, &n1, sizeof n1, hipMemcpyHostToDevice, s));
        RDX_HIP(launch_pinf_block(a, n, 1, s));
        RDX_HIP(hipStreamSynchronize(s));   // the host values above are on the stack
    }
    if (h.status != kPinfOk) {
        if (tuning().pinflate_prof)
            std::fprintf(stderr, "{\"pinf_declined\": {\"chain_status\": %u, \"n_chain\": %u, \"n_cand\": %u, "
                         "\"overflow\": %u}}\n", h.status, h.n_chain, h.n_cand, h.overflow);
        return kNotDecoded;
    }
    const uint64_t total = h.total;
    // the output, the sources, the long-match records (at most total / kPinfLongMatch of them), the tiles'
    // flags: about 5.5 bytes of HBM per output byte.  An allocation that fails here declines the stream (the
    // sequential decoder needs only the output) instead of failing the request.
    const uint64_t mcap = total / kPinfLongMatch, msta = (total + 3) / 4 * 4, tiles = (total + kPinfTile - 1) / kPinfTile;
    if ((st = ensure(ws, ws->raw, std::max<uint64_t>((total + 15) / 16 * 16, 16), s)) ||
        (st = ensure(ws, ws->psrc, std::max<uint64_t>(msta + 4 * mcap + tiles, 1), s))) {
        (void)hipGetLastError();
        return st == RDX_E_OUT_OF_MEMORY ? kNotDecoded : st;
    }
    a.src = ws->psrc.p;
    a.mlist = reinterpret_cast<uint4 *>(ws->psrc.p + msta);
    a.mcap = (uint32_t)mcap;
    a.tflag = ws->psrc.p + msta + 4 * mcap;
    a.out = ws->raw.p;
    a.tag = next_tag();
    RDX_HIP(launch_pinf_rest(a, h.n_chain, total, ws->cus, s));
    if (a.hslot && pinf_wait(a.hslot, 3, 4, a.tag, s)) {
        const uint64_t g3 = a.hslot[3];
        h.final_ok = (uint32_t)(g3 & 1);
        h.emit_err = (uint32_t)(g3 >> 8) & 0xff;
    } else {
        RDX_HIP(hipMemcpyAsync(&h, a.state, sizeof(PinfState), hipMemcpyDeviceToHost, s));
        RDX_HIP(hipStreamSynchronize(s));
    }
    if (a.prof) {   // tuning: the slowest workgroups of k_pinf_block / k_pinf_emit, phase by phase
        std::vector<uint64_t> pr(24ull * kPinfMaxCand);
        std::vector<uint64_t> keys(kPinfMaxCand);
        std::vector<PinfBlk> blks(kPinfMaxCand);
        std::vector<uint32_t> chain(kPinfMaxCand);
        RDX_HIP(hipMemcpy(pr.data(), a.prof, pr.size() * 8, hipMemcpyDeviceToHost));
        RDX_HIP(hipMemcpy(keys.data(), a.cand, keys.size() * 8, hipMemcpyDeviceToHost));
        RDX_HIP(hipMemcpy(blks.data(), a.blk, blks.size() * sizeof(PinfBlk), hipMemcpyDeviceToHost));
        RDX_HIP(hipMemcpy(chain.data(), a.chain, chain.size() * 4, hipMemcpyDeviceToHost));
        for (int k = 0; k < 2; ++k) {
            // (k_pinf_emit: kPinfEmitSplit workgroups per chain block)
            const uint32_t n = k == 0 ? std::min(h.n_cand, kPinfMaxCand) : std::min(h.n_chain * kPinfEmitSplit, kPinfMaxCand);
            uint64_t lo = ~0ull, hi = 0, worst = 0;
            uint32_t wi = 0;
            std::vector<uint64_t> d;
            for (uint32_t i = 0; i < n; ++i) {
                const uint64_t *w = &pr[8 * (k * kPinfMaxCand + i)];
                if (!w[0]) continue;
                lo = std::min(lo, w[0]);
                hi = std::max(hi, w[4]);
                d.push_back(w[4] - w[0]);
                if (w[4] - w[0] > worst) { worst = w[4] - w[0]; wi = i; }
            }
            std::sort(d.begin(), d.end());
            const uint32_t c = k == 0 ? wi : chain[wi / kPinfEmitSplit];
            const uint64_t *w = &pr[8 * (k * kPinfMaxCand + wi)];
            auto us = [&](uint64_t x) { return x > w[0] ? (x - w[0]) / 100.0 : -1.0; };
            std::fprintf(stderr, "{\"pinf_prof\": \"%s\", \"wgs\": %zu, \"span_us\": %.1f, \"median_us\": %.1f, "
                         "\"max_us\": %.1f, \"max_cand\": %u, \"type\": %u, \"bytes\": %llu, \"bits\": %llu, "
                         "\"lanes\": %u, \"status\": %u, \"t_tables\": %.1f, \"t_pass0\": %.1f, \"t_agree\": %.1f, "
                         "\"rounds\": %llu, \"t_parsed\": %.1f, \"exts\": %llu, \"walks\": %llu}\n", k ? "emit" : "block", d.size(),
                         (hi - lo) / 100.0, d.empty() ? 0.0 : d[d.size() / 2] / 100.0, worst / 100.0, c,
                         (unsigned)(keys[c] & 3), (unsigned long long)blks[c].bytes,
                         (unsigned long long)(blks[c].end - (keys[c] >> 2)), blks[c].nlanes, blks[c].status, us(w[1]),
                         // (emit: t_pass0 = its slowest lane's decode, rounds / exts / walks = that lane's symbols,
                         // decodes past the root table, refills from L2)
                         k ? (w[2] >> 32) / 100.0 : us(w[2]), us(w[3]), (unsigned long long)(k ? (w[2] >> 16) & 0xffff : w[5]),
                         k ? -1.0 : us(w[6]), (unsigned long long)(k ? (w[2] >> 8) & 0xff : w[7] & 0xffffffffu),
                         (unsigned long long)(k ? w[2] & 0xff : w[7] >> 32));
        }
    }
    if (a.prof) {   // k_pinf_find: the slowest workgroup's phases
        std::vector<uint64_t> pr(8ull * kPinfMaxCand);
        RDX_HIP(hipMemcpy(pr.data(), a.prof + 16ull * kPinfMaxCand, pr.size() * 8, hipMemcpyDeviceToHost));
        uint64_t lo = ~0ull, hi = 0, worst = 0, surv = 0;
        uint32_t wi = 0, n = 0;
        for (uint32_t i = 0; i < kPinfMaxCand; ++i) {
            const uint64_t *w = &pr[8ull * i];
            if (!w[0]) continue;
            ++n;
            surv += w[4];
            lo = std::min(lo, w[0]);
            hi = std::max(hi, w[3]);
            if (w[3] - w[0] > worst) { worst = w[3] - w[0]; wi = i; }
        }
        const uint64_t *w = &pr[8ull * wi];
        auto us = [&](uint64_t x) { return x > w[0] ? (x - w[0]) / 100.0 : -1.0; };
        std::fprintf(stderr, "{\"pinf_prof\": \"find\", \"wgs\": %u, \"span_us\": %.1f, \"max_us\": %.1f, "
                     "\"survivors\": %llu, \"max_wg\": %u, \"t_staged\": %.1f, \"t_headers\": %.1f, "
                     "\"wg_survivors\": %llu, \"t_lanes_done\": %.1f, \"wg_opens\": %llu}\n", n, (hi - lo) / 100.0,
                     worst / 100.0, (unsigned long long)surv, wi, us(w[1]), us(w[2]), (unsigned long long)w[4], us(w[5]),
                     (unsigned long long)w[6]);
    }
    // the sources of an unusually large stream are not kept at their high-water size
    if (ws->psrc.cap > kPinfKeepSources) {
        RDX_HIP(hipFree(ws->psrc.p));
        ws->psrc.p = nullptr;
        ws->psrc.cap = 0;
    }
    if (!h.final_ok) {
        if (tuning().pinflate_prof)   // tuning / diagnosis: why the parallel path declined
            std::fprintf(stderr, "{\"pinf_declined\": {\"emit_err\": %u, \"n_chain\": %u, \"total\": %llu, "
                         "\"n_cand\": %u, \"n_match\": %u}}\n", h.emit_err, h.n_chain, (unsigned long long)total,
                         h.n_cand, h.n_match);
        return kNotDecoded;
    }
    *raw_len = total;
    return RDX_OK;
}

// compression::decompress (compression.rs:18-27) of n device-resident streams into d_out (stream i at
// d_out + i*cap), asynchronous on s.
// blosc2: `may_zlib` false when the caller has read every chunk's header on the host and none is
// zlib- or zstd-coded: no stream table, no k_inflate / k_blosc2_zstd / zcheck launches.
constexpr uint64_t kZTableMaxRows = 1ull << 20;   // 48 B per row: <= 48 MiB of HBM

rdx_status decompress_launch(rdx_workspace *ws, uint32_t compression, uint64_t n, const uint8_t *const *h_ptrs,
                             const uint64_t *h_lens, uint8_t *d_out, uint64_t cap, uint64_t *d_out_len,
                             uint32_t *d_err, hipStream_t s, bool may_zlib = true) {
    rdx_status st;
    if ((st = ensure(ws, ws->zptrs, n, s))) return st;
    if ((st = ensure(ws, ws->zlens, n, s))) return st;
    if ((st = upload(ws, (void *)ws->zptrs.p, h_ptrs, n * sizeof(void *), ws->last_zptrs, s))) return st;
    if ((st = upload(ws, ws->zlens.p, h_lens, n * sizeof(uint64_t), ws->last_zlens, s))) return st;
    if (compression == RDX_COMPRESSION_BLOSC2) {
        uint64_t scratch_bytes = 0;
        if (n > 0xffffffffull || __builtin_mul_overflow(n, cap, &scratch_bytes)) return RDX_E_INVALID_ARGUMENT;
        if ((st = ensure(ws, ws->zscratch, scratch_bytes, s))) return st;
        RDX_HIP(hipMemsetAsync(d_err, 0, n * sizeof(uint32_t), s));
        KBlosc2Args a{};
        a.in = ws->zptrs.p;
        a.in_len = ws->zlens.p;
        a.out = d_out;
        a.scratch = ws->zscratch.p;
        a.cap = cap;
        a.out_len = d_out_len;
        a.err = d_err;
        a.n = (uint32_t)n;
        // waves per chunk: enough for one chunk's streams to fill the chip (4 waves per workgroup)
        a.wg_per_chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(128, 1024 / n));
        if (!may_zlib) {
            RDX_HIP(launch_blosc2(a, false, s));
            RDX_HIP(launch_blosc2_zcheck(a, s));   // (filters only: the table is absent)
            return RDX_OK;
        }
        // zlib-coded streams go through k_inflate, whose grid covers the table: 512 rows per chunk of the
        // batch, at least 8192 and at most kZTableMaxRows in all, handed out in arrival order across the
        // batch; a stream that finds the table full fails its chunk with RDX_BLOSC2_UNSUPPORTED (the host
        // decompresses that chunk)
        // (zstd-coded streams: the second half of the table, the same bound per codec, decoded by
        // k_blosc2_zstd)
        const uint64_t zcap = std::min<uint64_t>(kZTableMaxRows, std::max<uint64_t>(8192, n * 512));
        const uint64_t rows = 2 * zcap;
        if ((st = ensure(ws, ws->zt_in, rows, s)) || (st = ensure(ws, ws->zt_len, rows, s)) ||
            (st = ensure(ws, ws->zt_cap, rows, s)) || (st = ensure(ws, ws->zt_out_len, rows, s)) ||
            (st = ensure(ws, ws->zt_out, rows, s)) || (st = ensure(ws, ws->zt_chunk, rows, s)) ||
            (st = ensure(ws, ws->zt_err, rows, s)) || (st = ensure(ws, ws->zt_count, 2, s)))
            return st;
        RDX_HIP(hipMemsetAsync(ws->zt_count.p, 0, 2 * sizeof(uint32_t), s));
        a.z_in = ws->zt_in.p;
        a.z_len = ws->zt_len.p;
        a.z_out = ws->zt_out.p;
        a.z_cap = ws->zt_cap.p;
        a.z_chunk = ws->zt_chunk.p;
        a.z_out_len = ws->zt_out_len.p;
        a.z_err = ws->zt_err.p;
        a.z_count = ws->zt_count.p;
        a.z_capacity = zcap;
        RDX_HIP(launch_blosc2(a, false, s));
        RDX_HIP(launch_inflate_table(ws->zt_in.p, ws->zt_len.p, ws->zt_out.p, ws->zt_cap.p, ws->zt_count.p, zcap,
                                     ws->zt_out_len.p, ws->zt_err.p, s));
        RDX_HIP(launch_blosc2_zstd(a, s));
        RDX_HIP(launch_blosc2_zcheck(a, s));
        return RDX_OK;
    }
    RDX_HIP(launch_inflate(compression, ws->zptrs.p, ws->zlens.p, n, d_out, cap, d_out_len, d_err, s));
    return RDX_OK;
}

// A compressed request's chunk -> ws->raw (its decompressed bytes), synchronously: the operation's
// plan depends on the decompressed length.  The capacity starts at the size the request implies
// (shape x dtype size, else the gzip ISIZE hint, else 4x the compressed length) and grows on
// RDX_INFLATE_OUTPUT_OVERFLOW, so a stream longer than the shape implies still decodes to its end and
// meets validate_raw_size (app.rs:169-172) exactly like the reference.
rdx_status decompress_request(rdx_workspace *ws, const rdx_request &req, const uint8_t *d_src, uint64_t len,
                              uint64_t size_hint, hipStream_t s, uint64_t *raw_len, const uint8_t *h_src = nullptr,
                              bool any_size = false) {
    g_inflate_error = RDX_INFLATE_OK;
    const bool blosc2 = req.compression == RDX_COMPRESSION_BLOSC2;
    if (req.compression != RDX_COMPRESSION_GZIP && req.compression != RDX_COMPRESSION_ZLIB && !blosc2)
        return RDX_E_INVALID_ARGUMENT;
    uint64_t cap = size_hint;
    if (req.ndim && req.shape && req.dtype <= RDX_DTYPE_FLOAT64) {
        uint64_t e = (req.dtype == RDX_DTYPE_INT32 || req.dtype == RDX_DTYPE_UINT32 || req.dtype == RDX_DTYPE_FLOAT32) ? 4 : 8;
        bool ovf = false;
        for (uint32_t k = 0; k < req.ndim; ++k) ovf |= __builtin_mul_overflow(e, req.shape[k], &e);
        if (!ovf) cap = e;
    }
    if (blosc2 && size_hint) cap = size_hint;   // the header's nbytes (read on the host)
    if (cap == 0) cap = 4 * len + 4096;
    rdx_status st;
    g_inflate_path = RDX_INFLATE_PATH_SERIAL;
    if (!blosc2 && tuning().pinflate && (any_size || len >= (uint64_t)std::max(0, tuning().pinflate_min))) {
        // a lone stream: the whole device decodes it; anything it does not accept goes to k_inflate below
        st = pinflate_stream(ws, req.compression, d_src, len, s, raw_len);
        if (st == RDX_OK) {
            g_inflate_path = RDX_INFLATE_PATH_PARALLEL;
            return RDX_OK;
        }
        if (st != kNotDecoded) return st;
        // declined (an error anywhere, a chain it cannot follow, memory): the sequential k_inflate takes
        // 100-220 ms per 4 MiB where one host core's zlib takes 3.5-10 ms, so unless the context asks for the
        // device's own answer (inflate_fallback) a stream past a few KiB goes back to the caller, whose
        // host decoder gives the reference's bytes or error (integration/app_gpu.rs)
        if (!ws->inflate_fallback && len > (uint64_t)std::max(0, tuning().inflate_serial_max)) {
            g_inflate_path = RDX_INFLATE_PATH_DECLINED;
            return unsupported(RDX_UNSUPPORTED_INFLATE_DECLINED);
        }
        g_inflate_path = RDX_INFLATE_PATH_PARALLEL_FALLBACK;
    }
    if ((st = ensure(ws, ws->zout_len, 1, s))) return st;
    if ((st = ensure(ws, ws->zerr, 1, s))) return st;
    if (!ws->zback) RDX_HIP(hipHostMalloc((void **)&ws->zback, 2 * sizeof(uint64_t), hipHostMallocDefault));
    for (;;) {
        cap = (std::max<uint64_t>(cap, 16) + 15) / 16 * 16;
        if ((st = ensure(ws, ws->raw, cap, s))) return st;
        const uint8_t *ptrs[1] = {d_src};
        const uint64_t lens[1] = {len};
        // a blosc2 chunk in host memory: its header says whether any stream can be zlib- or zstd-coded
        // (codec 3 / 4: the stream table)
        const bool may_zlib = !(blosc2 && h_src && len >= 16 && (h_src[2] >> 5) != 3 && (h_src[2] >> 5) != 4);
        if ((st = decompress_launch(ws, req.compression, 1, ptrs, lens, ws->raw.p, cap, ws->zout_len.p, ws->zerr.p, s,
                                    may_zlib)))
            return st;
        RDX_HIP(hipMemcpyAsync(&ws->zback[0], ws->zout_len.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        RDX_HIP(hipMemcpyAsync(&ws->zback[1], ws->zerr.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        RDX_HIP(hipStreamSynchronize(s));
        const uint32_t e = (uint32_t)ws->zback[1];
        if (e == RDX_INFLATE_OUTPUT_OVERFLOW) {
            if (cap >= (1ull << 40)) return RDX_E_OUT_OF_MEMORY;
            // a blosc2 header states its size (k_blosc2 reports it with the overflow)
            cap = blosc2 && ws->zback[0] > cap ? ws->zback[0] : cap * 4;
            continue;
        }
        if (e != RDX_INFLATE_OK) {
            g_inflate_error = e;
            return e == RDX_BLOSC2_UNSUPPORTED ? unsupported(RDX_UNSUPPORTED_BLOSC2_CODEC) : RDX_E_DECOMPRESSION;
        }
        *raw_len = ws->zback[0];
        return RDX_OK;
    }
}

rdx_status create_workspace(int device, rdx_workspace **out, bool inflate_fallback) {
    RDX_HIP(hipSetDevice(device));
    auto *ws = new (std::nothrow) rdx_workspace();
    if (!ws) return RDX_E_OUT_OF_MEMORY;
    ws->device = device;
    ws->inflate_fallback = inflate_fallback;
#if RDX_PROBES
    if (tuning().epoch_start > 0) ws->epoch = (uint32_t)std::min(tuning().epoch_start, 0xffff);
#endif
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ws->cus = prop.multiProcessorCount;
    hipError_t e = hipStreamCreateWithFlags(&ws->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ws->upload_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ws->copy_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ws->done_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        delete ws;
        return map_err(e);
    }
    *out = ws;
    return RDX_OK;
}

void destroy_workspace(rdx_workspace *ws) {
    if (!ws) return;
    (void)hipSetDevice(ws->device);
    if (ws->own_stream) (void)hipStreamSynchronize(ws->own_stream);
    if (ws->upload_pending) (void)hipEventSynchronize(ws->upload_done);
    auto fr = [](void *p) { if (p) (void)hipFree(p); };
    fr(ws->partials.p);
    fr(ws->tickets.p);
    fr(ws->scratch[0].p);
    fr(ws->scratch[1].p);
    fr(ws->miss_list.p);
    fr((void *)ws->ptrs.p);
    fr(ws->chunk.p);
    fr(ws->body.p);
    fr(ws->counts.p);
    fr(ws->status.p);
    fr((void *)ws->zptrs.p);
    fr(ws->zlens.p);
    fr(ws->zout_len.p);
    fr(ws->zerr.p);
    fr(ws->raw.p);
    fr(ws->zscratch.p);
    fr((void *)ws->zt_in.p);
    fr(ws->zt_len.p);
    fr(ws->zt_cap.p);
    fr(ws->zt_out_len.p);
    fr((void *)ws->zt_out.p);
    fr(ws->zt_chunk.p);
    fr(ws->zt_err.p);
    fr(ws->zt_count.p);
    fr(ws->cbor.p);
    fr(ws->cbor_len.p);
    if (ws->aux_stream) {
        (void)hipStreamSynchronize(ws->aux_stream);
        (void)hipStreamDestroy(ws->aux_stream);
    }
    for (hipEvent_t e : ws->piece_ev)
        if (e) (void)hipEventDestroy(e);
    if (ws->zback) (void)hipHostFree(ws->zback);
    if (ws->h_back) (void)hipHostFree(ws->h_back);
    if (ws->h_slot) (void)hipHostFree(ws->h_slot);
    if (ws->pinf_back) (void)hipHostFree(ws->pinf_back);
    if (ws->pinf_slot) (void)hipHostFree(ws->pinf_slot);
    fr(ws->pinf.p);
    fr(ws->psrc.p);
    fr(ws->pprof.p);
    fr(ws->cbor_rec.p);
    fr(ws->cbor_stage.p);
    if (ws->pinned) (void)hipHostFree(ws->pinned);
    if (ws->upload_done) (void)hipEventDestroy(ws->upload_done);
    if (ws->copy_ev) (void)hipEventDestroy(ws->copy_ev);
    for (hipEvent_t e : ws->ph_ev)
        if (e) (void)hipEventDestroy(e);
    if (ws->done_ev) (void)hipEventDestroy(ws->done_ev);
    if (ws->own_stream) (void)hipStreamDestroy(ws->own_stream);
    delete ws;
}

bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// The staged CBOR scratch (~9 B per count) is not kept at its high-water size above this: a workspace that
// once encoded a very large count array would otherwise hold it (per workspace, per entry) and starve later,
// unrelated requests of HBM.
constexpr uint64_t kCborKeepStage = 512ull << 20;
rdx_status trim_cbor_stage(rdx_workspace *ws, hipStream_t s, uint64_t keep = kCborKeepStage) {
    if (ws->cbor_stage.cap <= keep) return RDX_OK;
    RDX_HIP(hipStreamSynchronize(s));   // in-flight k_cbor_place may still read it
    RDX_HIP(hipFree(ws->cbor_stage.p));
    ws->cbor_stage.p = nullptr;
    ws->cbor_stage.cap = 0;
    return RDX_OK;
}

// Response serialisation on the device (rdx_cbor_encode_device, k_cbor.hip), asynchronous on `s`.
rdx_status cbor_device(rdx_workspace *ws, const rdx_response_info *info, const void *d_body, const int64_t *d_counts,
                       uint32_t flags, void *d_out, uint64_t out_cap, uint64_t *d_out_len, uint32_t *d_status,
                       hipStream_t s) {
    if (!ws || !info || !d_out || !d_out_len) return RDX_E_INVALID_ARGUMENT;
    CborLayout L;
    if (rdx_status st = cbor_layout(*info, flags, L)) return st;
    if ((L.body_len && !d_body) || (L.n_counts && !d_counts)) return RDX_E_INVALID_ARGUMENT;
    if (out_cap < L.fixed() + (L.count_array ? 9 * L.n_counts : 0)) return RDX_E_BUFFER_TOO_SMALL;
    if (L.a.size() + L.b.size() > (size_t)kCborFixedMax || L.d.size() + L.f.size() > (size_t)kCborTailMax)
        return unsupported(RDX_UNSUPPORTED_RANK);   // cannot happen: ndim <= RDX_MAX_NDIM bounds both
    KCbor m{};
    uint8_t *out = static_cast<uint8_t *>(d_out);
    m.out = out;
    m.counts = d_counts;
    m.n = L.count_array ? L.n_counts : 0;
    const uint64_t tiles = (m.n + 2047) / 2048;   // k_cbor.hip kCborTile
    if (tiles > 0xffffffffull) return unsupported(RDX_UNSUPPORTED_CBOR_SIZE);
    m.n_tiles = (uint32_t)tiles;
    m.c_off = L.c_off();
    m.b_off = L.b_off();
    m.raw_len = L.count_raw ? 8 * L.n_counts : 0;
    m.out_len = d_out_len;
    m.vec = (reinterpret_cast<uintptr_t>(d_counts) % 16) == 0;
    m.a_len = (uint32_t)L.a.size();
    m.b_len = (uint32_t)L.b.size();
    m.d_len = (uint32_t)L.d.size();
    m.f_len = (uint32_t)L.f.size();
    std::memcpy(m.fixed, L.a.data(), L.a.size());
    std::memcpy(m.fixed + L.a.size(), L.b.data(), L.b.size());
    std::memcpy(m.tail, L.d.data(), L.d.size());
    std::memcpy(m.tail + L.d.size(), L.f.data(), L.f.size());
    // the body / count_as_bytes payload copies ride in the same launch when 16-byte loads and
    // dword-aligned 16-byte stores fit them (large bodies: the body head makes segment A 12 bytes)
    const auto al = [](const void *p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; };
    m.body = static_cast<const uint8_t *>(d_body);
    m.body_len = L.body_len;
    m.copy_body = L.body_len && al(d_body, 16) && al(out + L.body_off(), 4);
    m.copy_raw = L.count_raw && al(d_counts, 16) && al(out + m.c_off + L.d.size(), 4);
    const uint64_t copy_bytes = (m.copy_body ? L.body_len : 0) + (m.copy_raw ? m.raw_len : 0);
    const uint64_t copy_blocks = std::min<uint64_t>((copy_bytes + 65535) / 65536, (uint64_t)ws->cus * 8);
    // one encoding workgroup per tile; the copies share the grid.  (Resident workgroups looping over the
    // tiles with the next one prefetched: 142 vs 136 us for 32 Mi counts, profiles/r04_cbor_variants.jsonl)
    const uint32_t blocks = (uint32_t)std::max<uint64_t>({1, tiles, copy_blocks});
    rdx_status st;
    // the staged form (k_cbor_pack / k_cbor_place: the counts read once) unless RDX_CBOR_STAGED=0 or its
    // scratch (18 KiB per tile of 2048 counts) cannot be had
    m.staged = m.n_tiles && tuning().cbor_staged ? 1u : 0u;
    if (m.staged) {
        // tile lengths as tagged granules in the hand-off records, the sharded arrival counters
        m.tpg = cbor_pack_tpg(m.n_tiles);
        const uint64_t need = cbor_stage_bytes(m.n_tiles);
        if (need <= kCborKeepStage && (st = trim_cbor_stage(ws, s))) return st;   // an earlier huge one
        if (!m.tpg || ensure(ws, ws->cbor_stage, need, s) || ensure(ws, ws->partials, 2048, s, true) ||
            ensure(ws, ws->tickets, kTicketWords, s, true)) {
            (void)hipGetLastError();
            m.staged = 0;
        } else {
            m.stage = ws->cbor_stage.p;
            m.tagged = ws->partials.p;
            m.arrive = ws->tickets.p;
            m.status = d_status;
            if ((st = next_epoch(ws, s, m.epoch))) return st;
        }
    }
    if (m.n_tiles) {
        // (not the tagged hand-off records; the staged form: + 1 total + the group offsets)
        if ((st = ensure(ws, ws->cbor_rec, m.n_tiles + 1 + (m.staged ? 2048 : 0), s))) return st;
        m.records = ws->cbor_rec.p;
    }
    if (d_status) RDX_HIP(hipMemsetAsync(d_status, 0, sizeof(uint32_t), s));
    if (L.body_len && !m.copy_body)
        RDX_HIP(hipMemcpyAsync(out + L.body_off(), d_body, L.body_len, hipMemcpyDeviceToDevice, s));
    if (L.count_raw && !m.copy_raw)   // c.to_ne_bytes() of every count (models.rs:383-385), after segment D
        RDX_HIP(hipMemcpyAsync(out + m.c_off + L.d.size(), d_counts, m.raw_len, hipMemcpyDeviceToDevice, s));
    RDX_HIP(launch_cbor(m, blocks, s));
    return RDX_OK;
}

// ---- host-resident execution (rdx_execute / rdx_execute_owned) --------------------------------------
// Page-locked response buffers for rdx_execute_owned, pooled per context: pinning a buffer per request
// costs more than the request (hipHostMalloc of 128 MiB: milliseconds), so freed blocks are kept by size
// class (powers of two from 4 KiB) up to kPoolCap bytes per context.
constexpr uint64_t kPoolCap = 2ull << 30;

uint64_t pool_class(uint64_t bytes) {
    uint64_t c = 4096;
    while (c < bytes) c <<= 1;
    return c;
}

rdx_status pool_alloc(rdx_context *ctx, uint64_t bytes, void **out) {
    const uint64_t c = pool_class(std::max<uint64_t>(bytes, 1));
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        auto it = ctx->pinned_free.find(c);
        if (it != ctx->pinned_free.end() && !it->second.empty()) {
            *out = it->second.back();
            it->second.pop_back();
            ctx->pinned_cached -= c;
            ctx->pinned_class[*out] = c;
            return RDX_OK;
        }
    }
    RDX_HIP(hipSetDevice(ctx->devices[0]));
    RDX_HIP(hipHostMalloc(out, c, hipHostMallocPortable));
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->pinned_class[*out] = c;
    return RDX_OK;
}

void pool_free(rdx_context *ctx, void *p) {
    std::unique_lock<std::mutex> g(ctx->mu);
    auto it = ctx->pinned_class.find(p);
    if (it == ctx->pinned_class.end()) return;
    const uint64_t c = it->second;
    ctx->pinned_class.erase(it);
    if (ctx->pinned_cached + c <= kPoolCap) {
        ctx->pinned_free[c].push_back(p);
        ctx->pinned_cached += c;
        return;
    }
    g.unlock();
    (void)hipHostFree(p);
}

bool is_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();   // a pageable pointer is not an error for the caller
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// The device address of a page-locked host range (hipHostMalloc / rdx_host_alloc / hipHostRegister), or
// null for pageable memory.
const uint8_t *host_alias(const void *p) {
    if (!p) return nullptr;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost) return nullptr;
    return static_cast<const uint8_t *>(a.devicePointer ? a.devicePointer : p);
}

// RDX_PHASES=1: where a direct request's time goes (the idle-entry path a lone host request takes),
// summed over requests and printed as one JSON line per path when the context is destroyed.
struct PhaseSums {
    std::mutex mu;
    uint64_t n[3] = {};
    double sum[3][8] = {};   // [path][phase]: see print_phases
};
PhaseSums &phase_sums() {
    static PhaseSums p;
    return p;
}
void phase_add(int path, const double *v) {
    PhaseSums &P = phase_sums();
    std::lock_guard<std::mutex> g(P.mu);
    for (int k = 0; k < 8; ++k) P.sum[path][k] += v[k];
    ++P.n[path];
}
void print_phases() {
    PhaseSums &p = phase_sums();
    std::lock_guard<std::mutex> g(p.mu);
    static const char *const paths[3] = {"host_read", "dma_copy", "coalesced_host"};
    static const char *const fields[3][8] = {
        {"plan_place_lease_us", "copy_issue_us", "launch_issue_us", "issue_to_result_seen_us", "result_to_return_us",
         "total_us", "device_copy_us", "device_kernel_us"},
        {"plan_place_lease_us", "copy_issue_us", "launch_issue_us", "issue_to_result_seen_us", "result_to_return_us",
         "total_us", "device_copy_us", "device_kernel_us"},
        {"plan_place_lease_us", "copy_issue_us", "queued_to_woken_us", "total_us", "plan_place_lease_cpu_us",
         "copy_issue_cpu_us", "queued_to_woken_cpu_us", "total_cpu_us"}};
    for (int k = 0; k < 3; ++k) {
        if (!p.n[k]) continue;
        const double n = (double)p.n[k];
        std::string line = std::string("{\"rdx_phases\": {\"path\": \"") + paths[k] + "\", \"requests\": " +
                           std::to_string(p.n[k]);
        for (int f = 0; f < 8; ++f) {
            char b[96];
            std::snprintf(b, sizeof b, ", \"%s\": %.2f", fields[k][f], p.sum[k][f] / n);
            line += b;
        }
        std::fprintf(stderr, "%s}}\n", line.c_str());
    }
}
double thread_cpu_us() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

// Select / axis=[] (Mode::Map) from page-locked host memory into page-locked host memory, pipelined:
// the output is cut along its outermost dim into pieces; piece k's input slab crosses PCIe on the
// workspace stream while piece k-1 is gathered and its output comes back on the aux stream, so the H2D
// of the chunk and the D2H of the response (the two directions of the link) overlap instead of adding up
// (C5: 256 MiB in + 128 MiB out).
constexpr int kMapPieces = 8;

rdx_status wait_event(rdx_context *ctx, PoolEntry &e, hipEvent_t ev, double budget_us);
constexpr uint64_t kBackStage = 64ull << 10;    // rdx_workspace::h_back: small responses staged page-locked

rdx_status map_pipelined(rdx_context *ctx, PoolEntry &entry, rdx_workspace *ws, const ExecPlan &p, const uint8_t *chunk,
                         uint64_t len, uint8_t *body, int64_t *counts) {
    const KView &v = p.map.view;
    const int outer = v.ndim - 1;
    const uint64_t N = v.count[outer], inner = v.n / N;
    const int64_t vs = v.vstride[outer];
    const uint64_t out_es = p.info.body_bytes / v.n;
    const int S = (int)std::min<uint64_t>(N, kMapPieces);
    hipStream_t sa = ws->own_stream, sb = ws->aux_stream;
    rdx_status st;
    if ((st = ensure(ws, ws->chunk, std::max<uint64_t>(len, 16), sa))) return st;
    if ((st = ensure(ws, ws->body, std::max<uint64_t>(p.info.body_bytes, 16), sa))) return st;
    if ((st = ensure(ws, ws->counts, std::max<uint64_t>(p.map.kind == 0 ? (uint64_t)S : p.info.n_counts, 1), sa)))
        return st;
    if ((st = ensure(ws, ws->status, (uint64_t)S, sa))) return st;
    RDX_HIP(hipStreamSynchronize(sa));   // allocations done before the aux stream uses them
    int64_t lo_in = 0, hi_in = 0;        // element extent of one outer index over the inner dims
    for (int k = 0; k < outer; ++k) {
        const int64_t span = (int64_t)(v.count[k] - 1) * v.vstride[k];
        (span < 0 ? lo_in : hi_in) += span;
    }
    const uint64_t esz = p.fused ? 1 : p.esz;
    for (int k = 0; k < S; ++k) {
        const uint64_t a = (uint64_t)k * N / S, b = (uint64_t)(k + 1) * N / S;
        const int64_t o0 = v.base_off + (int64_t)a * vs, o1 = v.base_off + (int64_t)(b - 1) * vs;
        const int64_t lo = std::min(o0, o1) + lo_in, hi = std::max(o0, o1) + hi_in;
        const uint64_t blo = (uint64_t)lo * esz, bhi = std::min<uint64_t>(len, (uint64_t)(hi + 1) * esz);
        if (bhi > blo) RDX_HIP(hipMemcpyAsync(ws->chunk.p + blo, chunk + blo, bhi - blo, hipMemcpyHostToDevice, sa));
        RDX_HIP(hipEventRecord(ws->piece_ev[k], sa));
        RDX_HIP(hipStreamWaitEvent(sb, ws->piece_ev[k], 0));
        ExecPlan pk = p;
        KView &w = pk.map.view;
        w.count[outer] = (uint32_t)(b - a);
        w.div[outer] = make_div((uint32_t)(b - a));
        w.base_off = o0;
        w.n = inner * (b - a);
        uint8_t *d_body = ws->body.p + a * inner * out_es;
        int64_t *d_counts = p.map.kind == 0 ? ws->counts.p + k : ws->counts.p + a * inner;
        if ((st = run_device(ws, pk, ws->chunk.p, nullptr, 1, len, d_body, d_counts, ws->status.p + k, sb))) return st;
        RDX_HIP(hipMemcpyAsync(body + a * inner * out_es, d_body, inner * (b - a) * out_es, hipMemcpyDeviceToHost, sb));
        if (p.map.kind != 0)
            RDX_HIP(hipMemcpyAsync(counts + a * inner, d_counts, inner * (b - a) * sizeof(int64_t), hipMemcpyDeviceToHost, sb));
    }
    // the pieces' counts and statuses through the page-locked readback block (a copy into the stack would
    // be a synchronous, spinning one), then the caller sleeps through the transfers (wait_event)
    if (!ws->h_back) RDX_HIP(hipHostMalloc((void **)&ws->h_back, 16 + kBackStage, hipHostMallocDefault));
    int64_t *const piece_counts = reinterpret_cast<int64_t *>(ws->h_back + 2);
    uint32_t *const piece_status = reinterpret_cast<uint32_t *>(ws->h_back + 2 + kMapPieces);
    if (p.map.kind == 0) RDX_HIP(hipMemcpyAsync(piece_counts, ws->counts.p, S * sizeof(int64_t), hipMemcpyDeviceToHost, sb));
    RDX_HIP(hipMemcpyAsync(piece_status, ws->status.p, S * sizeof(uint32_t), hipMemcpyDeviceToHost, sb));
    RDX_HIP(hipEventRecord(ws->done_ev, sb));
    if ((st = wait_event(ctx, entry, ws->done_ev, 20.0))) return st;
    uint32_t any = 0;
    for (int k = 0; k < S; ++k) any |= piece_status[k];
    if (any) return (rdx_status)any;
    if (p.map.kind == 0) {
        int64_t c = 0;
        for (int k = 0; k < S; ++k) c += piece_counts[k];
        counts[0] = c;
    }
    return RDX_OK;
}

}  // namespace

// ====================================== C ABI ========================================================
extern "C" {

uint32_t rdx_abi_version(void) { return RDX_ABI_VERSION; }

const char *rdx_status_string(rdx_status s) {
    switch (s) {
        case RDX_OK: return "ok";
        case RDX_E_INVALID_ARGUMENT: return "invalid argument";
        case RDX_E_REQUEST_VALIDATION: return "request data is not valid";
        case RDX_E_FROM_BYTES: return "failed to convert from bytes";
        case RDX_E_SHAPE_INVALID: return "failed to create array from shape";
        case RDX_E_INCOMPATIBLE_MISSING: return "Incompatible value for missing";
        case RDX_E_SHUFFLE_LENGTH: return "data length is not a multiple of the shuffle element size";
        case RDX_E_NAN_UNORDERED: return "unexpected undefined order error for min";
        case RDX_E_UNSUPPORTED: return "unsupported by the device engine";
        case RDX_E_DEVICE: return "device error";
        case RDX_E_OUT_OF_MEMORY: return "out of memory";
        case RDX_E_BUFFER_TOO_SMALL: return "output buffer too small";
        case RDX_E_NO_DEVICE: return "no gfx950 device";
        case RDX_E_DECOMPRESSION: return "decompression failed";
    }
    return "unknown status";
}

const char *rdx_inflate_error_string(uint32_t code) {
    switch (code) {
        case RDX_INFLATE_OK: return "ok";
        case RDX_INFLATE_GZIP_HEADER: return "invalid gzip header";                  // compression.rs:173
        case RDX_INFLATE_ZLIB_METHOD: return "Unknown zlib compression method";      // compression.rs:185 (+ " N")
        case RDX_INFLATE_ZLIB_HEADER: return "invalid zlib header";
        case RDX_INFLATE_TRUNCATED: return "unexpected end of compressed data";
        case RDX_INFLATE_BLOCK_TYPE: return "invalid deflate block type";
        case RDX_INFLATE_STORED_LENGTH: return "invalid stored block lengths";
        case RDX_INFLATE_CODE_LENGTHS: return "invalid deflate code lengths";
        case RDX_INFLATE_BAD_SYMBOL: return "invalid deflate code";
        case RDX_INFLATE_DISTANCE: return "invalid distance too far back";
        case RDX_INFLATE_CHECKSUM: return "checksum mismatch";
        case RDX_INFLATE_OUTPUT_OVERFLOW: return "decompressed data larger than the output buffer";
        case RDX_BLOSC2_INVALID: return "invalid blosc2 compressed data";                  // compression.rs:37
        case RDX_BLOSC2_FAILED: return "failed to decompress blosc2 data";                 // compression.rs:47
        case RDX_BLOSC2_SIZE: return "unexpected decompressed size for blosc2 data";       // compression.rs:52
        case RDX_BLOSC2_UNSUPPORTED: return "blosc2 codec or filter not supported by the device engine";
    }
    return "unknown decompression error";
}

uint32_t rdx_inflate_last_error(void) { return g_inflate_error; }

uint32_t rdx_inflate_last_path(void) { return g_inflate_path; }

uint32_t rdx_last_unsupported_reason(void) { return last_unsupported(); }

// blosc2_cbuffer_sizes (blusc 0.0.2 / c-blosc2 read_chunk_header on the first 16 bytes), as the
// reference calls it (compression.rs:33): all zeros when the header is not a valid blosc chunk.
rdx_status rdx_blosc2_cbuffer_sizes(const void *src, uint64_t len, uint64_t *nbytes, uint64_t *cbytes,
                                    uint64_t *blocksize) {
    if ((!src && len) || !nbytes || !cbytes || !blocksize) return RDX_E_INVALID_ARGUMENT;
    *nbytes = *cbytes = *blocksize = 0;
    if (len < 16) return RDX_OK;
    const uint8_t *h = static_cast<const uint8_t *>(src);
    auto rd = [&](int k) {
        return (int32_t)((uint32_t)h[k] | (uint32_t)h[k + 1] << 8 | (uint32_t)h[k + 2] << 16 | (uint32_t)h[k + 3] << 24);
    };
    const int32_t nb = rd(4), bs = rd(8), cb = rd(12);
    if (cb < 16 || h[0] == 0 || h[0] > 5 || bs <= 0 || (nb > 0 && bs > nb) || bs > 536866816 || h[3] == 0 || nb <= 0)
        return RDX_OK;
    *nbytes = (uint64_t)nb;
    *cbytes = (uint64_t)cb;
    *blocksize = (uint64_t)bs;
    return RDX_OK;
}

int rdx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int c = 0;
    for (int d = 0; d < n; ++d) c += is_gfx950(d) ? 1 : 0;
    return c;
}

rdx_status rdx_context_create(const int *devices, int n_devices, rdx_context **out) {
    if (!out) return RDX_E_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return RDX_E_NO_DEVICE;
    auto *ctx = new (std::nothrow) rdx_context();
    if (!ctx) return RDX_E_OUT_OF_MEMORY;
    if (!devices || n_devices <= 0) ctx->devices.push_back(0);
    else ctx->devices.assign(devices, devices + n_devices);
    for (int d : ctx->devices) {
        if (d < 0 || d >= n || !is_gfx950(d)) {
            delete ctx;
            return RDX_E_NO_DEVICE;
        }
    }
    ctx->cfg = effective_config(rdx_context_config{0, 1, 0, 0, 0, 0});
    for (int d : ctx->devices) {
        auto e = std::unique_ptr<PoolEntry>(new (std::nothrow) PoolEntry());
        if (!e) {
            delete ctx;
            return RDX_E_OUT_OF_MEMORY;
        }
        e->device = d;
        ctx->entries.push_back(std::move(e));
    }
    *out = ctx;
    return RDX_OK;
}

void rdx_context_destroy(rdx_context *ctx) {
    if (!ctx) return;
    for (auto &e : ctx->entries) {
        {
            std::lock_guard<std::mutex> g(e->mu);
            e->stop = true;
        }
        e->job_cv.notify_all();
        if (e->dispatcher.joinable()) e->dispatcher.join();   // returns once its queue and lanes are empty
        if (env_int("RDX_DISPATCH_STATS", 0) && e->n_launch)
            std::fprintf(stderr,
                         "{\"rdx_dispatch\": {\"device\": %d, \"launches\": %llu, \"requests\": %llu, "
                         "\"launch_host_us\": %.2f, \"issue_to_seen_done_us\": %.2f, \"complete_us\": %.2f}}\n",
                         e->device, (unsigned long long)e->n_launch, (unsigned long long)e->coalesced,
                         e->t_launch / e->n_launch, e->t_flight / std::max<uint64_t>(1, e->n_done),
                         e->t_complete / std::max<uint64_t>(1, e->n_done));
        for (rdx_workspace *ws : e->all_ws) destroy_workspace(ws);
        for (Lane *l : e->lanes) destroy_lane(l);
    }
    for (auto &kv : ctx->pinned_free)
        for (void *p : kv.second) (void)hipHostFree(p);
    if (tuning().phases) print_phases();
    delete ctx;
}

rdx_status rdx_validate_request(const rdx_request *req) {
    if (!req) return RDX_E_INVALID_ARGUMENT;
    return validate_request(*req);
}

rdx_status rdx_plan(const rdx_request *req, uint64_t chunk_len, rdx_response_info *info) {
    if (!req || !info) return RDX_E_INVALID_ARGUMENT;
    ExecPlan p;
    const rdx_status st = make_plan(*req, chunk_len, p);
    if (st) return st;
    *info = p.info;
    return RDX_OK;
}

// src/types/dvalue.rs:43-83 TryFromDValue, for a JSON integer that fits i64.
rdx_status rdx_missing_from_i64(uint32_t dtype, int64_t v, void *out) {
    if (!out) return RDX_E_INVALID_ARGUMENT;
    switch (dtype) {
        case RDX_DTYPE_INT32: {
            if (v < INT32_MIN || v > INT32_MAX) return RDX_E_INCOMPATIBLE_MISSING;
            const int32_t x = (int32_t)v; std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_INT64: std::memcpy(out, &v, 8); return RDX_OK;
        case RDX_DTYPE_UINT32: {
            if (v < 0 || v > (int64_t)UINT32_MAX) return RDX_E_INCOMPATIBLE_MISSING;
            const uint32_t x = (uint32_t)v; std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_UINT64: {
            if (v < 0) return RDX_E_INCOMPATIBLE_MISSING;
            const uint64_t x = (uint64_t)v; std::memcpy(out, &x, 8); return RDX_OK;
        }
        case RDX_DTYPE_FLOAT32: {
            const float x = (float)(double)v;
            if (!std::isfinite(x)) return RDX_E_INCOMPATIBLE_MISSING;
            std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_FLOAT64: { const double x = (double)v; std::memcpy(out, &x, 8); return RDX_OK; }
    }
    return RDX_E_INVALID_ARGUMENT;
}

// ... for a JSON integer above i64::MAX (serde_json PosInt that as_i64() rejects).
rdx_status rdx_missing_from_u64(uint32_t dtype, uint64_t v, void *out) {
    if (!out) return RDX_E_INVALID_ARGUMENT;
    if (v <= (uint64_t)INT64_MAX) return rdx_missing_from_i64(dtype, (int64_t)v, out);
    switch (dtype) {
        case RDX_DTYPE_INT32: case RDX_DTYPE_INT64: case RDX_DTYPE_UINT32: return RDX_E_INCOMPATIBLE_MISSING;
        case RDX_DTYPE_UINT64: std::memcpy(out, &v, 8); return RDX_OK;
        case RDX_DTYPE_FLOAT32: {
            const float x = (float)(double)v;
            if (!std::isfinite(x)) return RDX_E_INCOMPATIBLE_MISSING;
            std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_FLOAT64: { const double x = (double)v; std::memcpy(out, &x, 8); return RDX_OK; }
    }
    return RDX_E_INVALID_ARGUMENT;
}

// ... for a JSON float (as_i64/as_u64 are None: integers are incompatible).
rdx_status rdx_missing_from_f64(uint32_t dtype, double v, void *out) {
    if (!out) return RDX_E_INVALID_ARGUMENT;
    switch (dtype) {
        case RDX_DTYPE_INT32: case RDX_DTYPE_INT64: case RDX_DTYPE_UINT32: case RDX_DTYPE_UINT64:
            return RDX_E_INCOMPATIBLE_MISSING;
        case RDX_DTYPE_FLOAT32: {
            const float x = (float)v;
            if (!std::isfinite(x)) return RDX_E_INCOMPATIBLE_MISSING;
            std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_FLOAT64: std::memcpy(out, &v, 8); return RDX_OK;
    }
    return RDX_E_INVALID_ARGUMENT;
}

rdx_status rdx_host_alloc(rdx_context *ctx, uint64_t bytes, void **out) {
    if (!ctx || !out) return RDX_E_INVALID_ARGUMENT;
    RDX_HIP(hipSetDevice(ctx->devices[0]));
    RDX_HIP(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable));
    return RDX_OK;
}

void rdx_host_free(rdx_context *ctx, void *p) {
    (void)ctx;
    if (p) (void)hipHostFree(p);
}

rdx_status rdx_workspace_create(rdx_context *ctx, int device, rdx_workspace **out) {
    if (!ctx || !out) return RDX_E_INVALID_ARGUMENT;
    return create_workspace(device, out, ctx->cfg.inflate_fallback != 0);
}

void rdx_workspace_destroy(rdx_workspace *ws) { destroy_workspace(ws); }

rdx_status rdx_execute_device(rdx_workspace *ws, const rdx_request *req, const void *d_chunk, uint64_t chunk_len,
                              void *d_body, int64_t *d_counts, uint32_t *d_status, void *stream,
                              rdx_response_info *info) {
    if (!ws || !req) return RDX_E_INVALID_ARGUMENT;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t *src = static_cast<const uint8_t *>(d_chunk);
    rdx_status st;
    if (req->compression != RDX_COMPRESSION_NONE) {  // filter_pipeline.rs:23-25, then plan on the raw size
        if (!d_chunk && chunk_len) return RDX_E_INVALID_ARGUMENT;
        RDX_HIP(hipSetDevice(ws->device));
        uint64_t raw_len = 0;
        if ((st = decompress_request(ws, *req, src, chunk_len, 0, s, &raw_len))) return st;
        src = ws->raw.p;
        chunk_len = raw_len;
    }
    ExecPlan p;
    if ((st = make_plan(*req, chunk_len, p))) return st;
    if (info) *info = p.info;
    if ((!src && chunk_len) || (!d_body && p.info.body_bytes) || (!d_counts && p.info.n_counts))
        return RDX_E_INVALID_ARGUMENT;
    RDX_HIP(hipSetDevice(ws->device));
    return run_device(ws, p, src, nullptr, 1, chunk_len, static_cast<uint8_t *>(d_body), d_counts, d_status, s);
}

rdx_status rdx_execute_batch_device(rdx_workspace *ws, const rdx_request *req, uint64_t n_chunks,
                                    const void *const *h_chunk_ptrs, uint64_t chunk_len, void *d_bodies,
                                    int64_t *d_counts, uint32_t *d_status, void *stream, rdx_response_info *info) {
    if (!ws || !req || (n_chunks && !h_chunk_ptrs)) return RDX_E_INVALID_ARGUMENT;
    // compressed chunks have per-chunk lengths: rdx_decompress_batch_device first, then this on the raw
    // buffers
    if (req->compression != RDX_COMPRESSION_NONE) return RDX_E_INVALID_ARGUMENT;
    ExecPlan p;
    rdx_status st = make_plan(*req, chunk_len, p);
    if (st) return st;
    if (info) *info = p.info;
    if (n_chunks == 0) return RDX_OK;
    if ((!d_bodies && p.info.body_bytes) || (!d_counts && p.info.n_counts)) return RDX_E_INVALID_ARGUMENT;
    RDX_HIP(hipSetDevice(ws->device));
    return run_device(ws, p, nullptr, reinterpret_cast<const uint8_t *const *>(h_chunk_ptrs), n_chunks, chunk_len,
                      static_cast<uint8_t *>(d_bodies), d_counts, d_status, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace {

bool fits_i32(int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; }

// A planned all-axes request as a k_multi descriptor; false when it runs as its own launch instead.
// Byte-shuffled chunks (fused unshuffle) stay out: the plane-transposing k_all_contig serves them far
// better than per-element byte gathers, and k_multi's register budget (its heaviest body sets every
// workgroup's occupancy) stays that of plain loads.
bool multi_req(const ExecPlan &p, const rdx_multi_item &it, KMultiReq &q) {
    if (p.fused || !p.unfused_es.empty() || !p.miss_list.empty()) return false;
    KView v{};
    uint32_t filt = 0;
    if (p.mode == Mode::AllStrided && p.all_strided.view.ndim <= kMultiDims && p.all_strided.view.ndim >= 1) {
        v = p.all_strided.view;
        filt = p.all_strided.filter_semantics;
    } else if (p.mode == Mode::AllContig && p.all_contig.n > 0 && p.all_contig.n < (1ull << 32)) {
        const KAllContig &c = p.all_contig;
        v.ndim = 1;
        v.base_off = (int64_t)c.off;
        v.r0 = c.r0;
        v.n = c.n;
        v.count[0] = (uint32_t)c.n;
        v.vstride[0] = 1;
        v.rstride[0] = c.rs;
        filt = c.filter_semantics;
    } else {
        return false;
    }
    if (v.n == 0 || v.n >= (1ull << 31)) return false;   // k_multi's 32-bit index arithmetic
    const KMissing &m = p.miss;
    if (m.kind == RDX_MISSING_VALUES && m.n > 2) return false;   // longer lists: k_all_strided's list scan
    q = KMultiReq{};
    for (int k = 0; k < kMultiDims; ++k) {
        const bool real = k < v.ndim;
        if (real && (!fits_i32(v.vstride[k]) || !fits_i32(v.rstride[k]))) return false;
        q.vstride[k] = real ? (int32_t)v.vstride[k] : 0;
        q.rstride[k] = real ? (int32_t)v.rstride[k] : 0;
        if (k < kMultiDims - 1) {
            q.count[k] = real ? v.count[k] : 1u;
            q.magic[k] = make_div(q.count[k]).magic;
        }
    }
    q.base = static_cast<const uint8_t *>(it.d_chunk);
    q.body = static_cast<uint8_t *>(it.d_body);
    q.counts = it.d_counts;
    q.status = it.d_status;
    q.base_off = v.base_off;
    q.r0 = v.r0;
    q.n = (uint32_t)v.n;
    q.dtype = (uint8_t)p.dtype;
    q.op = (uint8_t)p.op;
    q.ndim = (uint8_t)v.ndim;
    q.vec = (uint8_t)vec_width(v, p.esz, q.base, nullptr, 1, false);
    uint8_t f = p.bswap ? kMultiBswap : 0;
    if (filt) f |= kMultiFilt;
    switch (m.kind) {
        case RDX_MISSING_VALUE: f |= kMultiEq0; q.v0 = m.v0; break;
        case RDX_MISSING_VALUES:
            if (m.n >= 1) { f |= kMultiEq0; q.v0 = m.inl[0]; }
            if (m.n >= 2) { f |= kMultiEq1; q.v1 = m.inl[1]; }
            break;
        case RDX_MISSING_VALID_MIN: f |= kMultiLo; q.v0 = m.v0; break;
        case RDX_MISSING_VALID_MAX: f |= kMultiHi; q.v1 = m.v0; break;
        case RDX_MISSING_VALID_RANGE: f |= kMultiLo | kMultiHi; q.v0 = m.v0; q.v1 = m.v1; break;
        default: break;
    }
    q.flags = f;
    // workgroups for one load round trip per lane (scaled down when the launch overfills the chip)
    const uint64_t per_block = (uint64_t)kBlock * (q.vec > 1 ? 4 : 8);
    q.bpc = (uint32_t)std::max<uint64_t>(1, (v.n / q.vec + per_block - 1) / per_block);
    return true;
}

// One k_multi launch over reqs[0..n): one residency round of the chip (5 workgroups per CU) serves the
// whole launch; a launch that wants more gets proportionally fewer, longer-running workgroups per request
// (each lane keeps 4-8 loads in flight per step), so no request pays several dispatch + hand-off rounds.
rdx_status launch_multi_group(rdx_workspace *ws, const KMultiReq *reqs, uint32_t n, hipStream_t s,
                              uint32_t flags = 0) {
    KMultiArgs args;
    args.n_items = n;
    args.flags = flags | (tuning().fold_last ? kMultiFoldLast : 0u) |   // <= 24 folders: always fold-last
                 (fold_mode() == 2 ? kMultiAtomicFold : 0u);
    args.pad = 0;
    const uint64_t target = (uint64_t)ws->cus * tuning().multi_blocks_per_cu;
    uint64_t want = 0;
    for (uint32_t k = 0; k < n; ++k) want += std::min<uint64_t>(reqs[k].bpc, (uint64_t)ws->cus * 8);
    const double scale = want > target ? (double)target / (double)want : 1.0;
    uint64_t blocks = 0;
    for (uint32_t k = 0; k < n; ++k) {
        KMultiReq &q = args.req[k];
        q = reqs[k];
        q.bpc = (uint32_t)std::max<double>(1.0, std::ceil(std::min<uint64_t>(q.bpc, (uint64_t)ws->cus * 8) * scale));
        q.block0 = (uint32_t)blocks;
        blocks += q.bpc;
    }
    rdx_status st;
    if ((st = ensure(ws, ws->partials, blocks * kRecordU64, s, true))) return st;
    if ((st = ensure(ws, ws->tickets, (uint64_t)n * kTicketWords, s, true))) return st;
    if ((st = next_epoch(ws, s, args.epoch))) return st;
    args.partials = ws->partials.p;
    args.tickets = ws->tickets.p;
    RDX_HIP(launch_multi(args, (uint32_t)blocks, s));
    return RDX_OK;
}

}  // namespace

namespace {

// ---- the device pool: placement, workspaces with back-pressure, request coalescing ---------------------
// The server runs every request as its own synchronous operation<T>() call on a worker thread
// (app.rs:147-152, app_state.rs:21-37); the pool turns those concurrent calls into few, full launches.

rdx_context_config effective_config(const rdx_context_config &c) {
    rdx_context_config e = c;
    if (!e.max_workspaces) e.max_workspaces = 16;
    if (!e.coalesce_lanes) e.coalesce_lanes = 3;
    if (e.coalesce_lanes > 16) e.coalesce_lanes = 16;
    if (!e.coalesce_max_bytes) e.coalesce_max_bytes = 64ull << 20;
    if (!e.coalesce_host_max_bytes) e.coalesce_host_max_bytes = 1ull << 20;
    return e;
}

// A request's claim on a pool entry: its weight counts as in flight there until the request returns.
struct Placement {
    PoolEntry *e = nullptr;
    uint64_t weight = 0;
    Placement() = default;
    Placement(const Placement &) = delete;
    ~Placement() {
        if (e) e->outstanding.fetch_sub(weight, std::memory_order_relaxed);
    }
};

// Least outstanding bytes: the entry, among those on `device` (-1: any), with the fewest
// chunk bytes in flight; the scan starts at a rotating index so that ties spread over the pool.  A
// request weighs its chunk bytes plus 64 KiB (its fixed cost: launch, hand-off, round trip).
bool place(rdx_context *ctx, uint64_t bytes, int device, Placement &pl) {
    const size_t n = ctx->entries.size();
    const size_t start = (size_t)(ctx->rr.fetch_add(1, std::memory_order_relaxed) % n);
    size_t best = n;
    uint64_t best_load = 0;
    for (size_t k = 0; k < n; ++k) {
        const size_t i = (start + k) % n;
        const PoolEntry &e = *ctx->entries[i];
        if (device >= 0 && e.device != device) continue;
        const uint64_t load = e.outstanding.load(std::memory_order_relaxed);
        if (best == n || load < best_load) {
            best = i;
            best_load = load;
        }
    }
    if (best == n) return false;
    pl.e = ctx->entries[best].get();
    pl.weight = bytes + (64u << 10);
    const uint64_t now = pl.e->outstanding.fetch_add(pl.weight, std::memory_order_relaxed) + pl.weight;
    if (!ctx->served.load(std::memory_order_relaxed)) ctx->served.store(true, std::memory_order_relaxed);
    std::lock_guard<std::mutex> g(pl.e->mu);
    ++pl.e->requests;
    pl.e->placed_bytes += bytes;
    pl.e->peak_outstanding = std::max(pl.e->peak_outstanding, now);
    return true;
}

// A workspace of the entry for the duration of one request: a free one, a new one below the cap, or —
// with max_workspaces busy — the next one released (back-pressure, resource_manager.rs:54-89).
struct WsLease {
    PoolEntry *e = nullptr;
    rdx_workspace *ws = nullptr;
    WsLease() = default;
    WsLease(const WsLease &) = delete;
    ~WsLease() {
        if (!ws) return;
        {
            std::lock_guard<std::mutex> g(e->mu);
            e->free_ws.push_back(ws);
            --e->busy;
        }
        e->ws_cv.notify_one();
    }
};

const rdx_status kBusy = static_cast<rdx_status>(255);   // internal: no workspace free right now

// `wait` false: kBusy instead of waiting when every workspace is busy (the fast path's try).
rdx_status acquire_ws(rdx_context *ctx, PoolEntry &e, WsLease &lease, bool wait = true) {
    std::unique_lock<std::mutex> lk(e.mu);
    bool waited = false;
    while (e.free_ws.empty() && e.all_ws.size() + e.creating >= ctx->cfg.max_workspaces) {
        if (!wait) return kBusy;
        if (!waited) ++e.waits;
        waited = true;
        e.ws_cv.wait(lk);
    }
    ++e.busy;
    if (!e.free_ws.empty()) {
        lease.ws = e.free_ws.back();
        e.free_ws.pop_back();
        lease.e = &e;
        return RDX_OK;
    }
    ++e.creating;   // counts against the cap while it is created outside the lock
    lk.unlock();
    rdx_workspace *ws = nullptr;
    const rdx_status st = create_workspace(e.device, &ws, ctx->cfg.inflate_fallback != 0);
    lk.lock();
    --e.creating;
    if (st) {
        --e.busy;
        lk.unlock();
        e.ws_cv.notify_one();
        return st;
    }
    e.all_ws.push_back(ws);
    lease.ws = ws;
    lease.e = &e;
    return RDX_OK;
}

void destroy_lane(Lane *L) {
    if (!L) return;
    if (L->ws && L->owns_ws) destroy_workspace(L->ws);   // synchronises its stream first
    if (L->done) (void)hipEventDestroy(L->done);
    if (L->h_res) (void)hipHostFree(L->h_res);
    delete L;
}

// A lane: its own stream / workspace, or (`share`) the stream of another lane, so that a second launch
// queues behind the first on the device instead of waiting for its results on the host (launch-ahead).
rdx_status create_lane(int device, Lane **out, Lane *share = nullptr) {
    auto *L = new (std::nothrow) Lane();
    if (!L) return RDX_E_OUT_OF_MEMORY;
    rdx_status st = RDX_OK;
    if (share) {
        L->ws = share->ws;
        L->owns_ws = false;
    } else {
        st = create_workspace(device, &L->ws, false);
    }
    if (!st) {
        // fine-grained (coherent): the kernel's system-scope stores land in host memory directly
        hipError_t e = hipHostMalloc((void **)&L->h_res, kTableChunks * kSlotWords * sizeof(uint64_t),
                                     hipHostMallocCoherent);
        if (e == hipSuccess) std::memset(L->h_res, 0, kTableChunks * kSlotWords * sizeof(uint64_t));
        if (e == hipSuccess) e = hipEventCreateWithFlags(&L->done, hipEventDisableTiming);
        st = map_err(e);
    }
    if (st) {
        destroy_lane(L);
        return st;
    }
    if (share) {
        L->twin = share;
        share->twin = L;
    }
    *out = L;
    return RDX_OK;
}

// Launch a lane's batch: the queued requests' descriptors with their outputs bound to the lane's host
// slots (the folds write them over the link as tagged granules; KOut::host_slots).
rdx_status launch_lane(Lane &L) {
    rdx_workspace *ws = L.ws;
    // the epoch wraps at 2^16 launches: clear the slots so that no stale slot can carry a current tag (the
    // lane, and its twin on the same stream, are idle here: the dispatcher waits for that at a wrap; the
    // stream orders the next launch after everything before)
    if (ws->epoch + 1 > 0xffffu) {
        std::memset(L.h_res, 0, kTableChunks * kSlotWords * sizeof(uint64_t));
        if (L.twin) std::memset(L.twin->h_res, 0, kTableChunks * kSlotWords * sizeof(uint64_t));
    }
    rdx_status st;
    const hipStream_t s = ws->own_stream;
    // host chunks: the launch waits on the device for their H2D copies (no host synchronisation)
    for (uint32_t i = 0; i < L.n; ++i)
        if (L.batch[i]->dep) RDX_HIP(hipStreamWaitEvent(s, L.batch[i]->dep, 0));
    if (L.group) {   // one plan, the chunks in the kernel arguments, chunk i's result into slot i
        const Job &j0 = *L.batch[0];
        KOut out{};
        if ((st = next_epoch(ws, s, out.epoch))) return st;
        out.body = reinterpret_cast<uint8_t *>(L.h_res);
        out.host_slots = 1;
        out.fold_last = L.n <= kFoldLastChunks && tuning().fold_last ? fold_mode() : 0u;
        if (j0.mode == Mode::AllContig) {
            KAllContig a = j0.contig;
            a.src.table = 1;
            for (uint32_t i = 0; i < L.n; ++i) a.tbl.p[i] = L.batch[i]->chunk;
            const uint64_t te = a.src.fused ? 4096 : 16384 / j0.esz;
            a.blocks_per_chunk = pick_bpc((a.n + te - 1) / te, L.n, ws->cus);
            // chunks in host memory: a few workgroups in all stream them over PCIe (each workgroup that reads
            // host memory adds ~0.9 us to the launch: 1 MiB in 27 us with 8, 50 us with 32, 258 us with 256;
            // profiles/r05_hread_probe.jsonl)
            if (j0.host_read)
                a.blocks_per_chunk = std::max<uint32_t>(1, (uint32_t)std::max(1, tuning().host_read_wgs) / L.n);
            if ((st = ensure(ws, ws->partials, (uint64_t)L.n * a.blocks_per_chunk * kRecordU64, s, true))) return st;
            if ((st = ensure(ws, ws->tickets, (uint64_t)L.n * kTicketWords, s, true))) return st;
            out.partials = ws->partials.p;
            out.tickets = ws->tickets.p;
            a.out = out;
            RDX_HIP(launch_all_contig(j0.dtype, j0.op, a, L.n, s));
        } else {
            KAllStrided a = j0.strided;
            a.src.table = 1;
            for (uint32_t i = 0; i < L.n; ++i) a.tbl.p[i] = L.batch[i]->chunk;
            const uint64_t per_block = (uint64_t)kBlock * (a.vec > 1 ? 4 : 8);
            const uint64_t want = (a.view.n / a.vec + per_block - 1) / per_block;
            const uint64_t cap = ((uint64_t)ws->cus * 8 + L.n - 1) / L.n;
            a.blocks_per_chunk = (uint32_t)std::max<uint64_t>(1, std::min(want, std::max<uint64_t>(cap, 1)));
            if ((st = ensure(ws, ws->partials, (uint64_t)L.n * a.blocks_per_chunk * kRecordU64, s, true))) return st;
            if ((st = ensure(ws, ws->tickets, (uint64_t)L.n * kTicketWords, s, true))) return st;
            out.partials = ws->partials.p;
            out.tickets = ws->tickets.p;
            a.out = out;
            RDX_HIP(launch_all_strided(j0.dtype, j0.op, a, L.n, s));
        }
    } else {
        KMultiReq g[kMultiMaxItems];
        for (uint32_t i = 0; i < L.n; ++i) {
            g[i] = L.batch[i]->q;
            g[i].body = reinterpret_cast<uint8_t *>(L.h_res + (uint64_t)i * kSlotWords);
            g[i].counts = nullptr;
            g[i].status = nullptr;
        }
        if ((st = launch_multi_group(ws, g, L.n, s, kMultiHostSlots))) return st;
    }
    if (L.done) RDX_HIP(hipEventRecord(L.done, s));
    L.tag = ws->epoch;
    L.remaining = L.n;
    L.polls = 0;
    return RDX_OK;
}

// Completion: the result is in the caller's buffers; release it, and wake it only if it is asleep
// (rdx_jobsync.hpp: the exchange is the last access to the Job).
void finish_job(Job &j, rdx_status st) {
    j.st = st;
    job_finish(j.state);
}

// The caller's wait: spin RDX_WAIT_SPIN pause iterations (0 = sleep at once), then sleep on the futex.
void wait_job(Job &j) { job_wait(j.state, tuning().wait_spin); }

// Poll a launched lane's slots: every request whose three granules carry the launch's tag is decoded into
// its caller's buffers and released.  `kernel_done`: the launch has ended (its event), so a slot still
// without the tag will never get it (a device fault): its request fails with RDX_E_DEVICE.  Returns true
// when the lane became free.
bool poll_lane(Lane &L, bool kernel_done) {
    for (uint32_t i = 0; i < L.n; ++i) {
        Job *j = L.batch[i];
        if (!j) continue;
        const uint64_t *slot = L.h_res + (uint64_t)i * kSlotWords;
        const uint64_t g0 = __atomic_load_n(slot + 0, __ATOMIC_ACQUIRE);
        const uint64_t g1 = __atomic_load_n(slot + 1, __ATOMIC_ACQUIRE);
        const uint64_t g2 = __atomic_load_n(slot + 2, __ATOMIC_ACQUIRE);
        const bool fresh = (g0 >> 48) == L.tag && (g1 >> 48) == L.tag && (g2 >> 48) == L.tag;
        if (!fresh && !kernel_done) continue;
        if (!fresh) {
            finish_job(*j, RDX_E_DEVICE);
        } else {
            const uint64_t value = (g0 & 0xffffffffull) | (g1 & 0xffffffffull) << 32;
            const int64_t count = (int64_t)(g2 & ((1ull << 40) - 1));
            if (j->body_bytes) std::memcpy(j->h_body, &value, j->body_bytes);   // little-endian: low bytes first
            if (j->n_counts) std::memcpy(j->h_counts, &count, sizeof count);
            finish_job(*j, (rdx_status)((g2 >> 40) & 0xffu));
        }
        L.batch[i] = nullptr;
        --L.remaining;
    }
    if (L.remaining) return false;
    L.n = 0;
    return true;
}

// Same plan and launch descriptor but the chunk: one batched launch serves both.
bool same_group(const Job &a, const Job &b) {
    if (a.mode != b.mode || a.dtype != b.dtype || a.op != b.op || a.host_read != b.host_read) return false;
    return a.mode == Mode::AllContig ? std::memcmp(&a.contig, &b.contig, sizeof a.contig) == 0
                                     : std::memcmp(&a.strided, &b.strided, sizeof a.strided) == 0;
}

// The next launch of a free lane: the oldest request's group (every queued request with its plan, up to
// kTableChunks) as one batched launch; a lone request with no partner among heterogeneous ones goes with
// them into one k_multi launch (up to kMultiMaxItems, in queue order, every one k_multi can take).
void form_batch(std::deque<Job *> &pending, Lane &L) {
    L.n = 0;
    Job *first = pending.front();
    uint32_t mates = 0;
    for (size_t i = 1; i < pending.size() && mates + 1 < (uint32_t)kTableChunks; ++i)
        if (same_group(*first, *pending[i])) ++mates;
    if (mates > 0 || !first->multi_ok) {
        L.group = true;
        for (auto it = pending.begin(); it != pending.end() && L.n < (uint32_t)kTableChunks;) {
            if (*it == first || same_group(*first, **it)) {
                L.batch[L.n++] = *it;
                it = pending.erase(it);
            } else {
                ++it;
            }
        }
        return;
    }
    L.group = false;
    for (auto it = pending.begin(); it != pending.end() && L.n < (uint32_t)kMultiMaxItems;) {
        if ((*it)->multi_ok) {
            L.batch[L.n++] = *it;
            it = pending.erase(it);
        } else {
            ++it;
        }
    }
}

// The entry's dispatcher thread: the only thread that launches coalesced work on this entry.  It takes
// everything queued (up to kMultiMaxItems per launch, oldest first) onto any free lane at once, polls the
// lanes' events, and completes their requests.  While the lanes are busy the queue grows, so launches
// fill up by themselves under load; a lone request launches at once.  With nothing queued or in flight
// it sleeps on job_cv.
void dispatcher_loop(rdx_context *ctx, PoolEntry *e) {
    (void)hipSetDevice(e->device);
    (void)pthread_setname_np(pthread_self(), "rdx-dispatch");
    // this thread's naps: microseconds, not the default 50 us timer slack
    (void)prctl(PR_SET_TIMERSLACK, 2000UL, 0, 0, 0);
    std::deque<Job *> pending;
    std::vector<Waiter *> watched;
    uint32_t in_flight = 0;
    auto last_progress = std::chrono::steady_clock::now();
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(e->mu);
            if (pending.empty() && in_flight == 0 && watched.empty()) {
                e->dispatcher_idle = true;
                e->job_cv.wait(lk, [&] { return !e->jobs.empty() || !e->watch.empty() || e->stop; });
                e->dispatcher_idle = false;
                if (e->jobs.empty() && e->watch.empty() && e->stop) return;
                last_progress = std::chrono::steady_clock::now();
            }
            while (!e->jobs.empty()) {
                pending.push_back(e->jobs.front());
                e->jobs.pop_front();
            }
            if (!e->watch.empty()) {
                watched.insert(watched.end(), e->watch.begin(), e->watch.end());
                e->watch.clear();
            }
        }
        bool progressed = false;
        // launch on free lanes (created up to coalesce_lanes)
        while (!pending.empty()) {
            // a free lane on an idle stream first, then (launch-ahead pairs) a free lane whose twin is in
            // flight; at an epoch wrap only a lane whose twin is idle too
            Lane *lane = nullptr;
            for (Lane *l : e->lanes)
                if (l->n == 0 && (!l->twin || l->twin->n == 0)) { lane = l; break; }
            if (!lane) {
                for (Lane *l : e->lanes)
                    if (l->n == 0 && l->ws->epoch + 1 <= 0xffffu) { lane = l; break; }
            }
            if (!lane && e->lanes.size() < ctx->cfg.coalesce_lanes) {
                // with RDX_COALESCE_DEPTH=2 every second lane shares the stream of the one before
                Lane *share = tuning().coalesce_depth >= 2 && e->lanes.size() % 2 == 1 ? e->lanes.back() : nullptr;
                if (create_lane(e->device, &lane, share) == RDX_OK) e->lanes.push_back(lane);
                else lane = nullptr;
            }
            if (!lane) {
                if (e->lanes.empty()) {   // nothing can serve the queue: fail it
                    for (Job *j : pending) finish_job(*j, RDX_E_DEVICE);
                    pending.clear();
                }
                break;
            }
            form_batch(pending, *lane);
            const uint32_t n = lane->n;
            const bool host_reads = lane->group && lane->batch[0]->host_read;
            const auto t0 = std::chrono::steady_clock::now();
            const rdx_status st = launch_lane(*lane);
            lane->t0 = std::chrono::steady_clock::now();
            e->t_launch += std::chrono::duration<double, std::micro>(lane->t0 - t0).count();
            ++e->n_launch;
            if (st) {
                for (uint32_t i = 0; i < lane->n; ++i) finish_job(*lane->batch[i], st);
                lane->n = 0;
            } else {
                ++in_flight;
            }
            {
                std::lock_guard<std::mutex> g(e->mu);
                ++e->launches;
                e->coalesced += n;
                if (host_reads && !st) e->host_reads += n;
            }
            progressed = true;
        }
        // results of launched lanes: their slots, and (every 64th poll) the launch's event as the fault
        // fallback (the lane's stream idle)
        for (Lane *l : e->lanes) {
            if (l->n == 0) continue;
            bool kernel_done = false;
            if (++l->polls % 64 == 0) {   // the launch's end (an event query: a stream query on a busy stream
                                          // costs a HIP runtime thread spinning on a marker)
                const hipError_t q = hipEventQuery(l->done);
                kernel_done = q != hipErrorNotReady;
            }
            const uint32_t before = l->remaining;
            const auto t1 = std::chrono::steady_clock::now();
            if (poll_lane(*l, kernel_done)) {
                e->t_flight += std::chrono::duration<double, std::micro>(t1 - l->t0).count();
                ++e->n_done;
                --in_flight;
            }
            if (l->remaining != before) progressed = true;
        }
        // callers sleeping on an event of their own stream (wait_event): wake each one whose event completed
        // (the exchange in job_finish is the last access to its Waiter)
        for (size_t i = 0; i < watched.size();) {
            Waiter *w = watched[i];
            const hipError_t q = hipEventQuery(w->ev);
            if (q == hipErrorNotReady) {
                ++i;
                continue;
            }
            watched[i] = watched.back();
            watched.pop_back();
            w->st = q == hipSuccess ? RDX_OK : map_err(q);
            job_finish(w->state);
            progressed = true;
        }
        // nothing arrived and nothing completed: yield for RDX_DISPATCH_IDLE_US, then (a long launch or copy
        // in flight) nap RDX_DISPATCH_NAP_US between polls instead of keeping a core busy
        const auto now = std::chrono::steady_clock::now();
        if (progressed) {
            last_progress = now;
        } else if (std::chrono::duration<double, std::micro>(now - last_progress).count() < tuning().idle_us) {
            std::this_thread::yield();
        } else {
            const timespec ts{0, 1000L * std::max(1, tuning().nap_us)};
            nanosleep(&ts, nullptr);
        }
    }
}

// The entry's dispatcher thread, started on first use (with e.mu held).
bool ensure_dispatcher(rdx_context *ctx, PoolEntry &e) {
    if (e.dispatcher.joinable()) return true;
    try {
        e.dispatcher = std::thread(dispatcher_loop, ctx, &e);
    } catch (...) {
        return false;
    }
    return true;
}

// How long a caller spins for its own result before it sleeps (RDX_HOST_SPIN_US overrides): the time an
// idle device needs for the request (its PCIe bytes at >= 40 GB/s, its HBM bytes, a launch), so that a lone
// request is not slowed by a sleep / wake-up; only a short spin when other requests are in flight on the
// entry (this one queues behind them: the link or the device is busy, and the caller's core is worth
// more to the server's other threads than the microseconds a wake-up costs).
double spin_budget_us(const PoolEntry &e, uint64_t own_weight, uint64_t pcie_bytes, uint64_t hbm_bytes) {
    if (tuning().host_spin_us >= 0) return tuning().host_spin_us;
    if (e.outstanding.load(std::memory_order_relaxed) > own_weight + own_weight / 2) return 2.0;
    return 20.0 + (double)pcie_bytes / 40e3 + (double)hbm_bytes / 4e6;
}

// Wait for `ev` (recorded on a stream the caller owns): spin on it for `budget_us`, then sleep until the
// entry's dispatcher sees it complete.  HIP's own waits (hipStreamSynchronize / hipEventSynchronize, also
// with hipEventBlockingSync) spin for as long as the work takes (profiles/r05_wait_probe.jsonl).
rdx_status wait_event(rdx_context *ctx, PoolEntry &e, hipEvent_t ev, double budget_us) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return RDX_OK;
        if (q != hipErrorNotReady) return map_err(q);
        if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >= budget_us) break;
        for (int k = 0; k < 32; ++k) __builtin_ia32_pause();
    }
    Waiter w;
    w.ev = ev;
    e.sleeps.fetch_add(1, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(e.mu);
        if (!ensure_dispatcher(ctx, e)) return RDX_E_OUT_OF_MEMORY;
        e.watch.push_back(&w);
        if (e.dispatcher_idle) e.job_cv.notify_one();
    }
    job_wait(w.state, 0);
    return w.st;
}

// The end of everything queued on the workspace's stream so far (wait_event).
rdx_status wait_stream(rdx_context *ctx, PoolEntry &e, rdx_workspace *ws, double budget_us) {
    RDX_HIP(hipEventRecord(ws->done_ev, ws->own_stream));
    return wait_event(ctx, e, ws->done_ev, budget_us);
}

// The idle-queue fast path: a coalescible request arriving while its entry's coalescer has nothing queued
// does not hand over to the dispatcher thread (a wake-up, a launch, a completion and a wake-up: 21-33 us
// at one caller where a direct launch takes 16-18 us).  The caller launches it itself as a one-request
// batched launch on its own workspace's stream — the same kernels and the same tagged page-locked result
// slot as a coalescer lane (rdx_device.hpp put_host_slot) — and spins on the slot.  At most RDX_DIRECT_MAX
// callers per entry take it at once; the rest (a loaded server) queue and coalesce.
bool claim_direct(PoolEntry &e) {
    std::lock_guard<std::mutex> g(e.mu);
    if (!e.jobs.empty() || e.direct_active >= (uint32_t)std::max(0, tuning().direct_max)) return false;
    ++e.direct_active;
    return true;
}

void release_direct(PoolEntry &e, bool served, bool host_read = false) {
    std::lock_guard<std::mutex> g(e.mu);
    --e.direct_active;
    if (served) ++e.direct;
    if (served && host_read) ++e.host_reads;
}

// RDX_PHASES: when the launch call returned and when the result was seen (execute_host's phase record)
struct DirectTimes {
    std::chrono::steady_clock::time_point launched, seen;
};

rdx_status run_direct(rdx_context *ctx, PoolEntry &e, rdx_workspace *ws, Job &job, double budget_us,
                      DirectTimes *tm = nullptr) {
    RDX_HIP(hipSetDevice(ws->device));
    constexpr size_t slot_bytes = kTableChunks * kSlotWords * sizeof(uint64_t);
    if (!ws->h_slot) {
        void *p = nullptr;
        RDX_HIP(hipHostMalloc(&p, slot_bytes, hipHostMallocCoherent));
        std::memset(p, 0, slot_bytes);
        ws->h_slot = static_cast<uint64_t *>(p);
    }
    Lane L;   // a one-request lane over the caller's workspace
    L.ws = ws;
    L.owns_ws = false;
    L.h_res = ws->h_slot;
    L.group = true;
    L.batch[0] = &job;
    L.n = 1;
    L.done = ws->done_ev;   // recorded behind the launch
    rdx_status st = launch_lane(L);
    if (st) return st;
    if (tm) {
        if (ws->ph_ev[2]) RDX_HIP(hipEventRecord(ws->ph_ev[2], ws->own_stream));
        tm->launched = std::chrono::steady_clock::now();
    }
    // the slot's tag arrives with the fold; the stream query (every 64th poll) catches a launch that ended
    // without writing it (a device fault: RDX_E_DEVICE).  Past the spin budget the caller sleeps until
    // the launch has ended (wait_event), then reads its slot.
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t polls = 1;; ++polls) {
        const bool kernel_done = polls % 64 == 0 && hipEventQuery(ws->done_ev) != hipErrorNotReady;
        if (poll_lane(L, kernel_done)) {
            if (tm) tm->seen = std::chrono::steady_clock::now();
            return job.st;
        }
        if (polls % 16 == 0 &&
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >= budget_us)
            break;
        __builtin_ia32_pause();
    }
    if ((st = wait_event(ctx, e, ws->done_ev, 0.0))) return st;
    poll_lane(L, true);   // the slot was written before the launch ended, or the request fails: RDX_E_DEVICE
    if (tm) tm->seen = std::chrono::steady_clock::now();
    return job.st;
}

// Queue the request on its entry's coalescer and wait for its result (spinning: the result comes back
// within microseconds of the launch, far below a sleep/wake-up round trip).
rdx_status coalesce(rdx_context *ctx, PoolEntry &e, Job &job) {
    {
        std::lock_guard<std::mutex> g(e.mu);
        if (!ensure_dispatcher(ctx, e)) return RDX_E_OUT_OF_MEMORY;
        e.jobs.push_back(&job);
        if (e.dispatcher_idle) e.job_cv.notify_one();
    }
    wait_job(job);
    return job.st;
}

// rdx_execute_cbor: the response leaves the device as its CBOR body (k_cbor), in a pooled
// page-locked block.
struct CborOut {
    uint32_t flags = 0;
    void *host = nullptr;   // pool block (rdx_result.body)
    uint64_t len = 0;       // encoded bytes
};
constexpr uint64_t kCborOneTrip = 1ull << 20;   // bounds up to this come back whole, in one round trip

// operation<T>() for a chunk in host memory (app.rs:163-183): plan, bind the response buffers
// (caller-provided or pooled), H2D, kernels, D2H; blocks until the response is in host memory.
// With `cb`, the response is serialised on the device (serde_cbor CBORResponse, app.rs:33-40) and only
// its CBOR body comes back.
// `resident_device` >= 0: the chunk is in HBM of that device (rdx_execute_resident), nothing crosses PCIe
// but the response.
rdx_status execute_host(rdx_context *ctx, const rdx_request &req, const uint8_t *chunk, uint64_t chunk_len,
                        const std::function<rdx_status(const rdx_response_info &, void **, int64_t **)> &bind,
                        rdx_response_info *info, CborOut *cb = nullptr, int resident_device = -1) {
    const auto t_enter = std::chrono::steady_clock::now();
    const double c_enter = tuning().phases ? thread_cpu_us() : 0.0;
    const bool resident = resident_device >= 0;
    const bool compressed = req.compression != RDX_COMPRESSION_NONE;
    ExecPlan p;
    rdx_status st;
    void *body = nullptr;
    int64_t *counts = nullptr;
    if (!compressed) {
        if ((st = make_plan(req, chunk_len, p))) return st;
        *info = p.info;
        if ((st = bind(p.info, &body, &counts))) return st;
    }

    Placement pl;
    if (!place(ctx, chunk_len, resident_device, pl)) return resident ? RDX_E_INVALID_ARGUMENT : RDX_E_NO_DEVICE;
    PoolEntry &entry = *pl.e;
    // a small all-axes request joins the entry's coalesced k_multi launches (chunk at d_base in HBM)
    // (`host_read`: the direct host-read path's own size bound, RDX_HOST_READ_KIB)
    auto coalescible = [&](const uint8_t *d_base, Job &job, bool host_read = false) -> bool {
        if (compressed || cb || !ctx->cfg.coalesce) return false;
        const uint64_t cap = host_read ? (uint64_t)std::max(0, tuning().host_read_kib) * 1024
                                       : resident ? ctx->cfg.coalesce_max_bytes : ctx->cfg.coalesce_host_max_bytes;
        if (chunk_len > cap) return false;
        if ((p.mode != Mode::AllContig && p.mode != Mode::AllStrided) || !p.unfused_es.empty() || !p.miss_list.empty())
            return false;
        job.mode = p.mode;
        job.dtype = p.dtype;
        job.op = p.op;
        job.esz = p.esz;
        job.chunk = d_base;
        KSrc src{};
        src.plane = chunk_len / p.esz;
        src.fused = p.fused;
        src.bswap = p.bswap;
        if (p.mode == Mode::AllContig) {
            job.contig = p.all_contig;
            job.contig.src = src;
            job.contig.miss = p.miss;
        } else {
            job.strided = p.all_strided;
            job.strided.src = src;
            job.strided.miss = p.miss;
            job.strided.vec = vec_width(job.strided.view, p.esz, d_base, nullptr, 1, p.fused);
        }
        rdx_multi_item it{};
        it.req = &req;
        it.d_chunk = d_base;
        it.chunk_len = chunk_len;
        job.multi_ok = multi_req(p, it, job.q);
        job.body_bytes = p.info.body_bytes;
        job.n_counts = p.info.n_counts;
        job.h_body = body;
        job.h_counts = counts;
        return true;
    };
    if (resident) {
        Job job;
        if (coalescible(chunk, job)) {
            if (claim_direct(entry)) {
                WsLease lease;
                if (acquire_ws(ctx, entry, lease, false) == RDX_OK) {
                    st = run_direct(ctx, entry, lease.ws, job, spin_budget_us(entry, pl.weight, 0, chunk_len));
                    release_direct(entry, true);
                    return st;
                }
                release_direct(entry, false);
            }
            return coalesce(ctx, entry, job);
        }
    }
    // a small page-locked host chunk, all-axes over a contiguous run: no H2D copy and no workspace buffer —
    // the kernel reads the chunk over PCIe with a few workgroups (Job::host_read) and its fold writes the
    // result into a page-locked slot.  On an idle entry the caller launches it itself (direct); otherwise
    // same-plan host chunks share one coalesced launch that keeps the readers few (launch_lane).
    if (!resident && !compressed && !cb && chunk_len <= (uint64_t)std::max(0, tuning().host_read_kib) * 1024) {
        const uint8_t *alias = host_alias(chunk);
        Job job;
        if (alias && coalescible(alias, job, true) && job.mode == Mode::AllContig) {
            job.host_read = true;
            job.multi_ok = false;
            if (claim_direct(entry)) {
                WsLease lease;
                if (acquire_ws(ctx, entry, lease, false) == RDX_OK) {
                    DirectTimes tm;
                    const bool ph = tuning().phases != 0;
                    const auto t_ready = std::chrono::steady_clock::now();
                    st = run_direct(ctx, entry, lease.ws, job, spin_budget_us(entry, pl.weight, chunk_len, 0), &tm);
                    release_direct(entry, true, true);
                    if (ph && !st) {
                        const auto t_ret = std::chrono::steady_clock::now();
                        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
                            return std::chrono::duration<double, std::micro>(b - a).count();
                        };
                        const double v[8] = {us(t_enter, t_ready), 0.0, us(t_ready, tm.launched), us(tm.launched, tm.seen),
                                             us(tm.seen, t_ret), us(t_enter, t_ret), 0.0, 0.0};
                        phase_add(0, v);
                    }
                    return st;
                }
                release_direct(entry, false);
            }
            return coalesce(ctx, entry, job);
        }
    }
    WsLease lease;
    if ((st = acquire_ws(ctx, entry, lease))) return st;
    rdx_workspace *ws = lease.ws;
    auto run = [&]() -> rdx_status {
        RDX_HIP(hipSetDevice(ws->device));
        hipStream_t s = ws->own_stream;
        rdx_status r;
        if (!resident && !cb && !compressed && p.mode == Mode::Map && p.unfused_es.empty() && !p.fused && p.map.view.ndim >= 1 &&
            p.map.view.count[p.map.view.ndim - 1] >= 2 && chunk_len >= (32ull << 20) && is_pinned(chunk) &&
            is_pinned(body) && (p.map.kind == 0 || is_pinned(counts))) {
            if ((r = ensure_aux(ws))) return r;
            return map_pipelined(ctx, entry, ws, p, chunk, chunk_len, static_cast<uint8_t *>(body), counts);
        }
        const uint8_t *src = chunk;
        // RDX_PHASES: the direct path's record (phase_sums)
        const bool ph = tuning().phases != 0;
        auto phase_record = [&](int path, std::chrono::steady_clock::time_point t_ready,
                                std::chrono::steady_clock::time_point t_issued, const DirectTimes &tm) -> rdx_status {
            const auto t_ret = std::chrono::steady_clock::now();
            RDX_HIP(hipEventSynchronize(ws->ph_ev[2]));
            float copy_ms = 0, kern_ms = 0;
            if (path == 1) RDX_HIP(hipEventElapsedTime(&copy_ms, ws->ph_ev[0], ws->ph_ev[1]));
            RDX_HIP(hipEventElapsedTime(&kern_ms, ws->ph_ev[1], ws->ph_ev[2]));
            auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
                return std::chrono::duration<double, std::micro>(b - a).count();
            };
            const double v[8] = {us(t_enter, t_ready), us(t_ready, t_issued), us(t_issued, tm.launched),
                                 us(tm.launched, tm.seen), us(tm.seen, t_ret), us(t_enter, t_ret), 1e3 * copy_ms,
                                 1e3 * kern_ms};
            phase_add(path, v);
            return RDX_OK;
        };
        if (ph)
            for (hipEvent_t &ev : ws->ph_ev)
                if (!ev) RDX_HIP(hipEventCreate(&ev));
        if (!resident) {
            Job job;
            if ((r = ensure(ws, ws->chunk, std::max<uint64_t>(chunk_len, 16), s))) return r;
            const auto t_ready = std::chrono::steady_clock::now();
            const double c_ready = ph ? thread_cpu_us() : 0.0;
            if (ph) RDX_HIP(hipEventRecord(ws->ph_ev[0], s));
            if (chunk_len) RDX_HIP(hipMemcpyAsync(ws->chunk.p, chunk, chunk_len, hipMemcpyHostToDevice, s));
            src = ws->chunk.p;
            if (coalescible(src, job)) {
                if (claim_direct(entry)) {   // launched behind the copy on the same stream
                    const auto t_issued = std::chrono::steady_clock::now();
                    if (ph) RDX_HIP(hipEventRecord(ws->ph_ev[1], s));
                    DirectTimes tm;
                    r = run_direct(ctx, entry, ws, job, spin_budget_us(entry, pl.weight, chunk_len, chunk_len),
                                   ph ? &tm : nullptr);
                    release_direct(entry, true);
                    if (ph && !r && (r = phase_record(1, t_ready, t_issued, tm))) return r;
                    return r;
                }
                // the coalesced launch waits for the copy on the device; this thread does not
                RDX_HIP(hipEventRecord(ws->copy_ev, s));
                job.dep = ws->copy_ev;
                if (!ph) return coalesce(ctx, entry, job);
                const auto t_q = std::chrono::steady_clock::now();
                const double c_q = thread_cpu_us();
                r = coalesce(ctx, entry, job);
                const auto t_w = std::chrono::steady_clock::now();
                const double c_w = thread_cpu_us();
                auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
                    return std::chrono::duration<double, std::micro>(b - a).count();
                };
                const double v[8] = {us(t_enter, t_ready), us(t_ready, t_q), us(t_q, t_w), us(t_enter, t_w),
                                     c_ready - c_enter, c_q - c_ready, c_w - c_q, c_w - c_enter};
                phase_add(2, v);
                return r;
            }
        }
        if ((r = ensure(ws, ws->body, std::max<uint64_t>(p.info.body_bytes, 16), s))) return r;
        if ((r = ensure(ws, ws->counts, std::max<uint64_t>(p.info.n_counts, 1), s))) return r;
        if ((r = ensure(ws, ws->status, 2, s))) return r;   // [0] the operation's, [1] the CBOR encoder's
        uint64_t len = chunk_len;
        if (compressed) {  // the chunk crossed PCIe compressed; inflate it in HBM, then plan on its size
            uint64_t hint = 0;
            if (!resident && req.compression == RDX_COMPRESSION_GZIP && chunk_len >= 18) {  // RFC 1952 ISIZE
                const uint8_t *t = chunk + chunk_len - 4;
                hint = (uint64_t)t[0] | (uint64_t)t[1] << 8 | (uint64_t)t[2] << 16 | (uint64_t)t[3] << 24;
            }
            if (!resident && req.compression == RDX_COMPRESSION_BLOSC2) {  // blosc2_cbuffer_sizes, compression.rs:33
                uint64_t cb = 0, bs = 0;
                rdx_blosc2_cbuffer_sizes(chunk, chunk_len, &hint, &cb, &bs);
            }
            if ((r = decompress_request(ws, req, src, chunk_len, hint, s, &len, resident ? nullptr : chunk))) return r;
            src = ws->raw.p;
            if ((r = make_plan(req, len, p))) return r;
            *info = p.info;
            if ((r = bind(p.info, &body, &counts))) return r;
            if ((r = ensure(ws, ws->body, std::max<uint64_t>(p.info.body_bytes, 16), s))) return r;
            if ((r = ensure(ws, ws->counts, std::max<uint64_t>(p.info.n_counts, 1), s))) return r;
        }
        RDX_HIP(hipMemsetAsync(ws->status.p, 0, sizeof(uint32_t), s));
        if ((r = run_device(ws, p, src, nullptr, 1, len, ws->body.p, ws->counts.p, ws->status.p, s)))
            return r;
        if (!ws->h_back) RDX_HIP(hipHostMalloc((void **)&ws->h_back, 16 + kBackStage, hipHostMallocDefault));
        uint32_t &status = *reinterpret_cast<uint32_t *>(ws->h_back);
        status = 0;
        if (cb) {   // encode on the device; the length (and, for small bounds, the bytes) in one trip
            const uint64_t bound = rdx_cbor_bound(&p.info, cb->flags);
            if (!bound) return RDX_E_INVALID_ARGUMENT;
            if ((r = ensure(ws, ws->cbor, bound, s))) return r;
            if ((r = ensure(ws, ws->cbor_len, 1, s))) return r;
            if ((r = pool_alloc(ctx, bound, &cb->host))) return r;
            // the encoder's own status word (a hand-off fault in k_cbor_pack) next to the operation's: cbor_device
            // clears the one it is given
            if ((r = cbor_device(ws, &p.info, ws->body.p, ws->counts.p, cb->flags, ws->cbor.p, bound, ws->cbor_len.p,
                                 ws->status.p + 1, s)))
                return r;
            uint64_t &n = ws->h_back[1];
            n = 0;
            uint32_t &enc_status = *(reinterpret_cast<uint32_t *>(ws->h_back) + 1);
            enc_status = 0;
            RDX_HIP(hipMemcpyAsync(&n, ws->cbor_len.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
            RDX_HIP(hipMemcpyAsync(&status, ws->status.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            if (bound <= kCborOneTrip) RDX_HIP(hipMemcpyAsync(cb->host, ws->cbor.p, bound, hipMemcpyDeviceToHost, s));
            if ((r = wait_stream(ctx, entry, ws, spin_budget_us(entry, pl.weight, resident ? 0 : chunk_len, len))))
                return r;
            if (status) return (rdx_status)status;
            if (enc_status) return (rdx_status)enc_status;
            if (n > bound) return RDX_E_DEVICE;   // a length the encoder cannot produce: never copy past the block
            if (bound > kCborOneTrip) {
                RDX_HIP(hipMemcpyAsync(cb->host, ws->cbor.p, n, hipMemcpyDeviceToHost, s));
                if ((r = wait_stream(ctx, entry, ws, spin_budget_us(entry, pl.weight, n, 0)))) return r;
            }
            cb->len = n;
            return trim_cbor_stage(ws, s);   // (the stream is idle here)
        }
        // a small response into pageable buffers goes through the page-locked block (then one host memcpy)
        const uint64_t bb = p.info.body_bytes, cbytes = p.info.n_counts * sizeof(int64_t);
        const uint64_t bb16 = (bb + 15) / 16 * 16;
        const bool stage = bb16 + cbytes <= kBackStage && ((bb && !is_pinned(body)) || (cbytes && !is_pinned(counts)));
        uint8_t *const st_body = reinterpret_cast<uint8_t *>(ws->h_back + 2);
        if (bb) RDX_HIP(hipMemcpyAsync(stage ? st_body : body, ws->body.p, bb, hipMemcpyDeviceToHost, s));
        if (cbytes) RDX_HIP(hipMemcpyAsync(stage ? st_body + bb16 : (uint8_t *)counts, ws->counts.p, cbytes, hipMemcpyDeviceToHost, s));
        RDX_HIP(hipMemcpyAsync(&status, ws->status.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        if ((r = wait_stream(ctx, entry, ws, spin_budget_us(entry, pl.weight, (resident ? 0 : chunk_len) + bb + cbytes, len))))
            return r;
        if (status) return (rdx_status)status;
        if (stage) {
            if (bb) std::memcpy(body, st_body, bb);
            if (cbytes) std::memcpy(counts, st_body + bb16, cbytes);
        }
        return RDX_OK;
    };
    return run();
}

}  // namespace

extern "C" {

rdx_status rdx_execute_multi_device(rdx_workspace *ws, uint64_t n, const rdx_multi_item *items, void *stream,
                                    uint32_t *statuses, rdx_response_info *infos) {
    if (!ws || (n && (!items || !statuses))) return RDX_E_INVALID_ARGUMENT;
    if (n == 0) return RDX_OK;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    RDX_HIP(hipSetDevice(ws->device));
    KMultiReq group[kMultiMaxItems];
    uint32_t in_group = 0;
    std::vector<uint64_t> rest;   // requests that run as their own launches
    rdx_status st;
    for (uint64_t i = 0; i < n; ++i) {
        const rdx_multi_item &it = items[i];
        statuses[i] = RDX_E_INVALID_ARGUMENT;
        if (!it.req) continue;
        if (it.req->compression != RDX_COMPRESSION_NONE) continue;
        ExecPlan p;
        st = make_plan(*it.req, it.chunk_len, p);
        statuses[i] = st;
        if (st) continue;
        if (infos) infos[i] = p.info;
        if ((!it.d_chunk && it.chunk_len) || (!it.d_body && p.info.body_bytes) || (!it.d_counts && p.info.n_counts)) {
            statuses[i] = RDX_E_INVALID_ARGUMENT;
            continue;
        }
        if (!multi_req(p, it, group[in_group])) {
            rest.push_back(i);
            continue;
        }
        if (++in_group == (uint32_t)kMultiMaxItems) {
            if ((st = launch_multi_group(ws, group, in_group, s))) return st;
            in_group = 0;
        }
    }
    if (in_group && (st = launch_multi_group(ws, group, in_group, s))) return st;
    for (uint64_t i : rest) {
        const rdx_multi_item &it = items[i];
        ExecPlan p;
        if ((st = make_plan(*it.req, it.chunk_len, p))) return st;   // planned above
        statuses[i] = run_device(ws, p, static_cast<const uint8_t *>(it.d_chunk), nullptr, 1, it.chunk_len,
                                 static_cast<uint8_t *>(it.d_body), it.d_counts, it.d_status, s);
        if (statuses[i] == RDX_E_DEVICE || statuses[i] == RDX_E_OUT_OF_MEMORY) return (rdx_status)statuses[i];
    }
    return RDX_OK;
}

rdx_status rdx_cbor_encode_device(rdx_workspace *ws, const rdx_response_info *info, const void *d_body,
                                  const int64_t *d_counts, uint32_t flags, void *d_out, uint64_t out_cap,
                                  uint64_t *d_out_len, uint32_t *d_status, void *stream) {
    if (!ws) return RDX_E_INVALID_ARGUMENT;
    RDX_HIP(hipSetDevice(ws->device));
    return cbor_device(ws, info, d_body, d_counts, flags, d_out, out_cap, d_out_len, d_status,
                       static_cast<hipStream_t>(stream));
}

rdx_status rdx_decompress_batch_device(rdx_workspace *ws, uint32_t compression, uint64_t n,
                                       const void *const *h_in_ptrs, const uint64_t *h_in_lens, void *d_out,
                                       uint64_t out_capacity, uint64_t *d_out_lens, uint32_t *d_errors, void *stream) {
    if (!ws || (compression != RDX_COMPRESSION_GZIP && compression != RDX_COMPRESSION_ZLIB &&
                compression != RDX_COMPRESSION_BLOSC2))
        return RDX_E_INVALID_ARGUMENT;
    if (n == 0) return RDX_OK;
    if (!h_in_ptrs || !h_in_lens || !d_out || !d_out_lens || !d_errors || out_capacity % 16 ||
        (uintptr_t)d_out % 16)
        return RDX_E_INVALID_ARGUMENT;
    for (uint64_t i = 0; i < n; ++i)
        if (!h_in_ptrs[i] && h_in_lens[i]) return RDX_E_INVALID_ARGUMENT;
    RDX_HIP(hipSetDevice(ws->device));
    return decompress_launch(ws, compression, n, reinterpret_cast<const uint8_t *const *>(h_in_ptrs), h_in_lens,
                             static_cast<uint8_t *>(d_out), out_capacity, d_out_lens, d_errors,
                             static_cast<hipStream_t>(stream));
}

rdx_status rdx_decompress_one_device(rdx_workspace *ws, uint32_t compression, const void *d_in, uint64_t len,
                                     void *d_out, uint64_t out_cap, uint64_t *out_len, uint32_t *error,
                                     void *stream) {
    if (!ws || !out_len || !error || (!d_in && len) || (!d_out && out_cap) ||
        (compression != RDX_COMPRESSION_GZIP && compression != RDX_COMPRESSION_ZLIB))
        return RDX_E_INVALID_ARGUMENT;
    RDX_HIP(hipSetDevice(ws->device));
    const hipStream_t s = static_cast<hipStream_t>(stream);
    rdx_request req{};
    req.abi_version = RDX_ABI_VERSION;
    req.compression = compression;
    uint64_t n = 0;
    *out_len = 0;
    const rdx_status st = decompress_request(ws, req, static_cast<const uint8_t *>(d_in), len, 0, s, &n, nullptr, true);
    if (st == RDX_E_DECOMPRESSION) {
        *error = g_inflate_error;
        return RDX_OK;
    }
    if (st) return st;
    *out_len = n;
    if (n > out_cap) {
        *error = RDX_INFLATE_OUTPUT_OVERFLOW;
        return RDX_OK;
    }
    if (n) RDX_HIP(hipMemcpyAsync(d_out, ws->raw.p, n, hipMemcpyDeviceToDevice, s));
    RDX_HIP(hipStreamSynchronize(s));
    *error = RDX_INFLATE_OK;
    return RDX_OK;
}

rdx_status rdx_execute(rdx_context *ctx, const rdx_request *req, const void *chunk, uint64_t chunk_len, void *body,
                       uint64_t body_capacity, int64_t *counts, uint64_t counts_capacity, rdx_response_info *info) {
    if (!ctx || !req || !info || (!chunk && chunk_len)) return RDX_E_INVALID_ARGUMENT;
    auto bind = [&](const rdx_response_info &inf, void **b, int64_t **c) -> rdx_status {
        if (body_capacity < inf.body_bytes || counts_capacity < inf.n_counts) return RDX_E_BUFFER_TOO_SMALL;
        if ((!body && inf.body_bytes) || (!counts && inf.n_counts)) return RDX_E_INVALID_ARGUMENT;
        *b = body;
        *c = counts;
        return RDX_OK;
    };
    return execute_host(ctx, *req, static_cast<const uint8_t *>(chunk), chunk_len, bind, info);
}

rdx_status rdx_execute_owned(rdx_context *ctx, const rdx_request *req, const void *chunk, uint64_t chunk_len,
                             rdx_result **out) {
    if (!ctx || !req || !out || (!chunk && chunk_len)) return RDX_E_INVALID_ARGUMENT;
    *out = nullptr;
    auto *r = new (std::nothrow) rdx_result();
    if (!r) return RDX_E_OUT_OF_MEMORY;
    auto bind = [&](const rdx_response_info &inf, void **b, int64_t **c) -> rdx_status {
        // one page-locked block: body (16 B aligned) then the counts
        const uint64_t bb = (inf.body_bytes + 15) / 16 * 16;
        void *mem = nullptr;
        rdx_status st = pool_alloc(ctx, bb + inf.n_counts * sizeof(int64_t), &mem);
        if (st) return st;
        r->body = mem;
        r->counts = reinterpret_cast<int64_t *>(static_cast<uint8_t *>(mem) + bb);
        *b = r->body;
        *c = r->counts;
        return RDX_OK;
    };
    const rdx_status st = execute_host(ctx, *req, static_cast<const uint8_t *>(chunk), chunk_len, bind, &r->info);
    if (st) {
        rdx_result_free(ctx, r);
        return st;
    }
    *out = r;
    return RDX_OK;
}

rdx_status rdx_execute_cbor(rdx_context *ctx, const rdx_request *req, const void *chunk, uint64_t chunk_len,
                            uint32_t flags, rdx_result **out) {
    if (!ctx || !req || !out || (!chunk && chunk_len) || (flags & ~(RDX_CBOR_SHAPE_AS_BYTES | RDX_CBOR_COUNT_AS_BYTES)))
        return RDX_E_INVALID_ARGUMENT;
    *out = nullptr;
    auto *r = new (std::nothrow) rdx_result();
    if (!r) return RDX_E_OUT_OF_MEMORY;
    auto bind = [&](const rdx_response_info &, void **b, int64_t **c) -> rdx_status {
        *b = nullptr;   // the response stays on the device until it is encoded
        *c = nullptr;
        return RDX_OK;
    };
    CborOut cb;
    cb.flags = flags;
    const rdx_status st = execute_host(ctx, *req, static_cast<const uint8_t *>(chunk), chunk_len, bind, &r->info, &cb);
    r->body = cb.host;
    r->cbor_bytes = cb.len;
    if (st) {
        rdx_result_free(ctx, r);
        return st;
    }
    *out = r;
    return RDX_OK;
}

void rdx_result_free(rdx_context *ctx, rdx_result *r) {
    if (!r) return;
    if (r->body) pool_free(ctx, r->body);
    delete r;
}

rdx_status rdx_execute_resident(rdx_context *ctx, int device, const rdx_request *req, const void *d_chunk,
                                uint64_t chunk_len, void *body, uint64_t body_capacity, int64_t *counts,
                                uint64_t counts_capacity, rdx_response_info *info) {
    if (!ctx || !req || !info || device < 0 || (!d_chunk && chunk_len)) return RDX_E_INVALID_ARGUMENT;
    auto bind = [&](const rdx_response_info &inf, void **b, int64_t **c) -> rdx_status {
        if (body_capacity < inf.body_bytes || counts_capacity < inf.n_counts) return RDX_E_BUFFER_TOO_SMALL;
        if ((!body && inf.body_bytes) || (!counts && inf.n_counts)) return RDX_E_INVALID_ARGUMENT;
        *b = body;
        *c = counts;
        return RDX_OK;
    };
    return execute_host(ctx, *req, static_cast<const uint8_t *>(d_chunk), chunk_len, bind, info, nullptr, device);
}

rdx_status rdx_context_configure(rdx_context *ctx, const rdx_context_config *cfg) {
    if (!ctx || !cfg || cfg->coalesce > 1 || cfg->inflate_fallback > 1) return RDX_E_INVALID_ARGUMENT;
    // the dispatchers, the placement and acquire_ws read the configuration without a lock: it is frozen
    // once the first request has been placed (rdx.h: configure before the context is shared)
    if (ctx->served.load(std::memory_order_relaxed)) return RDX_E_INVALID_ARGUMENT;
    ctx->cfg = effective_config(*cfg);
    return RDX_OK;
}

rdx_status rdx_context_stats(rdx_context *ctx, uint32_t index, rdx_device_stats *out) {
    if (!ctx || !out || index >= ctx->entries.size()) return RDX_E_INVALID_ARGUMENT;
    PoolEntry &e = *ctx->entries[index];
    std::lock_guard<std::mutex> g(e.mu);
    *out = rdx_device_stats{};
    out->device = e.device;
    out->workspaces = (uint32_t)e.all_ws.size();
    out->workspaces_busy = e.busy;
    out->max_workspaces = ctx->cfg.max_workspaces;
    out->requests = e.requests;
    out->coalesced_requests = e.coalesced;
    out->coalesced_launches = e.launches;
    out->outstanding_bytes = e.outstanding.load(std::memory_order_relaxed);
    out->waits = e.waits;
    out->direct_requests = e.direct;
    out->placed_bytes = e.placed_bytes;
    out->peak_outstanding_bytes = e.peak_outstanding;
    out->host_read_requests = e.host_reads;
    out->sleeps = e.sleeps.load(std::memory_order_relaxed);
    return RDX_OK;
}

}  // extern "C"
