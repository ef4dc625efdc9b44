// Device building blocks shared by the gfx950 kernels: element fetch (plain / fused byte-unshuffle,
// optional byte-order swap), the missing-data predicate, the reduction state of each operation and
// the deterministic cross-workgroup finalisation.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <limits>
#include <type_traits>

#include "../../include/rdx.h"
#include "rdx_kdesc.h"

namespace rdx {

template <typename T> struct UIntOf;
template <> struct UIntOf<int32_t> { using type = uint32_t; };
template <> struct UIntOf<uint32_t> { using type = uint32_t; };
template <> struct UIntOf<float> { using type = uint32_t; };
template <> struct UIntOf<int64_t> { using type = uint64_t; };
template <> struct UIntOf<uint64_t> { using type = uint64_t; };
template <> struct UIntOf<double> { using type = uint64_t; };

template <typename T>
__device__ __forceinline__ T from_u(typename UIntOf<T>::type u) { return __builtin_bit_cast(T, u); }
template <typename T>
__device__ __forceinline__ typename UIntOf<T>::type to_u(T v) { return __builtin_bit_cast(typename UIntOf<T>::type, v); }

template <typename T>
__device__ __forceinline__ T from_bits64(uint64_t b) {
    using U = typename UIntOf<T>::type;
    return from_u<T>((U)b);
}

// Loads through the GLOBAL address space (global_load_*): generic pointers compile to flat_load_*,
// which the compiler can only drain with vmcnt(0)+lgkmcnt(0) and which serialise the stream.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ V gld(const void *p) {
    if constexpr (std::is_same_v<V, uint4>) {  // HIP_vector_type has no address-space copy ctor
        typedef const __attribute__((address_space(1))) u32x4_t GV;
        const u32x4_t v = *(GV *)(p);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        typedef const __attribute__((address_space(1))) V GV;
        return *(GV *)(p);
    }
}

// Streaming loads of chunk bytes that are read exactly once: non-temporal (`global_load … nt`), so
// the lines are not kept in L2 / Infinity Cache at the expense of the rest of the stream.  Measured
// on the C2 shape (tools/probe_ceiling.hip): 6.63 TB/s nt vs 6.04 TB/s default policy.
#ifndef RDX_NT_LOADS
#define RDX_NT_LOADS 1
#endif
template <typename V>
__device__ __forceinline__ V gld_stream(const void *p) {
#if RDX_NT_LOADS
    if constexpr (std::is_same_v<V, uint4>) {
        typedef const __attribute__((address_space(1))) u32x4_t GV;
        const u32x4_t v = __builtin_nontemporal_load((GV *)(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        typedef const __attribute__((address_space(1))) V GV;
        return __builtin_nontemporal_load((GV *)(p));
    }
#else
    return gld<V>(p);
#endif
}

template <typename V>
__device__ __forceinline__ void gst(void *p, V v) {
    if constexpr (std::is_same_v<V, uint4>) {
        typedef __attribute__((address_space(1))) u32x4_t GV;
        u32x4_t w = {v.x, v.y, v.z, v.w};
        *(GV *)(p) = w;
    } else {
        typedef __attribute__((address_space(1))) V GV;
        *(GV *)(p) = v;
    }
}

__device__ __forceinline__ uint32_t bswap_u(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap_u(uint64_t x) { return __builtin_bswap64(x); }

// Magic-number division of a 32-bit index (rdx_plan.cpp make_div).
__device__ __forceinline__ uint32_t udiv(uint32_t n, uint64_t magic) {
    return magic ? (uint32_t)__umul64hi((uint64_t)n, magic) : n;
}

__device__ __forceinline__ const uint8_t *chunk_base(const KSrc &s, uint32_t chunk) {
    return s.ptrs ? gld<const uint8_t *>(s.ptrs + chunk) : s.base;
}

// One element by index e.  FUSED: byte k of element e is base[k*plane + e] (the inverse of
// src/filters/shuffle.rs:32-83 evaluated on the fly); bswap: array.rs:147-154.
template <typename T, bool FUSED>
__device__ __forceinline__ T load_elem(const uint8_t *base, uint64_t plane, bool bswap, uint64_t e) {
    using U = typename UIntOf<T>::type;
    U u;
    if constexpr (FUSED) {
        u = 0;
#pragma unroll
        for (int k = 0; k < (int)sizeof(T); ++k) u |= (U)gld<uint8_t>(base + (uint64_t)k * plane + e) << (8 * k);
    } else {
        u = gld<U>(reinterpret_cast<const U *>(base) + e);
    }
    if (bswap) u = bswap_u(u);
    return from_u<T>(u);
}

// Two-phase loads for gathers: a lane first issues the raw loads of all its kU vectors (offsets
// clamped into the view, so no load sits in a branch), then converts and consumes them.  A
// conversion placed right after a conditional load makes the compiler wait for that load, which
// serialises the lane's loads into kU round trips.
template <typename T, bool FUSED, int VW>
struct Raw {
    using U = typename UIntOf<T>::type;
    static constexpr int kBytes = VW * (int)sizeof(T);
    // VW > 1: one 8- or 16-byte load; VW == 1: one element (fused: its bytes from the planes)
    using V = std::conditional_t<kBytes == 16, uint4, std::conditional_t<kBytes == 8, uint64_t, U>>;
    V w;
    uint32_t b[FUSED ? sizeof(T) : 1];
};

template <typename T, bool FUSED, int VW>
__device__ __forceinline__ void raw_load(Raw<T, FUSED, VW> &r, const uint8_t *base, uint64_t plane, uint64_t off) {
    using V = typename Raw<T, FUSED, VW>::V;
    if constexpr (FUSED) {
        static_assert(VW == 1, "fused loads are per element");
#pragma unroll
        for (int k = 0; k < (int)sizeof(T); ++k) r.b[k] = gld<uint8_t>(base + (uint64_t)k * plane + off);
    } else if constexpr (VW > 1) {
        r.w = gld_stream<V>(base + off * sizeof(T));  // a contiguous 8/16 B run, read once
    } else {
        r.w = gld<V>(base + off * sizeof(T));
    }
}

// The loaded registers "used" in place (an empty asm): a load whose value is consumed only under a condition
// (a clamped row past the slice end) is otherwise sunk into that condition's block by the compiler, where it
// issues after the earlier loads' values came back and waits on all of them (k_axis_cols: two round trips
// per pass instead of one).
template <typename T, bool FUSED, int VW>
__device__ __forceinline__ void raw_pin(Raw<T, FUSED, VW> &r) {
    if constexpr (FUSED) {
#pragma unroll
        for (int k = 0; k < (int)sizeof(T); ++k) asm volatile("" : "+v"(r.b[k]));
    } else if constexpr (sizeof(r.w) == 16) {
        asm volatile("" : "+v"(r.w.x), "+v"(r.w.y), "+v"(r.w.z), "+v"(r.w.w));
    } else {
        asm volatile("" : "+v"(r.w));
    }
}

template <typename T, bool FUSED, int VW>
__device__ __forceinline__ void raw_cvt(const Raw<T, FUSED, VW> &r, bool bswap, T (&x)[VW]) {
    using U = typename UIntOf<T>::type;
    U e[VW];
    if constexpr (FUSED) {
        U u = 0;
#pragma unroll
        for (int k = 0; k < (int)sizeof(T); ++k) u |= (U)(r.b[k] & 0xffu) << (8 * k);
        e[0] = u;
    } else {
        __builtin_memcpy(e, &r.w, sizeof(e));
    }
#pragma unroll
    for (int j = 0; j < VW; ++j) x[j] = from_u<T>(bswap ? bswap_u(e[j]) : e[j]);
}

// ---- missing-data predicate ---------------------------------------------------------------------
// Missing::is_missing (src/types/missing.rs:114-122).
template <typename T>
__device__ __forceinline__ bool is_missing(const KMissing &m, T x) {
    switch (m.kind) {
        case RDX_MISSING_VALUE: return x == from_bits64<T>(m.v0);
        case RDX_MISSING_VALUES: {
            if (m.n & 0x80000000u) {  // sorted device list: binary search (Vec::contains semantics)
                uint32_t lo = 0, hi = m.n & 0x7fffffffu;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (from_bits64<T>(m.list[mid]) < x) lo = mid + 1;
                    else hi = mid;
                }
                return lo < (m.n & 0x7fffffffu) && from_bits64<T>(m.list[lo]) == x;
            }
            bool hit = false;
            for (uint32_t i = 0; i < m.n; ++i) hit |= x == from_bits64<T>(m.inl[i]);
            return hit;
        }
        case RDX_MISSING_VALID_MIN: return x < from_bits64<T>(m.v0);
        case RDX_MISSING_VALID_MAX: return x > from_bits64<T>(m.v0);
        case RDX_MISSING_VALID_RANGE: return x < from_bits64<T>(m.v0) || x > from_bits64<T>(m.v1);
        default: return false;
    }
}

// Included in the operation?  fold semantics: !is_missing (operations.rs:227-241 etc.);
// filter semantics: missing_filter (operations.rs:25-33, used by Count(All) and Select's count),
// which differs only for NaN under valid_min/valid_max/valid_range (NaN >= min is false).
template <typename T>
__device__ __forceinline__ bool included(const KMissing &m, T x, bool filter_semantics) {
    bool inc = !is_missing(m, x);
    if constexpr (std::is_floating_point_v<T>) {
        if (filter_semantics && m.kind >= RDX_MISSING_VALID_MIN) inc = inc && (x == x);
    }
    return inc;
}

// The predicate specialised at compile time by the kernels' MK parameter:
//   MK 0: no missing data;  MK 1: one comparison form (missing_value / valid_min / valid_max /
//   valid_range) evaluated branch-free from wave-uniform flags;  MK 2: anything (missing_values lists).
// Small kernels pay for code size (a cold instruction cache per CU): the generic switch of
// `included` in every element loop cost ~1.2 us of a 10 us C3 launch.
enum MissKind : int { MK_NONE = 0, MK_CMP = 1, MK_ANY = 2 };

template <typename T, int MK>
__device__ __forceinline__ bool included_mk(const KMissing &m, T x, bool filter_semantics) {
    if constexpr (MK == MK_NONE) {
        return true;
    } else if constexpr (MK == MK_ANY) {
        return included(m, x, filter_semantics);
    } else {
        const uint32_t k = m.kind;
        const T a = from_bits64<T>(m.v0), b = from_bits64<T>(m.v1);
        const bool eq_on = k == RDX_MISSING_VALUE;
        const bool lo_on = k == RDX_MISSING_VALID_MIN || k == RDX_MISSING_VALID_RANGE;
        const bool hi_on = k == RDX_MISSING_VALID_MAX || k == RDX_MISSING_VALID_RANGE;
        const T hi = k == RDX_MISSING_VALID_MAX ? a : b;
        const bool missing = (eq_on & (x == a)) | (lo_on & (x < a)) | (hi_on & (x > hi));
        bool inc = !missing;
        if constexpr (std::is_floating_point_v<T>) inc = inc & !(filter_semantics & (lo_on | hi_on) & (x != x));
        return inc;
    }
}

__host__ __device__ inline int miss_kind_of(uint32_t kind) {
    return kind == RDX_MISSING_NONE ? MK_NONE : kind == RDX_MISSING_VALUES ? MK_ANY : MK_CMP;
}

// ---- reduction state ------------------------------------------------------------------------------
// SUM:   integers wrap (release profile) — accumulated in u64 and truncated to T;
//        f32 accumulated in f64 and rounded once; f64 Neumaier-compensated (operations.rs:622-632
//        sums sequentially in T: results agree exactly for exactly-summable data and within the
//        tolerance stated in DESIGN.md otherwise).
// MAX/MIN: identity T::min_value()/max_value() (f32::MIN, not -inf), NaN -> RDX_E_NAN_UNORDERED,
//        ±0 ties resolved by the fold-order rank of the zeros (max_by keeps the LAST equal element,
//        min_by the FIRST; operations.rs:229-241,459-469).
template <typename T, int OP>
struct Red {
    static constexpr bool kFloat = std::is_floating_point_v<T>;
    static constexpr bool kRank = kFloat && (OP == OP_MAX || OP == OP_MIN);
    double s, c;
    uint64_t si;
    T v;
    int64_t cnt;
    int64_t zp, zn;
    uint32_t nan;

    __device__ __forceinline__ void init() {
        s = 0.0;
        c = 0.0;
        si = 0;
        v = OP == OP_MAX ? std::numeric_limits<T>::lowest() : std::numeric_limits<T>::max();
        cnt = 0;
        zp = zn = OP == OP_MAX ? -1 : INT64_MAX;
        nan = 0;
    }

    __device__ __forceinline__ static void neumaier(double &s_, double &c_, double x) {
        const double t = s_ + x;
        if (fabs(s_) >= fabs(x)) c_ += (s_ - t) + x;
        else c_ += (x - t) + s_;
        s_ = t;
    }
    // Knuth's TwoSum: a + b = s + e exactly (branch-free, 6 flops)
    __device__ __forceinline__ static double two_sum(double a, double b, double &e) {
        const double s_ = a + b, bb = s_ - a;
        e = (a - (s_ - bb)) + (b - bb);
        return s_;
    }
    // A group of elements added pairwise with every rounding error kept (TwoSum), then one compensated
    // add: the same result class as a Neumaier step per element (e.g. [1e16, 1, -1e16, 1] sums to 2,
    // exactly), a quarter of the dependent steps.
    __device__ __forceinline__ static void add4(double &s_, double &c_, double x0, double x1, double x2, double x3) {
        double e0, e1, e2;
        const double p = two_sum(x0, x1, e0), q = two_sum(x2, x3, e1);
        neumaier(s_, c_, two_sum(p, q, e2));
        c_ += (e0 + e1) + e2;
    }
    __device__ __forceinline__ static void add2(double &s_, double &c_, double x0, double x1) {
        double e0;
        neumaier(s_, c_, two_sum(x0, x1, e0));
        c_ += e0;
    }

    // value only (count handled by caller for batched adds)
    template <class RankFn>
    __device__ __forceinline__ void add_value(T x, RankFn &&rank) {
        if constexpr (OP == OP_SUM) {
            if constexpr (kFloat) {
                if constexpr (sizeof(T) == 4) s += (double)x;
                else neumaier(s, c, (double)x);
            } else {
                si += (uint64_t)x;
            }
        } else if constexpr (OP == OP_MAX || OP == OP_MIN) {
            if constexpr (kFloat) {
                nan |= (x != x);
                // ±0 fold-order ranks behind a wave-uniform branch: without it the compiler
                // if-converts the zero case and every element pays a 64-bit rank and two selects.
                if (__builtin_amdgcn_ballot_w64(x == T(0))) {
                    if (x == T(0)) {
                        const int64_t r = rank();
                        if (__builtin_signbit(x)) zn = OP == OP_MAX ? max(zn, r) : min(zn, r);
                        else zp = OP == OP_MAX ? max(zp, r) : min(zp, r);
                    }
                }
                // order-free value fold: a NaN operand leaves v unchanged (and sets the error flag);
                // a zero's sign is decided from the ranks in value()
                if constexpr (OP == OP_MAX) v = __builtin_fmax(v, x);
                else v = __builtin_fmin(v, x);
            } else {
                if constexpr (OP == OP_MAX) v = x > v ? x : v;
                else v = x < v ? x : v;
            }
        }
    }

    template <class RankFn>
    __device__ __forceinline__ void add(T x, RankFn &&rank) {
        add_value(x, rank);
        cnt += 1;
    }

    __device__ __forceinline__ void merge(const Red &o) {
        if constexpr (OP == OP_SUM) {
            if constexpr (kFloat) {
                if constexpr (sizeof(T) == 4) {
                    s += o.s;
                } else {
                    neumaier(s, c, o.s);
                    c += o.c;
                }
            } else {
                si += o.si;
            }
        } else if constexpr (OP == OP_MAX) {
            v = o.v > v ? o.v : v;
        } else if constexpr (OP == OP_MIN) {
            v = o.v < v ? o.v : v;
        }
        if constexpr (kRank) {
            zp = OP == OP_MAX ? max(zp, o.zp) : min(zp, o.zp);
            zn = OP == OP_MAX ? max(zn, o.zn) : min(zn, o.zn);
            nan |= o.nan;
        }
        cnt += o.cnt;
    }

    __device__ __forceinline__ T value() const {
        if constexpr (OP == OP_SUM) {
            if constexpr (kFloat) {
                if constexpr (sizeof(T) == 4) return (T)s;
                else return __builtin_isfinite(s) ? s + c : s;
            } else {
                return (T)si;
            }
        } else {
            T r = v;
            if constexpr (kRank) {
                if (r == T(0)) {
                    const bool neg = OP == OP_MAX ? (zn > zp) : (zn < zp);
                    r = neg ? -T(0) : T(0);
                }
            }
            return r;
        }
    }

    __device__ __forceinline__ void to_words(uint64_t w[kPartialWords]) const {
        w[0] = OP == OP_SUM ? (kFloat ? __builtin_bit_cast(uint64_t, s) : si) : (uint64_t)to_u<T>(v);
        w[1] = __builtin_bit_cast(uint64_t, c);
        w[2] = (uint64_t)cnt;
        w[3] = (uint64_t)zp;
        w[4] = (uint64_t)zn;
        w[5] = nan;
    }
    __device__ __forceinline__ void from_words(const uint64_t w[kPartialWords]) {
        init();
        if constexpr (OP == OP_SUM) {
            if constexpr (kFloat) s = __builtin_bit_cast(double, w[0]);
            else si = w[0];
        } else {
            v = from_bits64<T>(w[0]);
        }
        c = __builtin_bit_cast(double, w[1]);
        cnt = (int64_t)w[2];
        zp = (int64_t)w[3];
        zn = (int64_t)w[4];
        nan = (uint32_t)w[5];
    }
};

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
    const int lo = __shfl_xor((int)(uint32_t)x, m, 64);
    const int hi = __shfl_xor((int)(uint32_t)(x >> 32), m, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Which of the kPartialWords a reduction state actually carries (the rest stay at their identity).
template <typename T, int OP>
__device__ __forceinline__ constexpr bool word_used(int i) {
    constexpr bool kRank = Red<T, OP>::kRank;
    switch (i) {
        case 0: return OP != OP_COUNT;                                              // value / sum
        case 1: return OP == OP_SUM && std::is_same_v<T, double>;                   // compensation
        case 2: return true;                                                        // count
        default: return kRank;                                                      // zero ranks, NaN flag
    }
}

// Partial records in memory carry only the used words, packed (f32 sum: 2 words, float min/max: 5).
template <typename T, int OP>
__device__ __forceinline__ constexpr int packed_words() {
    int n = 0;
    for (int i = 0; i < kPartialWords; ++i) n += word_used<T, OP>(i) ? 1 : 0;
    return n;
}

// ---- cross-workgroup hand-off records ----------------------------------------------------------------
// A partial record published to another workgroup of the same launch travels as tagged granules: 8-byte
// words {48-bit payload, 16-bit launch epoch}, each written by ONE relaxed agent-scope atomic store
// (global_store sc1, write-through) and read back by relaxed agent-scope atomic loads (sc1:
// device-coherent, never served from a stale L1 copy) that retry until the granule carries this
// launch's epoch.  Every access to a record is atomic (no data race) and a reader accepts exactly the
// value this launch's producer stored (single-copy atomicity of an aligned 8-byte atomic), so the HIP
// memory model needs no release/acquire pair for the record bytes: the arrival counters (relaxed RMWs,
// totally ordered per location) only elect the workgroup that folds.  Measured against the fence form
// (release before the counter add, acquire in the last arriver; profiles/r02_handoff_ab.jsonl): the
// fences cost +1.5 us per 64 MiB single-chunk launch, +3 us per batched launch and +29 us on the
// sliced axis kernels (every slice's buffer_wbl2).  Epochs come from the workspace (rdx_runtime.cpp
// next_epoch): never 0, and the record buffer is cleared whenever the 16-bit epoch wraps, so a stale
// granule can never carry the current tag.  A reader that sees no fresh granule within kSpinLimit polls
// (a producer that never published: impossible short of a device fault) gives up and reports
// RDX_E_DEVICE instead of hanging the GPU.
//
// Record fields -> granules: a 64-bit value / sum / compensation as two 32-bit halves; a 32-bit min/max
// value as one; the count (< 2^47) with the NaN flag in bit 47 as one; each ±0 fold-order rank (48-bit
// two's complement, INT64_MAX as 0x7fff_ffff_ffff) as one.  Sums carry the count (< 2^32: the planner
// refuses views of 2^32 elements or more) in the spare 16 bits of their two sum halves instead of a
// granule of its own.  f32 / integer sum: 2 granules (16 B), f32 min/max: 4, f64 sum: 4, f64 min/max: 5,
// count: 1.
// Phase timeline of the all-axes kernels (probe builds only, make EXTRA=-DRDX_PROBES=1): per workgroup
// [0] first instruction, [1] streaming done, [2] record published + counter added, [3] fold done (last
// arriver), in wall-clock ticks (100 MHz); [4] the HW_ID register at the start (CU / SH / SE placement).
// Read back by rdx_probe_read_<dtype> (k_all.hip).
#if RDX_PROBES
static __device__ uint64_t g_rdx_probe[8 * 8192];
#define RDX_STAMP(slot)                                                                              \
    do {                                                                                             \
        if (threadIdx.x == 0 && blockIdx.x < 8192) {                                                 \
            g_rdx_probe[8 * blockIdx.x + (slot)] = wall_clock64();                                   \
            if ((slot) == 0) g_rdx_probe[8 * blockIdx.x + 4] = __builtin_amdgcn_s_getreg(4 | (31 << 11)); \
        }                                                                                            \
    } while (0)
#else
#define RDX_STAMP(slot) \
    do {                \
    } while (0)
#endif

#if RDX_PROBES
constexpr uint32_t kSpinLimit = 1u << 12;   // probe builds: a missing record surfaces as RDX_E_DEVICE quickly
#else
constexpr uint32_t kSpinLimit = 1u << 22;
#endif
constexpr uint64_t kPayload = (1ull << 48) - 1;
constexpr int kMaxGranules = 6;

__device__ __forceinline__ void put_granule(uint64_t *g, uint64_t payload, uint32_t tag) {
    __hip_atomic_store(g, (payload & kPayload) | ((uint64_t)tag << 48), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Cold path: poll one granule until it carries `tag`; after kSpinLimit polls it returns the stale value
// and the caller reports a fault.
__device__ __attribute__((noinline)) uint64_t poll_granule(const uint64_t *g, uint32_t tag) {
    uint64_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = 0; (uint32_t)(v >> 48) != tag && i < kSpinLimit; ++i) {
        __builtin_amdgcn_s_sleep(1);
        v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return v;
}

template <typename T, int OP>
__device__ __forceinline__ constexpr int granules() {
    constexpr bool kRank = Red<T, OP>::kRank;
    if (OP == OP_SUM) return std::is_same_v<T, double> ? 4 : 2;          // sum (+ compensation), count packed
    int n = 0;
    if (OP != OP_COUNT) n += sizeof(T) == 8 ? 2 : 1;                      // value
    n += 1;                                                               // count (+ NaN flag)
    if (kRank) n += 2;                                                    // ±0 ranks
    return n;
}

__device__ __forceinline__ uint64_t rank48(int64_t r) {
    return r == INT64_MAX ? 0x7fffffffffffull : (uint64_t)r & kPayload;
}
__device__ __forceinline__ int64_t unrank48(uint64_t p) {
    p &= kPayload;
    if (p == 0x7fffffffffffull) return INT64_MAX;
    return (int64_t)(p << 16) >> 16;
}

template <typename T, int OP>
__device__ __forceinline__ void encode(const Red<T, OP> &r, uint64_t (&g)[kMaxGranules]) {
    uint64_t w[kPartialWords];
    r.to_words(w);
    if constexpr (OP == OP_SUM) {   // {sum lo32, count lo16}, {sum hi32, count hi16} [, compensation]
        g[0] = (w[0] & 0xffffffffull) | (w[2] & 0xffffull) << 32;
        g[1] = (w[0] >> 32) | ((w[2] >> 16) & 0xffffull) << 32;
        if constexpr (std::is_same_v<T, double>) {
            g[2] = w[1] & 0xffffffffull;
            g[3] = w[1] >> 32;
        }
        return;
    }
    int k = 0;
    if constexpr (OP != OP_COUNT) {
        if constexpr (sizeof(T) == 8) {
            g[k++] = w[0] & 0xffffffffull;
            g[k++] = w[0] >> 32;
        } else {
            g[k++] = w[0] & 0xffffffffull;
        }
    }
    g[k++] = (w[2] & ((1ull << 47) - 1)) | (Red<T, OP>::kRank && w[5] ? (1ull << 47) : 0ull);
    if constexpr (Red<T, OP>::kRank) {
        g[k++] = rank48((int64_t)w[3]);
        g[k++] = rank48((int64_t)w[4]);
    }
}

template <typename T, int OP>
__device__ __forceinline__ void decode(const uint64_t (&g)[kMaxGranules], Red<T, OP> &r) {
    Red<T, OP> id;
    id.init();
    uint64_t w[kPartialWords];
    id.to_words(w);
    if constexpr (OP == OP_SUM) {
        w[0] = (g[0] & 0xffffffffull) | (g[1] & 0xffffffffull) << 32;
        w[2] = ((g[0] >> 32) & 0xffffull) | ((g[1] >> 32) & 0xffffull) << 16;
        if constexpr (std::is_same_v<T, double>) w[1] = (g[2] & 0xffffffffull) | (g[3] & 0xffffffffull) << 32;
        r.from_words(w);
        return;
    }
    int k = 0;
    if constexpr (OP != OP_COUNT) {
        if constexpr (sizeof(T) == 8) {
            w[0] = (g[k] & 0xffffffffull) | ((g[k + 1] & 0xffffffffull) << 32);
            k += 2;
        } else {
            w[0] = g[k++] & 0xffffffffull;
        }
    }
    w[2] = g[k] & ((1ull << 47) - 1);
    if constexpr (Red<T, OP>::kRank) {
        w[5] = (g[k] >> 47) & 1;
        w[3] = (uint64_t)unrank48(g[k + 1]);
        w[4] = (uint64_t)unrank48(g[k + 2]);
    }
    r.from_words(w);
}

// Granule j of a record at P[j * stride] (stride 1 = record-major; a word-major record array, stride =
// record count, makes a wave's per-lane stores / loads of one granule coalesced).
template <typename T, int OP>
__device__ __forceinline__ void publish(uint64_t *P, const Red<T, OP> &r, uint32_t tag, uint64_t stride = 1) {
    uint64_t g[kMaxGranules];
    encode(r, g);
#pragma unroll
    for (int j = 0; j < granules<T, OP>(); ++j) put_granule(P + j * stride, g[j], tag);
}

// collect() in two halves, so that a folder can have several records' loads in flight before it waits
// on the first: load_record issues the granule loads, accept_record checks their tags (polling a stale
// one) and decodes.
template <typename T, int OP>
__device__ __forceinline__ void load_record(const uint64_t *P, uint64_t (&g)[kMaxGranules], uint64_t stride = 1) {
#pragma unroll
    for (int j = 0; j < granules<T, OP>(); ++j)
        g[j] = __hip_atomic_load(P + j * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, int OP>
__device__ __forceinline__ void accept_record(const uint64_t *P, uint64_t (&g)[kMaxGranules], Red<T, OP> &r,
                                              uint32_t tag, uint32_t &fault, uint64_t stride = 1) {
    constexpr int kG = granules<T, OP>();
    bool fresh = true;
#pragma unroll
    for (int j = 0; j < kG; ++j) fresh &= (uint32_t)(g[j] >> 48) == tag;
    if (__builtin_expect(!fresh, 0)) {
#pragma unroll
        for (int j = 0; j < kG; ++j)
            if ((uint32_t)(g[j] >> 48) != tag) {
                // one spin budget per lane: after a granule timed out, a faulted launch does not poll again
                // (so many missing records cost one kSpinLimit period, not one each)
                if (!fault) g[j] = poll_granule(P + j * stride, tag);
                fault |= (uint32_t)(g[j] >> 48) != tag;
            }
    }
    decode(g, r);
}

template <typename T, int OP>
__device__ __forceinline__ void collect(const uint64_t *P, Red<T, OP> &r, uint32_t tag, uint32_t &fault,
                                        uint64_t stride = 1) {
    constexpr int kG = granules<T, OP>();
    uint64_t g[kMaxGranules] = {};
#pragma unroll
    for (int j = 0; j < kG; ++j) g[j] = __hip_atomic_load(P + j * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool fresh = true;
#pragma unroll
    for (int j = 0; j < kG; ++j) fresh &= (uint32_t)(g[j] >> 48) == tag;
    if (__builtin_expect(!fresh, 0)) {
#pragma unroll
        for (int j = 0; j < kG; ++j)
            if ((uint32_t)(g[j] >> 48) != tag) {
                if (!fault) g[j] = poll_granule(P + j * stride, tag);   // (one spin budget per lane)
                fault |= (uint32_t)(g[j] >> 48) != tag;
            }
    }
    decode(g, r);
}

// Plain (untagged) packed records: within a workgroup (LDS) or read by a LATER launch (the kernel
// boundary orders them).  Word k of the record at P[k * stride].
template <typename T, int OP>
__device__ __forceinline__ void store_packed(uint64_t *P, const Red<T, OP> &r, uint64_t stride = 1) {
    uint64_t w[kPartialWords];
    r.to_words(w);
    int k = 0;
#pragma unroll
    for (int i = 0; i < kPartialWords; ++i) {
        if (!word_used<T, OP>(i)) continue;
        P[k * stride] = w[i];
        ++k;
    }
}

template <typename T, int OP>
__device__ __forceinline__ void load_packed(const uint64_t *P, Red<T, OP> &r, uint64_t stride = 1) {
    Red<T, OP> id;
    id.init();
    uint64_t w[kPartialWords];
    id.to_words(w);
    int k = 0;
#pragma unroll
    for (int i = 0; i < kPartialWords; ++i) {
        if (!word_used<T, OP>(i)) continue;
        w[i] = P[k * stride];
        ++k;
    }
    r.from_words(w);
}

template <typename T, int OP>
__device__ __forceinline__ void xor_merge(Red<T, OP> &r, int m) {
    uint64_t w[kPartialWords], o[kPartialWords];
    r.to_words(w);
#pragma unroll
    for (int i = 0; i < kPartialWords; ++i) o[i] = word_used<T, OP>(i) ? shfl_xor_u64(w[i], m) : w[i];
    Red<T, OP> other;
    other.from_words(o);
    r.merge(other);
}

// Float min/max without a zero in the wave: only the value, count and NaN words move (the ±0 ranks
// stay at their identity in every lane, so merging them is a no-op).
template <typename T, int OP>
__device__ __forceinline__ void xor_merge_noranks(Red<T, OP> &r, int m) {
    uint64_t w[kPartialWords], o[kPartialWords];
    r.to_words(w);
#pragma unroll
    for (int i = 0; i < kPartialWords; ++i) o[i] = (i == 0 || i == 2 || i == 5) ? shfl_xor_u64(w[i], m) : w[i];
    Red<T, OP> other;
    other.from_words(o);
    r.merge(other);
}

// Deterministic butterfly over the 64 lanes; every lane ends with the wave total.
template <typename T, int OP>
__device__ __forceinline__ void wave_reduce(Red<T, OP> &r) {
    if constexpr (Red<T, OP>::kRank) {
        const int64_t id = OP == OP_MAX ? -1 : INT64_MAX;
        if (!__builtin_amdgcn_ballot_w64(r.zp != id || r.zn != id)) {   // wave-uniform: no zero seen
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) xor_merge_noranks(r, m);
            return;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) xor_merge(r, m);
}

// The same within aligned groups of `width` lanes (a power of two <= 64).
template <typename T, int OP>
__device__ __forceinline__ void group_reduce(Red<T, OP> &r, uint32_t width) {
    for (int m = (int)width >> 1; m >= 1; m >>= 1) xor_merge(r, m);
}

// Workgroup total in thread 0 (waves merged in wave order).
template <typename T, int OP>
__device__ __forceinline__ void block_reduce(Red<T, OP> &r) {
    __shared__ uint64_t lds[kBlock / 64][kPartialWords];
    wave_reduce(r);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        uint64_t w[kPartialWords];
        r.to_words(w);
#pragma unroll
        for (int i = 0; i < kPartialWords; ++i) lds[wave][i] = w[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kBlock / 64; ++k) {
            Red<T, OP> o;
            o.from_words(lds[k]);
            r.merge(o);
        }
    }
    __syncthreads();
}

// Arrival counting of the cross-workgroup hand-off: after publishing its record(s) (tagged granules,
// above) one lane of each workgroup adds to an arrival counter; the workgroup whose add completes the
// count collects every record.  The counter is sharded 8 ways by workgroup index
// (b % 8 groups share an XCD under round-robin dispatch) so that arrivals do not serialise on one word
// (~11 ns per atomic, MI355X_MICROARCH.md "fanin" row); the last arrival of each shard adds to the top
// counter.  All counters self-reset for the next launch.
__device__ __forceinline__ bool arrive_last(uint32_t *tk, uint32_t n, uint32_t b) {
    const uint32_t nsh = n < kTicketShards ? n : kTicketShards;
    const uint32_t sh = b % kTicketShards;
    const uint32_t members = (n - sh + kTicketShards - 1) / kTicketShards;
    const uint32_t p1 = __hip_atomic_fetch_add(tk + (1 + sh) * kTicketStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p1 != members - 1) return false;
    __hip_atomic_store(tk + (1 + sh) * kTicketStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1;
}

// A chunk's response as 3 tagged granules in a page-locked host slot (KOut::host_slots): the host polls
// them for this launch's tag, as the in-launch hand-off does (no fence, no end-of-kernel flush in the way:
// the caller sees its result as soon as the fold's stores cross the link).  {value lo32}, {value hi32},
// {count (< 2^40) | status << 40}, each with the epoch in bits 48-63; system-scope vector stores.
__device__ __forceinline__ void put_host_slot(uint64_t *slot, uint64_t value, int64_t count, uint32_t status,
                                              uint32_t tag) {
    const uint64_t t = (uint64_t)tag << 48;
    __hip_atomic_store(slot + 0, (value & 0xffffffffull) | t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot + 1, (value >> 32) | t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(slot + 2, ((uint64_t)count & ((1ull << 40) - 1)) | ((uint64_t)(status & 0xffu) << 40) | t,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T, int OP>
__device__ __forceinline__ void write_folded(const KOut &out, uint32_t chunk, const Red<T, OP> &acc, bool fault);
constexpr int kWaveFold = 6;   // records per lane of a wave-0 fold (nrec <= 384)

// The hand-off's second half: this workgroup's records are published; elect the folder and let it fold
// records P[0 .. nrec) in index order (deterministic) and write the chunk's response.
//   fold_last == 0: count the arrival (8-way sharded counters, `members` workgroups per chunk); the last
//     to arrive folds.  Costs two dependent atomic round trips per workgroup (~1.1 us each under load).
//   fold_last == 1: the chunk's last block (b == members - 1) folds, polling each record until it carries
//     this launch's tag; every other block publishes and exits.  Workgroups are dispatched in index order
//     (per XCD), so every block the folder waits on was dispatched before it and runs to completion
//     without waiting on anything; the host uses this form only for launches of <= kFoldLastChunks
//     folders, far fewer than one XCD's workgroup slots, so folders can never fill an XCD and keep a
//     lower-index block of their own chunk from being dispatched.  A record that never
//     arrives (a device fault) still ends in RDX_E_DEVICE after kSpinLimit polls, never in a hang.
template <typename T, int OP>
__device__ void arrive_and_fold(const KOut &out, const uint64_t *P, uint32_t chunk, uint32_t members, uint32_t nrec,
                                uint32_t b) {
    __shared__ uint32_t s_last, s_fault;
    constexpr int kR = granules<T, OP>();   // u64 granules per record
    if (threadIdx.x == 0) {
        s_last = out.fold_last ? (b == members - 1) : arrive_last(out.tickets + (uint64_t)chunk * kTicketWords, members, b);
        s_fault = 0;
    }
    RDX_STAMP(2);
    __syncthreads();
    if (!s_last) return;
    Red<T, OP> acc;
    acc.init();
    uint32_t fault = 0;
    if (nrec <= 64 * kWaveFold) {
        // Up to 384 records (C1: 128, C3: 336): wave 0 alone folds them — lane l merges records l, l + 64,
        // ... (all of its loads in flight at once: one round trip), then the wave butterfly; no LDS, no
        // workgroup barrier on the folder's critical path
        if (threadIdx.x >= 64) return;
        uint64_t g[kWaveFold][kMaxGranules];
#pragma unroll
        for (int u = 0; u < kWaveFold; ++u) {
            const uint32_t j = threadIdx.x + 64u * u;
            if (j < nrec) load_record<T, OP>(P + (uint64_t)j * kR, g[u]);
        }
        // Records not yet visible (the folder's own streaming often ends before the last publisher's): every
        // stale granule of the wave is re-read in the same round — one round trip per retry for all of
        // them, not one per granule in turn — until all carry the tag or the spin budget is spent.
        for (uint32_t it = 0;; ++it) {
            bool stale = false;
#pragma unroll
            for (int u = 0; u < kWaveFold; ++u) {
                const bool live = threadIdx.x + 64u * u < nrec;
#pragma unroll
                for (int q = 0; q < kR; ++q) stale |= live && (uint32_t)(g[u][q] >> 48) != out.epoch;
            }
            if (!__builtin_amdgcn_ballot_w64(stale)) break;
            if (it >= kSpinLimit) {
                fault = stale ? 1u : 0u;
                break;
            }
            // backing off: a folder whose publishers are far from done (a batch launch that fills the chip)
            // must not flood the fabric with re-reads while they stream.  (RDX_FOLD_POLL_SHORT=1: ~0.1 us sleeps
            // for the few folders of a fold_last launch — measured no better: C3 7.98 -> 8.22 us, C1 within
            // noise, profiles/r05_fold_poll_ab.jsonl)
#ifndef RDX_FOLD_POLL_SHORT
#define RDX_FOLD_POLL_SHORT 0
#endif
            if (RDX_FOLD_POLL_SHORT && out.fold_last) {
                if (it < 8) __builtin_amdgcn_s_sleep(1);
                else __builtin_amdgcn_s_sleep(4);
            } else if (it < 2) __builtin_amdgcn_s_sleep(1);
            else if (it < 6) __builtin_amdgcn_s_sleep(8);
            else __builtin_amdgcn_s_sleep(32);
#pragma unroll
            for (int u = 0; u < kWaveFold; ++u) {
                const uint32_t j = threadIdx.x + 64u * u;
#pragma unroll
                for (int q = 0; q < kR; ++q)
                    if (j < nrec && (uint32_t)(g[u][q] >> 48) != out.epoch)
                        g[u][q] = __hip_atomic_load(P + (uint64_t)j * kR + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int u = 0; u < kWaveFold; ++u) {
            const uint32_t j = threadIdx.x + 64u * u;
            if (j >= nrec) continue;
            Red<T, OP> o;
            decode<T, OP>(g[u], o);
            acc.merge(o);
        }
        wave_reduce(acc);
        const bool any_fault = __builtin_amdgcn_ballot_w64(fault != 0) != 0;
        if (threadIdx.x == 0) write_folded<T, OP>(out, chunk, acc, any_fault);
        RDX_STAMP(3);
        return;
    }
    // records j = tid, tid + 256, ... merged in that order; two in flight per thread, so up to 512
    // records cost one load round trip instead of one per 256
    for (uint32_t j0 = threadIdx.x; j0 < nrec; j0 += 2 * kBlock) {
        const uint32_t j1 = j0 + kBlock;
        uint64_t g0[kMaxGranules] = {}, g1[kMaxGranules] = {};
        load_record<T, OP>(P + (uint64_t)j0 * kR, g0);
        if (j1 < nrec) load_record<T, OP>(P + (uint64_t)j1 * kR, g1);
        Red<T, OP> o;
        accept_record<T, OP>(P + (uint64_t)j0 * kR, g0, o, out.epoch, fault);
        acc.merge(o);
        if (j1 < nrec) {
            accept_record<T, OP>(P + (uint64_t)j1 * kR, g1, o, out.epoch, fault);
            acc.merge(o);
        }
    }
    if (fault) s_fault = 1;   // benign race: every writer stores 1
    block_reduce(acc);
    if (threadIdx.x == 0) write_folded<T, OP>(out, chunk, acc, s_fault != 0);
    RDX_STAMP(3);
}

// The folded response of a chunk (thread 0 of the folder): its body / count / status, or its host slot.
template <typename T, int OP>
__device__ __forceinline__ void write_folded(const KOut &out, uint32_t chunk, const Red<T, OP> &acc, bool fault) {
    {
        uint32_t e = (Red<T, OP>::kRank && acc.nan) ? (uint32_t)RDX_E_NAN_UNORDERED : 0u;
        if (fault) e = RDX_E_DEVICE;
        if (out.host_slots) {
            const uint64_t v = OP == OP_COUNT ? (uint64_t)acc.cnt : (uint64_t)to_u<T>(acc.value());
            put_host_slot(reinterpret_cast<uint64_t *>(out.body) + 3 * (uint64_t)chunk, v, acc.cnt, e, out.epoch);
        } else {
            if constexpr (OP == OP_COUNT) {
                reinterpret_cast<int64_t *>(out.body + chunk * out.body_stride)[0] = acc.cnt;
            } else {
                reinterpret_cast<T *>(out.body + chunk * out.body_stride)[0] = acc.value();
            }
            out.counts[chunk * out.counts_stride] = acc.cnt;
            if (out.status) {
                if (!out.status_any) out.status[chunk] = e;
                else if (e) __hip_atomic_fetch_or(out.status, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (!Red<T, OP>::kRank && chunk == 0) out.status[0] = 0;   // nothing can fail
            }
        }
        if (!out.fold_last)
            __hip_atomic_store(out.tickets + (uint64_t)chunk * kTicketWords, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- order-free folds through device-scope atomics (KOut::fold_last == 2) ---------------------------------
// Count, integer sums (wrapping: u64 adds commute) and min / max of every dtype — the float ±0 tie ranks
// are a min / max of ranks and the NaN flag an OR, so they commute too — need no record per workgroup:
// each workgroup merges its partial into 8 per-XCD accumulator lines of the chunk (the arrival-counter
// lines of the ticket area, which fold-last launches leave unused) with no-return atomics, waits for
// their acknowledgement (`s_waitcnt vmcnt(0)`: on gfx9 no-return atomics stay counted until performed),
// then adds {count << 20 | 1} to its line — the arrival and the count in one word.  The chunk's last
// block polls the 8 count words (one load per lane of 8 lanes) until the other bpc - 1 arrivals are in,
// then takes every accumulator with an atomic exchange to 0 (the value it returns is final: each
// publisher's merge was performed before its arrival, and nobody else adds; the exchange also leaves the
// lines zeroed for the next launch).  Stored forms make 0 the identity of every word: a value as its
// order-preserving key (min: the key's complement, so both are atomic max), a ±0 rank likewise.
// Float sums keep the records: their fold order is part of the result.
template <typename T, int OP>
constexpr bool kAtomicFold = OP == OP_COUNT || OP == OP_MAX || OP == OP_MIN || (OP == OP_SUM && !std::is_floating_point_v<T>);

template <typename T>
__device__ __forceinline__ uint64_t okey(T v) {   // order-preserving unsigned key
    using U = typename UIntOf<T>::type;
    constexpr U kSign = (U)1 << (8 * sizeof(U) - 1);
    U u = to_u<T>(v);
    if constexpr (std::is_floating_point_v<T>) u = (u & kSign) ? (U)~u : (U)(u | kSign);
    else if constexpr (std::is_signed_v<T>) u ^= kSign;
    return (uint64_t)u;
}
template <typename T>
__device__ __forceinline__ T from_okey(uint64_t k) {
    using U = typename UIntOf<T>::type;
    constexpr U kSign = (U)1 << (8 * sizeof(U) - 1);
    U u = (U)k;
    if constexpr (std::is_floating_point_v<T>) u = (u & kSign) ? (U)(u & ~kSign) : (U)~u;
    else if constexpr (std::is_signed_v<T>) u ^= kSign;
    return from_u<T>(u);
}
template <typename T, int OP>
__device__ __forceinline__ uint64_t stored_value(T v) {   // 0 = identity; larger = further from it
    using U = typename UIntOf<T>::type;
    const uint64_t k = okey<T>(v);
    return OP == OP_MIN ? (uint64_t)(U)~(U)k : k;
}
template <typename T, int OP>
__device__ __forceinline__ T value_of_stored(uint64_t s) {
    using U = typename UIntOf<T>::type;
    return from_okey<T>(OP == OP_MIN ? (uint64_t)(U)~(U)s : s);
}
template <int OP>
__device__ __forceinline__ uint64_t stored_rank(int64_t r) {   // max keeps the largest rank, min the smallest
    const uint64_t k = (uint64_t)r ^ (1ull << 63);
    return OP == OP_MAX ? k : ~k;
}
template <int OP>
__device__ __forceinline__ int64_t rank_of_stored(uint64_t s) {   // 0 (nothing stored) -> the identity
    if (s == 0) return OP == OP_MAX ? -1 : INT64_MAX;
    return (int64_t)((OP == OP_MAX ? s : ~s) ^ (1ull << 63));
}

constexpr uint32_t kArriveBits = 20;   // {count << 20 | arrivals}: arrivals per line < 2^20, count < 2^44
constexpr uint32_t kDirtyWord = 48;    // u32 index in the chunk's ticket top line: set by a fold that timed out
// accumulator line of shard s (0..7) of the chunk: u64 words [0] count | arrivals, [1] value / sum,
// [2] +0 rank, [3] -0 rank, [4] NaN flag
__device__ __forceinline__ uint64_t *acc_line(const KOut &out, uint32_t chunk, uint32_t s) {
    return reinterpret_cast<uint64_t *>(out.tickets + (uint64_t)chunk * kTicketWords + (1 + s) * kTicketStride);
}

template <typename T, int OP>
__device__ void atomic_fold(const Red<T, OP> &r, const KOut &out, uint32_t chunk, uint32_t bpc, uint32_t b) {
    constexpr bool kRank = Red<T, OP>::kRank;
    const int64_t rid = OP == OP_MAX ? -1 : INT64_MAX;
#if RDX_PROBES
    const bool drop = out.drop_block == 1 + blockIdx.x;
#else
    constexpr bool drop = false;
#endif
    if (b != bpc - 1) {   // a publisher: merge, wait for the merges, arrive
        if (threadIdx.x == 0 && !drop) {
            uint64_t *L = acc_line(out, chunk, b % kTicketShards);
            bool merged = false;
            if constexpr (OP == OP_SUM) {
                __hip_atomic_fetch_add(L + 1, r.si, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                merged = true;
            } else if constexpr (OP != OP_COUNT) {
                if (r.cnt) {
                    __hip_atomic_fetch_max(L + 1, stored_value<T, OP>(r.v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    merged = true;
                }
                if constexpr (kRank) {
                    if (r.zp != rid) __hip_atomic_fetch_max(L + 2, stored_rank<OP>(r.zp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (r.zn != rid) __hip_atomic_fetch_max(L + 3, stored_rank<OP>(r.zn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (r.nan) __hip_atomic_fetch_or(L + 4, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    merged = true;
                }
            }
            if (merged) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // performed before the arrival
            __hip_atomic_fetch_add(L, ((uint64_t)r.cnt << kArriveBits) | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        RDX_STAMP(2);
        return;
    }
    // the folder (the chunk's last block): wave 0, lane s < 8 watches line s
    if (threadIdx.x >= 64) return;
    const uint32_t lane = threadIdx.x;
    const bool mine = lane < kTicketShards;
    uint64_t *L = acc_line(out, chunk, mine ? lane : 0);
    const uint32_t want = bpc - 1;
    // A fold that timed out (a publisher that never arrived: a device fault, or one held back for seconds)
    // cannot know whether its late publishers will still add to the lines it zeroed, so it leaves the chunk's
    // DIRTY word set, and every later order-free fold of that workspace slot reports RDX_E_DEVICE instead of
    // folding over stale words (read with the first poll: no extra round trip).  Only a new workspace clears it.
    uint64_t *const dirty = reinterpret_cast<uint64_t *>(out.tickets + (uint64_t)chunk * kTicketWords + kDirtyWord);
    uint32_t fault = 0;
    for (uint32_t it = 0;; ++it) {
        const uint64_t w = mine ? __hip_atomic_load(L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        if (it == 0 && lane == kTicketShards && __hip_atomic_load(dirty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            fault = 1;
        uint32_t got = (uint32_t)(w & ((1u << kArriveBits) - 1));
#pragma unroll
        for (int m = 4; m >= 1; m >>= 1) got += __shfl_xor(got, m, 64);
        if (__builtin_amdgcn_ballot_w64(fault != 0)) {
            fault = 1;
            break;
        }
        if (__shfl(got, 0, 64) >= want) break;
        if (it >= kSpinLimit) {
            fault = 1;
            if (lane == 0) __hip_atomic_store(dirty, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        if (it < 2) __builtin_amdgcn_s_sleep(1);
        else if (it < 6) __builtin_amdgcn_s_sleep(4);
        else __builtin_amdgcn_s_sleep(16);
    }
    // take the totals (and zero the lines for the next launch)
    uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0;
    if (mine) {
        w0 = __hip_atomic_exchange(L, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (OP != OP_COUNT) w1 = __hip_atomic_exchange(L + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (kRank) {
            w2 = __hip_atomic_exchange(L + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w3 = __hip_atomic_exchange(L + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w4 = __hip_atomic_exchange(L + 4, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    auto umax = [](uint64_t a, uint64_t c) { return a > c ? a : c; };
#pragma unroll
    for (int m = 4; m >= 1; m >>= 1) {
        w0 += shfl_xor_u64(w0, m);
        if constexpr (OP == OP_SUM) w1 += shfl_xor_u64(w1, m);
        else if constexpr (OP != OP_COUNT) w1 = umax(w1, shfl_xor_u64(w1, m));
        if constexpr (kRank) {
            w2 = umax(w2, shfl_xor_u64(w2, m));
            w3 = umax(w3, shfl_xor_u64(w3, m));
            w4 |= shfl_xor_u64(w4, m);
        }
    }
    if (lane != 0) return;
    Red<T, OP> acc = r;   // the folder's own partial (thread 0 holds the block total)
    Red<T, OP> o;
    o.init();
    o.cnt = (int64_t)(w0 >> kArriveBits);
    if constexpr (OP == OP_SUM) o.si = w1;
    else if constexpr (OP != OP_COUNT) {
        if (w1) o.v = value_of_stored<T, OP>(w1);
    }
    if constexpr (kRank) {
        o.zp = rank_of_stored<OP>(w2);
        o.zn = rank_of_stored<OP>(w3);
        o.nan = (uint32_t)(w4 & 1);
    }
    acc.merge(o);
    write_folded<T, OP>(out, chunk, acc, fault != 0 || drop);
    RDX_STAMP(3);
}

// Publish this workgroup's partial and let the LAST arriving workgroup of the chunk fold all
// partials in workgroup order and write the response (one launch, no second kernel).
template <typename T, int OP>
__device__ void finalize_all(Red<T, OP> &r, const KOut &out, uint32_t chunk, uint32_t bpc, uint32_t b) {
    constexpr int kR = granules<T, OP>();
    block_reduce(r);
    if constexpr (kAtomicFold<T, OP>) {
        if (out.fold_last == 2) {
            atomic_fold<T, OP>(r, out, chunk, bpc, b);
            return;
        }
    }
    const uint64_t *P = out.partials + (uint64_t)chunk * bpc * kR;
#if RDX_PROBES
    // fault injection (probe builds): grid block drop_block - 1 never publishes its record (it still
    // arrives / folds as usual), the way a faulted producer would look to the folder
    const bool drop = out.drop_block == 1 + blockIdx.x;
#else
    constexpr bool drop = false;
#endif
    if (threadIdx.x == 0 && !drop) publish<T, OP>(out.partials + ((uint64_t)chunk * bpc + b) * kR, r, out.epoch);
    if (out.fold_last && b != bpc - 1) {   // only the folder goes on (no arrival to count)
        RDX_STAMP(2);
        return;
    }
    arrive_and_fold<T, OP>(out, P, chunk, bpc, bpc, b);
}

// Integer count across workgroups without a hot atomic: every workgroup publishes its count (one
// tagged record word), the sharded arrival counters elect the last one, which sums the counts
// (order-free: integers) and writes `*dst`.  Same hand-off form as finalize_all.
__device__ inline void finalize_count(int64_t cnt, int64_t *dst, uint32_t *status, uint64_t *partials,
                                      uint32_t *tickets, uint32_t epoch, uint32_t nblocks, uint32_t b) {
    __shared__ int64_t part[kBlock / 64];
    __shared__ uint32_t s_last, s_fault;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) cnt += (int64_t)shfl_xor_u64((uint64_t)cnt, m);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int k = 0; k < kBlock / 64; ++k) t += part[k];
        put_granule(partials + b, (uint64_t)t, epoch);   // a count < 2^48
        s_last = arrive_last(tickets, nblocks, b);
        s_fault = 0;
    }
    __syncthreads();
    if (!s_last) return;
    int64_t t = 0;
    uint32_t fault = 0;
    for (uint32_t j = threadIdx.x; j < nblocks; j += kBlock) {
        uint64_t v = __hip_atomic_load(partials + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_expect((uint32_t)(v >> 48) != epoch, 0)) {
            if (!fault) v = poll_granule(partials + j, epoch);   // (one spin budget per lane)
            fault |= (uint32_t)(v >> 48) != epoch;
        }
        t += (int64_t)(v & kPayload);
    }
    if (fault) s_fault = 1;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) t += (int64_t)shfl_xor_u64((uint64_t)t, m);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t tot = 0;
        for (int k = 0; k < kBlock / 64; ++k) tot += part[k];
        *dst = tot;
        if (status) *status = s_fault ? (uint32_t)RDX_E_DEVICE : 0u;
        __hip_atomic_store(tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace rdx
