// Host planner: request checks, hyperslab translation and canonicalisation (see rdx_plan.hpp).
#include "rdx_plan.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace rdx {

uint32_t dtype_size(uint32_t dtype) {
    switch (dtype) {
        case RDX_DTYPE_INT32: case RDX_DTYPE_UINT32: case RDX_DTYPE_FLOAT32: return 4;
        case RDX_DTYPE_INT64: case RDX_DTYPE_UINT64: case RDX_DTYPE_FLOAT64: return 8;
        default: return 0;
    }
}

namespace {
thread_local uint32_t g_unsupported = RDX_UNSUPPORTED_NONE;
}

rdx_status unsupported(uint32_t reason) {
    g_unsupported = reason;
    return RDX_E_UNSUPPORTED;
}

uint32_t last_unsupported() { return g_unsupported; }

Div make_div(uint32_t d) {
    Div v{};
    v.d = d;
    v.magic = d <= 1 ? 0 : (~0ull / d) + 1;  // ceil(2^64 / d), exact quotients for 32-bit operands
    return v;
}

namespace {

bool is_float_dtype(uint32_t dt) { return dt == RDX_DTYPE_FLOAT32 || dt == RDX_DTYPE_FLOAT64; }

rdx_status basic_checks(const rdx_request &req) {
    if (req.abi_version != RDX_ABI_VERSION) return RDX_E_INVALID_ARGUMENT;
    if (req.op > RDX_OP_SUM || req.dtype > RDX_DTYPE_FLOAT64 || req.byte_order > RDX_BYTE_ORDER_BIG ||
        req.order > RDX_ORDER_F || req.axes_kind > RDX_AXES_MULTI || req.compression > RDX_COMPRESSION_BLOSC2 ||
        req.missing.kind > RDX_MISSING_VALID_RANGE)
        return RDX_E_INVALID_ARGUMENT;
    if (req.ndim > RDX_MAX_NDIM) return unsupported(RDX_UNSUPPORTED_RANK);
    if (req.ndim && !req.shape) return RDX_E_INVALID_ARGUMENT;
    if (req.axes_kind == RDX_AXES_ONE && !req.axes) return RDX_E_INVALID_ARGUMENT;
    if (req.axes_kind == RDX_AXES_MULTI && req.n_axes && !req.axes) return RDX_E_INVALID_ARGUMENT;
    if (req.n_filters && !req.filters) return RDX_E_INVALID_ARGUMENT;
    for (uint32_t k = 0; k < req.n_filters; ++k)
        if (req.filters[k].id != RDX_FILTER_SHUFFLE && req.filters[k].id != RDX_FILTER_SHUFFLE_SIMD)
            return RDX_E_INVALID_ARGUMENT;
    const uint32_t mk = req.missing.kind;
    if (mk != RDX_MISSING_NONE && !(mk == RDX_MISSING_VALUES && req.missing.n_values == 0) && !req.missing.values)
        return RDX_E_INVALID_ARGUMENT;
    return RDX_OK;
}

// src/models.rs:214-239
rdx_status validate_raw_size(uint64_t raw, const rdx_request &req) {
    const uint64_t ds = dtype_size(req.dtype);
    if (req.ndim) {
        uint64_t expected = 1;
        for (uint32_t k = 0; k < req.ndim; ++k)
            if (__builtin_mul_overflow(expected, req.shape[k], &expected)) return RDX_E_REQUEST_VALIDATION;
        if (__builtin_mul_overflow(expected, ds, &expected)) return RDX_E_REQUEST_VALIDATION;
        if (raw != expected) return RDX_E_REQUEST_VALIDATION;
    } else if (raw % ds != 0) {
        return RDX_E_REQUEST_VALIDATION;
    }
    return RDX_OK;
}

// Structural part of models.rs:242-313 that the reference relies on before ndarray would panic.
rdx_status structural_checks(const rdx_request &req, bool for_plan) {
    if (req.selection) {
        if (req.ndim == 0) return RDX_E_REQUEST_VALIDATION;  // "Selection requires shape"
        for (uint32_t k = 0; k < req.ndim; ++k)
            if (req.selection[k].stride == 0) return RDX_E_REQUEST_VALIDATION;  // validate_slice
    }
    // Select ignores `axis` (operations.rs:494-495); request-level validation still checks it.
    if ((req.axes_kind == RDX_AXES_ONE || req.axes_kind == RDX_AXES_MULTI) && (req.op != RDX_OP_SELECT || !for_plan)) {
        if (req.ndim == 0) return RDX_E_REQUEST_VALIDATION;  // "Axis requires shape"
        const uint32_t na = req.axes_kind == RDX_AXES_ONE ? 1 : req.n_axes;
        if (na > req.ndim) return RDX_E_REQUEST_VALIDATION;
        for (uint32_t i = 0; i < na; ++i) {
            if (req.axes[i] > req.ndim - 1) return RDX_E_REQUEST_VALIDATION;
            if (i && req.axes[i] <= req.axes[i - 1]) return RDX_E_REQUEST_VALIDATION;  // order + dups
        }
    }
    return RDX_OK;
}

template <class T>
T raw_as(const void *p, size_t i) {
    T v;
    std::memcpy(&v, static_cast<const uint8_t *>(p) + i * sizeof(T), sizeof(T));
    return v;
}

template <class T>
uint64_t bits_of(T v) {
    uint64_t b = 0;
    std::memcpy(&b, &v, sizeof(T));
    return b;
}

template <class T>
bool range_ok(const rdx_missing &m) { return raw_as<T>(m.values, 0) < raw_as<T>(m.values, 1); }

// Sorted, de-duplicated list for binary search (semantics of Vec::contains with PartialEq:
// NaN never matches, -0.0 == +0.0, so NaNs are dropped and -0.0 folded to +0.0).
template <class T>
std::vector<uint64_t> sorted_list(const rdx_missing &m) {
    std::vector<T> v;
    for (uint64_t i = 0; i < m.n_values; ++i) {
        T x = raw_as<T>(m.values, i);
        if constexpr (std::is_floating_point_v<T>) {
            if (std::isnan(x)) continue;
            if (x == T(0)) x = T(0);
        }
        v.push_back(x);
    }
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    std::vector<uint64_t> out;
    for (T x : v) out.push_back(bits_of(x));
    return out;
}

rdx_status build_missing(const rdx_request &req, ExecPlan &p) {
    const rdx_missing &m = req.missing;
    KMissing km{};
    km.kind = m.kind;
    const uint32_t es = p.esz;
    auto raw = [&](size_t i) {
        uint64_t b = 0;
        std::memcpy(&b, static_cast<const uint8_t *>(m.values) + i * es, es);
        return b;
    };
    switch (m.kind) {
        case RDX_MISSING_NONE: break;
        case RDX_MISSING_VALUE: case RDX_MISSING_VALID_MIN: case RDX_MISSING_VALID_MAX: km.v0 = raw(0); break;
        case RDX_MISSING_VALID_RANGE: km.v0 = raw(0); km.v1 = raw(1); break;
        case RDX_MISSING_VALUES:
            if (m.n_values <= (uint64_t)kInlineMissing) {
                km.n = (uint32_t)m.n_values;
                for (uint32_t i = 0; i < km.n; ++i) km.inl[i] = raw(i);
            } else {
                switch (req.dtype) {
                    case RDX_DTYPE_INT32: p.miss_list = sorted_list<int32_t>(m); break;
                    case RDX_DTYPE_INT64: p.miss_list = sorted_list<int64_t>(m); break;
                    case RDX_DTYPE_UINT32: p.miss_list = sorted_list<uint32_t>(m); break;
                    case RDX_DTYPE_UINT64: p.miss_list = sorted_list<uint64_t>(m); break;
                    case RDX_DTYPE_FLOAT32: p.miss_list = sorted_list<float>(m); break;
                    case RDX_DTYPE_FLOAT64: p.miss_list = sorted_list<double>(m); break;
                }
                if (p.miss_list.size() > 0xffffffffull) return unsupported(RDX_UNSUPPORTED_MISSING_LIST);
                km.n = (uint32_t)p.miss_list.size();
                if (km.n <= (uint32_t)kInlineMissing) {  // collapsed by de-duplication
                    for (uint32_t i = 0; i < km.n; ++i) km.inl[i] = p.miss_list[i];
                    p.miss_list.clear();
                } else {
                    km.n |= 0x80000000u;  // marks "sorted device list"
                }
            }
            break;
    }
    p.miss = km;
    return RDX_OK;
}

struct SDim {
    uint64_t count;
    int64_t vstride;    // element stride of the sliced view (signed)
    int64_t nd_stride;  // ndarray's stride after slicing: 0 when count <= 1
};

struct CDim {
    uint64_t count;
    int64_t vs;  // memory stride
    int64_t rs;  // rank / output stride
};

// ndarray Dimension::is_contiguous on the sliced view (negative strides allowed).
bool nd_is_contiguous(const std::vector<SDim> &sd) {
    const size_t n = sd.size();
    bool any_zero = false;
    for (const SDim &d : sd) any_zero |= d.count == 0;
    std::vector<int64_t> def(n, 0);
    if (!any_zero) {
        int64_t acc = 1;
        for (size_t k = n; k-- > 0;) { def[k] = acc; acc *= (int64_t)sd[k].count; }
    }
    bool eq = true;
    for (size_t k = 0; k < n; ++k) eq &= sd[k].nd_stride == def[k];
    if (eq) return true;
    if (n == 1) return sd[0].count <= 1 || sd[0].nd_stride == -1;
    std::vector<size_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return std::llabs(sd[a].nd_stride) < std::llabs(sd[b].nd_stride);
    });
    uint64_t c = 1;
    for (size_t i : order) {
        if (sd[i].count != 1 && (uint64_t)std::llabs(sd[i].nd_stride) != c) return false;
        c *= sd[i].count;
    }
    return true;
}

// Rank of each element in ndarray's fold visiting order (ArrayBase::fold: memory order when
// contiguous, else logical order after move_min_stride_axis_to_last).  Only used to reproduce
// max_by/min_by's ±0 tie rule (operations.rs:229-241, 459-469).
void fold_rank_strides(const std::vector<SDim> &sd, int64_t base_off, std::vector<int64_t> &rs, int64_t &r0) {
    const size_t n = sd.size();
    rs.assign(n, 0);
    if (nd_is_contiguous(sd)) {
        for (size_t k = 0; k < n; ++k) rs[k] = sd[k].vstride;
        r0 = base_off;
        return;
    }
    std::vector<size_t> perm(n);
    std::iota(perm.begin(), perm.end(), 0);
    if (n == 2) {
        if (sd[1].count <= 1 ||
            (sd[0].count > 1 && std::llabs(sd[0].nd_stride) < std::llabs(sd[1].nd_stride)))
            std::swap(perm[0], perm[1]);
    } else if (n > 2) {
        size_t best = n;
        for (size_t ax = 0; ax < n; ++ax) {
            if (sd[ax].count <= 1) continue;
            if (best == n || std::llabs(sd[ax].nd_stride) < std::llabs(sd[best].nd_stride)) best = ax;
        }
        if (best != n) std::swap(perm[n - 1], perm[best]);
    }
    int64_t w = 1;
    for (size_t j = n; j-- > 0;) {
        rs[perm[j]] = w;
        w *= (int64_t)sd[perm[j]].count;
    }
    r0 = 0;
}

rdx_status fill_view(KView &v, const std::vector<CDim> &inner_first, int64_t base_off, int64_t r0, uint64_t n) {
    if (inner_first.size() > (size_t)kMaxKDims) return unsupported(RDX_UNSUPPORTED_VIEW_DIMS);
    if (n > 0xffffffffull) return unsupported(RDX_UNSUPPORTED_VIEW_SIZE);
    v = KView{};
    v.ndim = (int32_t)inner_first.size();
    v.base_off = base_off;
    v.r0 = r0;
    v.n = n;
    for (size_t k = 0; k < inner_first.size(); ++k) {
        if (inner_first[k].count > 0xffffffffull) return unsupported(RDX_UNSUPPORTED_VIEW_SIZE);
        v.count[k] = (uint32_t)inner_first[k].count;
        v.div[k] = make_div((uint32_t)inner_first[k].count);
        v.vstride[k] = inner_first[k].vs;
        v.rstride[k] = inner_first[k].rs;
    }
    return RDX_OK;
}

// Merge neighbours of an innermost-first list when both strides continue the inner one.
std::vector<CDim> merge_inner_first(const std::vector<CDim> &in, bool check_rs) {
    std::vector<CDim> out;
    for (const CDim &d : in) {
        if (!out.empty()) {
            CDim &i = out.back();
            if (d.vs == i.vs * (int64_t)i.count && (!check_rs || d.rs == i.rs * (int64_t)i.count)) {
                i.count *= d.count;
                continue;
            }
        }
        out.push_back(d);
    }
    return out;
}

}  // namespace

rdx_status validate_request(const rdx_request &req) {
    rdx_status st = basic_checks(req);
    if (st) return st;
    for (uint32_t k = 0; k < req.ndim; ++k)
        if (req.shape[k] == 0) return RDX_E_REQUEST_VALIDATION;  // validate_shape, models.rs:179-185
    if (req.has_size) {
        if (req.size < 1) return RDX_E_REQUEST_VALIDATION;  // range(min = 1)
        if (req.compression == RDX_COMPRESSION_NONE && (st = validate_raw_size(req.size, req))) return st;
    }
    if ((st = structural_checks(req, false))) return st;
    if (req.missing.kind == RDX_MISSING_VALID_RANGE) {  // missing.rs:58-68: min < max
        bool ok = true;
        switch (req.dtype) {
            case RDX_DTYPE_INT32: ok = range_ok<int32_t>(req.missing); break;
            case RDX_DTYPE_INT64: ok = range_ok<int64_t>(req.missing); break;
            case RDX_DTYPE_UINT32: ok = range_ok<uint32_t>(req.missing); break;
            case RDX_DTYPE_UINT64: ok = range_ok<uint64_t>(req.missing); break;
            case RDX_DTYPE_FLOAT32: ok = range_ok<float>(req.missing); break;
            case RDX_DTYPE_FLOAT64: ok = range_ok<double>(req.missing); break;
        }
        if (!ok) return RDX_E_REQUEST_VALIDATION;
    }
    return RDX_OK;
}

rdx_status make_plan(const rdx_request &req, uint64_t len, ExecPlan &p) {
    rdx_status st = basic_checks(req);
    if (st) return st;
    p = ExecPlan{};
    p.op = req.op;
    p.dtype = req.dtype;
    p.esz = dtype_size(req.dtype);
    p.is_float = is_float_dtype(req.dtype);
    p.need_rank = p.is_float && (req.op == RDX_OP_MIN || req.op == RDX_OP_MAX);

    // filter_pipeline.rs:23-25 — gzip/zlib/blosc2 are decompressed on the device BEFORE planning
    // (k_inflate.hip, k_blosc2.hip), so `len` is the decompressed length here.
    for (uint32_t k = 0; k < req.n_filters; ++k) {
        const uint64_t es = req.filters[k].element_size;
        if (es == 0 || len % es != 0) return RDX_E_SHUFFLE_LENGTH;  // shuffle.rs:21 assert
    }
    // app.rs:169-172: validated when compressed (the raw size is only known now) or when `size` is absent
    if ((req.compression != RDX_COMPRESSION_NONE || !req.has_size) && (st = validate_raw_size(len, req))) return st;
    // array.rs:18-27 from_bytes (alignment is moot: the chunk is copied to / lives in HBM)
    if (len % p.esz != 0) return RDX_E_FROM_BYTES;
    const uint64_t n = len / p.esz;
    p.chunk_elems = n;
    if ((st = structural_checks(req, true))) return st;

    // array.rs:35-63 shape + from_shape (OutOfBounds when the shape needs more elements)
    std::vector<uint64_t> dims = req.ndim ? std::vector<uint64_t>(req.shape, req.shape + req.ndim)
                                          : std::vector<uint64_t>{n};
    uint64_t need = 1;
    for (uint64_t d : dims)
        if (__builtin_mul_overflow(need, d, &need)) return RDX_E_SHAPE_INVALID;
    if (need > n) return RDX_E_SHAPE_INVALID;
    const size_t nd = dims.size();
    std::vector<int64_t> ms(nd, 0);
    if (req.order == RDX_ORDER_F) {
        int64_t acc = 1;
        for (size_t k = 0; k < nd; ++k) { ms[k] = acc; acc *= (int64_t)dims[k]; }
    } else {
        int64_t acc = 1;
        for (size_t k = nd; k-- > 0;) { ms[k] = acc; acc *= (int64_t)dims[k]; }
    }

    // array.rs:93-144 numpy -> ndarray slices, then ndarray do_slice.
    std::vector<SDim> sd(nd);
    int64_t base_off = 0;
    uint64_t n_sel = 1;
    for (size_t k = 0; k < nd; ++k) {
        uint64_t count = dims[k];
        int64_t step = 1;
        int64_t first = 0;
        if (req.selection) {
            const rdx_slice &s = req.selection[k];
            const int64_t L = (int64_t)dims[k];
            const bool rev = s.stride < 0;
            auto idx = [&](int64_t i) {
                const int64_t r = rev ? i + 1 : i;
                return i < 0 ? std::max<int64_t>(r + L, 0) : std::min<int64_t>(r, L);
            };
            int64_t a = idx(s.start), b = idx(s.end);
            if (rev) std::swap(a, b);
            if (b < a) b = a;
            const uint64_t m = (uint64_t)(b - a);
            step = s.stride;
            const uint64_t as = (uint64_t)(step < 0 ? -step : step);
            count = m / as + (m % as ? 1 : 0);
            first = m == 0 ? 0 : (step < 0 ? b - 1 : a);
        }
        base_off += first * ms[k];
        sd[k].count = count;
        sd[k].vstride = step * ms[k];
        sd[k].nd_stride = count <= 1 ? 0 : sd[k].vstride;
        n_sel *= count;
    }

    // missing + filters
    if ((st = build_missing(req, p))) return st;
    p.bswap = req.byte_order == RDX_BYTE_ORDER_BIG;
    for (uint32_t k = req.n_filters; k-- > 1;)
        if (req.filters[k].element_size != 1) p.unfused_es.push_back(req.filters[k].element_size);
    if (req.n_filters) {
        const uint64_t es0 = req.filters[0].element_size;
        if (es0 == p.esz) p.fused = true;
        else if (es0 != 1) p.unfused_es.push_back(es0);
    }

    // response info (models.rs:316-351 as filled by operations.rs)
    rdx_response_info &info = p.info;
    info = rdx_response_info{};
    info.dtype = req.op == RDX_OP_COUNT ? RDX_DTYPE_INT64 : req.dtype;
    const uint64_t out_es = req.op == RDX_OP_COUNT ? 8 : p.esz;
    auto set_shape = [&](const std::vector<uint64_t> &s) {
        info.ndim = (uint32_t)s.size();
        for (size_t k = 0; k < s.size(); ++k) info.shape[k] = s[k];
    };
    std::vector<uint64_t> sliced_shape(nd);
    for (size_t k = 0; k < nd; ++k) sliced_shape[k] = sd[k].count;

    std::vector<uint64_t> axes;
    if (req.axes_kind == RDX_AXES_ONE) axes.push_back(req.axes[0]);
    if (req.axes_kind == RDX_AXES_MULTI) axes.assign(req.axes, req.axes + req.n_axes);

    const bool is_map = req.op == RDX_OP_SELECT || (req.axes_kind != RDX_AXES_ALL && axes.empty());
    if (is_map) {
        // Output traversal: Select -> C order unless the UNSLICED array is not standard layout
        // (operations.rs:508-513); axis=() -> F traversal when order == F (operations.rs:204-209),
        // except Count which always maps in C order (operations.rs:58-67).
        bool f_traversal = false;
        if (req.op == RDX_OP_SELECT) {
            bool standard = true;
            bool any_zero = false;
            for (uint64_t d : dims) any_zero |= d == 0;
            if (!any_zero && req.order == RDX_ORDER_F) {
                int nonunit = 0;
                for (uint64_t d : dims) nonunit += d != 1;
                standard = nonunit <= 1;
            }
            f_traversal = !standard;
            set_shape(sliced_shape);
            info.body_bytes = n_sel * p.esz;
            info.n_counts = 1;
            p.map.kind = 0;
        } else {
            f_traversal = req.op != RDX_OP_COUNT && req.order == RDX_ORDER_F;
            set_shape(sliced_shape);
            info.body_bytes = n_sel * out_es;
            info.n_counts = n_sel;
            p.map.kind = req.op == RDX_OP_COUNT ? 2 : 1;
        }
        std::vector<CDim> inner_first;  // output order, innermost first
        for (size_t j = 0; j < nd; ++j) {
            const size_t k = f_traversal ? j : nd - 1 - j;
            if (sd[k].count != 1) inner_first.push_back({sd[k].count, sd[k].vstride, 0});
        }
        if (n_sel == 0) inner_first.clear();
        p.mode = Mode::Map;
        return fill_view(p.map.view, merge_inner_first(inner_first, false), base_off, 0, n_sel);
    }

    if (req.axes_kind == RDX_AXES_ALL) {
        set_shape({});
        info.body_bytes = out_es;
        info.n_counts = 1;
        std::vector<int64_t> rs(nd, 0);
        int64_t r0 = 0;
        if (p.need_rank) fold_rank_strides(sd, base_off, rs, r0);
        if (n_sel == 0) {
            p.mode = Mode::AllContig;
            p.all_contig.off = 0;
            p.all_contig.n = 0;
            p.all_contig.filter_semantics = req.op == RDX_OP_COUNT;
            return RDX_OK;
        }
        std::vector<CDim> cd;
        int64_t off = base_off;
        for (size_t k = 0; k < nd; ++k) {
            if (sd[k].count == 1) continue;
            CDim d{sd[k].count, sd[k].vstride, rs[k]};
            if (d.vs < 0) {  // traverse ascending: ties are resolved by rank, not visiting order
                off += (int64_t)(d.count - 1) * d.vs;
                r0 += (int64_t)(d.count - 1) * d.rs;
                d.vs = -d.vs;
                d.rs = -d.rs;
            }
            cd.push_back(d);
        }
        std::stable_sort(cd.begin(), cd.end(), [](const CDim &a, const CDim &b) { return a.vs < b.vs; });
        cd = merge_inner_first(cd, p.need_rank);
        if (cd.empty() || (cd.size() == 1 && cd[0].vs == 1)) {
            p.mode = Mode::AllContig;
            p.all_contig.off = (uint64_t)off;
            p.all_contig.n = n_sel;
            p.all_contig.r0 = r0;
            p.all_contig.rs = cd.empty() ? 0 : cd[0].rs;
            p.all_contig.filter_semantics = req.op == RDX_OP_COUNT;
            return RDX_OK;
        }
        p.mode = Mode::AllStrided;
        p.all_strided.filter_semantics = req.op == RDX_OP_COUNT;
        return fill_view(p.all_strided.view, cd, off, r0, n_sel);
    }

    // Reduction over a subset of axes (count_array_multi_axis / *_array_multi_axis).
    std::vector<bool> is_red(nd, false);
    for (uint64_t a : axes) is_red[a] = true;
    std::vector<uint64_t> out_shape;
    for (size_t k = 0; k < nd; ++k)
        if (!is_red[k]) out_shape.push_back(sd[k].count);
    set_shape(out_shape);
    uint64_t n_out = 1, n_red = 1;
    for (size_t k = 0; k < nd; ++k) (is_red[k] ? n_red : n_out) *= sd[k].count;
    info.body_bytes = n_out * out_es;
    info.n_counts = n_out;
    p.mode = Mode::Axis;
    KAxis &ax = p.axis;
    ax.n_out = n_out;
    ax.n_red = n_red;
    if (n_out == 0) return RDX_OK;
    // kept: output C-order strides; reduced: tie rank = F order over the axes in request order
    std::vector<CDim> K, R;
    {
        int64_t os = 1;
        std::vector<int64_t> ostr(nd, 0);
        for (size_t k = nd; k-- > 0;)
            if (!is_red[k]) { ostr[k] = os; os *= (int64_t)sd[k].count; }
        for (size_t k = 0; k < nd; ++k)
            if (!is_red[k] && sd[k].count != 1) K.push_back({sd[k].count, sd[k].vstride, ostr[k]});
        int64_t w = 1;
        for (uint64_t a : axes) {
            if (sd[a].count != 1) R.push_back({sd[a].count, sd[a].vstride, w});
            w *= (int64_t)sd[a].count;
        }
    }
    if (n_red == 0) R.clear();
    int64_t off = base_off, r0 = 0;
    for (CDim &d : R)
        if (d.vs < 0) {
            off += (int64_t)(d.count - 1) * d.vs;
            r0 += (int64_t)(d.count - 1) * d.rs;
            d.vs = -d.vs;
            d.rs = -d.rs;
        }
    int64_t minK = INT64_MAX, minR = INT64_MAX;
    for (const CDim &d : K) minK = std::min<int64_t>(minK, std::llabs(d.vs));
    for (const CDim &d : R) minR = std::min<int64_t>(minR, d.vs);
    std::stable_sort(R.begin(), R.end(), [](const CDim &a, const CDim &b) { return a.vs < b.vs; });
    R = merge_inner_first(R, p.need_rank);
    // rows (a wave per output) when the innermost memory dim is reduced AND its contiguous run fills
    // at least a 64-lane x 4 B wave access; otherwise a lane per output along the innermost kept dim.
    const bool long_run = !R.empty() && R[0].vs == 1 && R[0].count * p.esz >= 256;
    ax.mode = (minR <= minK && (long_run || K.empty())) ? 0u : 1u;
    if (ax.mode == 1)
        std::stable_sort(K.begin(), K.end(), [](const CDim &a, const CDim &b) { return std::llabs(a.vs) < std::llabs(b.vs); });
    else
        std::stable_sort(K.begin(), K.end(), [](const CDim &a, const CDim &b) { return a.rs < b.rs; });
    {   // merge kept dims when both memory and output strides continue
        std::vector<CDim> m;
        for (const CDim &d : K) {
            if (!m.empty() && d.vs == m.back().vs * (int64_t)m.back().count &&
                d.rs == m.back().rs * (int64_t)m.back().count) {
                m.back().count *= d.count;
                continue;
            }
            m.push_back(d);
        }
        K = m;
    }
    if ((st = fill_view(ax.kept, K, off, 0, n_out))) return st;
    if ((st = fill_view(ax.red, R, 0, r0, n_red))) return st;
    return RDX_OK;
}

}  // namespace rdx
