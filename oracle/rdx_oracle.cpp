// ============================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.
//
//  A sequential CPU restatement of reductionist-rs's synchronous request path, used by tests/,
//  __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.  It is never linked
//  into, loaded by, or called from the product library (reductionist-rs_amd/), which has no CPU
//  fallback.  It shares only the plain-C interface structs of include/rdx.h with the product; no
//  logic is shared.
//
//  Reference: /root/reference (reductionist 0.13.1).  Every function below cites the file:line it
//  restates.  The reference is Rust and cannot be built here (no cargo/rustc, no crates registry),
//  so this restatement is pinned against the known-answer tests transcribed from the reference's
//  own #[cfg(test)] modules into tests/golden/ (see tests/golden/make_golden.py and
//  tests/test_oracle_golden.py).  Behaviour that lives in un-vendored crates is restated from
//  their published algorithms:
//    * ndarray 0.15.6 — slicing (do_slice/to_abs_slice), is_contiguous/is_standard_layout,
//      fold (memory order if contiguous, else min-stride axis swapped last), fold_axis, map, t().
//    * byteshuffle 0.1.2 (shuffle_simd) — same output as filters/shuffle.rs (pinned by identical
//      KATs in shuffle_simd.rs:32-57 and filters.rs:41-50).
//    * num-traits 0.2.19 — Bounded::min_value/max_value identities, from_be_bytes(to_le_bytes).
//  The exact f32/f64 summation order of ndarray's fold over strided views is restated from the
//  0.15.6 source as recalled (not verifiable here: crate not vendored) — "parity unpinned" for the
//  ORDER of floating-point sums on non-contiguous views; integer, count, select and min/max results
//  are order independent except for the ±0 tie rule, which follows max_by/min_by exactly.
//
//  Build: oracle/Makefile (g++ -O2, no -ffast-math) -> oracle/build/liboracle.so
// ============================================================================================
#include "../include/rdx.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <type_traits>
#include <vector>

extern "C" void oracle_blosc2_sizes(const uint8_t *src, uint64_t len, uint64_t *nbytes, uint64_t *cbytes,
                                   uint64_t *blocksize);
extern "C" uint32_t oracle_blosc2_decompress(const uint8_t *src, uint64_t len, uint8_t *out, uint64_t cap,
                                             uint64_t *out_len);
extern "C" uint32_t oracle_decompress(uint32_t compression, const uint8_t *in, uint64_t len, uint8_t *out,
                                      uint64_t cap, uint64_t *out_len);  // oracle_inflate.cpp

namespace {

using i64 = int64_t;
using u64 = uint64_t;

struct OracleError {
    rdx_status status;
};

// ----------------------------------------------------------------------------------------------
// src/filters/shuffle.rs:20-85 — deshuffle: out[i*es + k] = in[k*N + i].  assert_eq!(len % es, 0)
// panics (es == 0 panics with a remainder-by-zero).
std::vector<uint8_t> deshuffle(const std::vector<uint8_t> &data, u64 element_size) {
    if (element_size == 0 || data.size() % element_size != 0) throw OracleError{RDX_E_SHUFFLE_LENGTH};
    std::vector<uint8_t> m(data.size(), 0);  // shuffle.rs:22-26 zero-filled result
    const u64 n = data.size() / element_size;
    u64 dest = 0;
    for (u64 i = 0; i < n; ++i) {
        u64 src = i;
        for (u64 k = 0; k < element_size; ++k) {
            m[dest++] = data[src];
            src += n;
        }
    }
    return m;
}

// src/filters/shuffle.rs:124-135 — test-only encoder.
std::vector<uint8_t> shuffle(const std::vector<uint8_t> &data, u64 element_size) {
    std::vector<uint8_t> r;
    r.reserve(data.size());
    for (u64 i = 0; i < element_size; ++i) {
        u64 src = i;
        for (u64 j = 0; j < data.size() / element_size; ++j) {
            r.push_back(data[src]);
            src += element_size;
        }
    }
    return r;
}

u64 dtype_size(uint32_t dtype) {
    switch (dtype) {
        case RDX_DTYPE_INT32: case RDX_DTYPE_UINT32: case RDX_DTYPE_FLOAT32: return 4;
        case RDX_DTYPE_INT64: case RDX_DTYPE_UINT64: case RDX_DTYPE_FLOAT64: return 8;
        default: throw OracleError{RDX_E_INVALID_ARGUMENT};
    }
}

// ----------------------------------------------------------------------------------------------
// ndarray 0.15.6 view emulation.  Element offsets are relative to the data start.
struct View {
    std::vector<u64> dim;
    std::vector<i64> strides;
    i64 offset = 0;  // element offset of logical index 0
    u64 len() const {
        u64 n = 1;
        for (u64 d : dim) n *= d;
        return n;
    }
};

// ndarray Dimension::default_strides / fortran_strides: all zeros if any axis is empty.
std::vector<i64> default_strides(const std::vector<u64> &dim, bool fortran) {
    std::vector<i64> s(dim.size(), 0);
    for (u64 d : dim)
        if (d == 0) return s;
    if (!fortran) {
        i64 acc = 1;
        for (size_t k = dim.size(); k-- > 0;) { s[k] = acc; acc *= (i64)dim[k]; }
    } else {
        i64 acc = 1;
        for (size_t k = 0; k < dim.size(); ++k) { s[k] = acc; acc *= (i64)dim[k]; }
    }
    return s;
}

// ndarray is_contiguous (Dimension::is_contiguous, dimension/dimension_trait.rs).
bool is_contiguous(const View &v) {
    const size_t n = v.dim.size();
    if (v.strides == default_strides(v.dim, false)) return true;
    if (n == 1) return v.dim[0] <= 1 || v.strides[0] == -1;
    // _fastest_varying_stride_order: axes sorted by |stride| ascending (stable on index)
    std::vector<size_t> order(n);
    for (size_t k = 0; k < n; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return std::llabs(v.strides[a]) < std::llabs(v.strides[b]);
    });
    u64 cstride = 1;
    for (size_t i : order) {
        if (v.dim[i] != 1 && (u64)std::llabs(v.strides[i]) != cstride) return false;
        cstride *= v.dim[i];
    }
    return true;
}

// ndarray is_standard_layout (impl_methods.rs) for IxDyn.
bool is_standard_layout(const View &v) {
    for (u64 d : v.dim)
        if (d == 0) return true;
    std::vector<i64> def = default_strides(v.dim, false);
    for (size_t k = 0; k < v.dim.size(); ++k)
        if (v.dim[k] != 1 && v.strides[k] != def[k]) return false;
    return true;
}

// src/array.rs:93-101 to_ndarray_index
i64 to_ndarray_index(i64 index, u64 length, bool reverse) {
    const i64 len = (i64)length;
    const i64 result = reverse ? index + 1 : index;
    if (index < 0) return std::max<i64>(result + len, 0);
    return std::min<i64>(result, len);
}

// src/array.rs:108-118 to_ndarray_slice + ndarray do_slice/to_abs_slice (dimension/mod.rs).
void slice_axis(View &v, size_t ax, const rdx_slice &s) {
    const bool reverse = s.stride < 0;
    i64 start = to_ndarray_index(s.start, v.dim[ax], reverse);
    i64 end = to_ndarray_index(s.end, v.dim[ax], reverse);
    if (reverse) std::swap(start, end);
    // to_abs_slice: (start,end already in [0,len]) end = max(end, start)
    if (end < start) end = start;
    const i64 step = s.stride;
    const u64 m = (u64)(end - start);
    const i64 stride = v.strides[ax];
    i64 off = 0;
    if (m == 0) off = 0;
    else if (step < 0) off = (end - 1) * stride;
    else off = start * stride;
    // stride 0 never gets here in the reference (models.rs:187-194 rejects it; ndarray asserts step != 0)
    if (step == 0) throw OracleError{RDX_E_REQUEST_VALIDATION};
    const u64 abs_step = (u64)(step < 0 ? -step : step);
    u64 d = abs_step == 1 ? m : (m / abs_step + (m % abs_step ? 1 : 0));
    v.offset += off;
    v.dim[ax] = d;
    v.strides[ax] = d <= 1 ? 0 : stride * step;
}

// src/array.rs:121-144 build_slice_info + ArrayView::slice
// No selection still slices every axis with [0, len, 1] (array.rs:133-141), which zeroes the
// stride of unit axes exactly as ndarray does.
View slice_view(const View &a, const rdx_slice *selection) {
    View v = a;
    for (size_t ax = 0; ax < v.dim.size(); ++ax) {
        const rdx_slice full{0, (int64_t)v.dim[ax], 1};
        slice_axis(v, ax, selection ? selection[ax] : full);
    }
    return v;
}

View transpose(const View &a) {  // ndarray ArrayBase::t()
    View v = a;
    std::reverse(v.dim.begin(), v.dim.end());
    std::reverse(v.strides.begin(), v.strides.end());
    return v;
}

// Logical (C) order iteration: ArrayBase::iter()
template <class F>
void for_each_logical(const View &v, F &&f) {
    const size_t n = v.dim.size();
    if (v.len() == 0) return;
    std::vector<u64> idx(n, 0);
    i64 off = v.offset;
    while (true) {
        f(off);
        // increment last axis fastest
        size_t k = n;
        while (k > 0) {
            --k;
            if (++idx[k] < v.dim[k]) { off += v.strides[k]; break; }
            off -= (i64)(idx[k] - 1) * v.strides[k];
            idx[k] = 0;
            if (k == 0) return;
        }
        if (n == 0) return;
    }
}

// ndarray ArrayBase::fold: memory order if as_slice_memory_order() succeeds, otherwise
// move_min_stride_axis_to_last + logical iteration (impl_methods.rs, dimension/mod.rs).
template <class F>
void for_each_fold_order(const View &v, F &&f) {
    if (v.len() == 0) return;
    if (is_contiguous(v)) {
        // offset_from_low_addr_ptr_to_logical_ptr: lowest address among elements
        i64 low = v.offset;
        for (size_t k = 0; k < v.dim.size(); ++k)
            if (v.strides[k] < 0 && v.dim[k] > 0) low += (i64)(v.dim[k] - 1) * v.strides[k];
        const u64 n = v.len();
        for (u64 i = 0; i < n; ++i) f(low + (i64)i);
        return;
    }
    View w = v;
    const size_t n = w.dim.size();
    if (n == 2) {
        if (w.dim[1] <= 1 || (w.dim[0] > 1 && std::llabs(w.strides[0]) < std::llabs(w.strides[1]))) {
            std::swap(w.dim[0], w.dim[1]);
            std::swap(w.strides[0], w.strides[1]);
        }
    } else if (n > 2) {
        size_t best = n;  // min_by_key: first minimum among axes with dim > 1
        for (size_t ax = 0; ax < n; ++ax) {
            if (w.dim[ax] <= 1) continue;
            if (best == n || std::llabs(w.strides[ax]) < std::llabs(w.strides[best])) best = ax;
        }
        if (best != n) {
            std::swap(w.dim[n - 1], w.dim[best]);
            std::swap(w.strides[n - 1], w.strides[best]);
        }
    }
    for_each_logical(w, f);
}

// ----------------------------------------------------------------------------------------------
// src/types/missing.rs:31-42,114-122 and src/operations.rs:25-33
template <class T>
struct Missing {
    uint32_t kind = RDX_MISSING_NONE;
    std::vector<T> values;
    bool present() const { return kind != RDX_MISSING_NONE; }
    // Missing::is_missing (missing.rs:114-122)
    bool is_missing(T x) const {
        switch (kind) {
            case RDX_MISSING_VALUE: return x == values[0];
            case RDX_MISSING_VALUES:
                for (const T &v : values)
                    if (v == x) return true;
                return false;
            case RDX_MISSING_VALID_MIN: return x < values[0];
            case RDX_MISSING_VALID_MAX: return x > values[0];
            case RDX_MISSING_VALID_RANGE: return x < values[0] || x > values[1];
            default: return false;
        }
    }
    // missing_filter (operations.rs:25-33): keep when true
    bool filter_keep(T x) const {
        switch (kind) {
            case RDX_MISSING_VALUE: return x != values[0];
            case RDX_MISSING_VALUES:
                for (const T &v : values)
                    if (v == x) return false;
                return true;
            case RDX_MISSING_VALID_MIN: return x >= values[0];
            case RDX_MISSING_VALID_MAX: return x <= values[0];
            case RDX_MISSING_VALID_RANGE: return x >= values[0] && x <= values[1];
            default: return true;
        }
    }
};

// partial_cmp for max_by/min_by (operations.rs:166-184, 337-358): NaN panics.
template <class T>
int partial_cmp(T a, T b) {
    if constexpr (std::is_floating_point_v<T>) {
        if (std::isnan(a) || std::isnan(b)) throw OracleError{RDX_E_NAN_UNORDERED};
    }
    return a < b ? -1 : (a > b ? 1 : 0);
}
// std::cmp::max_by: Less|Equal -> v2, Greater -> v1
template <class T>
T max_by(T v1, T v2) { return partial_cmp(v1, v2) > 0 ? v1 : v2; }
// std::cmp::min_by: Less|Equal -> v1, Greater -> v2
template <class T>
T min_by(T v1, T v2) { return partial_cmp(v1, v2) > 0 ? v2 : v1; }

// Release-profile arithmetic: integers wrap (Dockerfile builds release), floats IEEE.
template <class T>
T add(T a, T b) {
    if constexpr (std::is_integral_v<T>) {
        using U = std::make_unsigned_t<T>;
        return (T)(U)((U)a + (U)b);
    } else {
        return a + b;
    }
}

template <class T>
T bswap_value(T x) {  // array.rs:147-154 reverse_byte_order: from_be_bytes(to_le_bytes)
    uint8_t b[sizeof(T)];
    std::memcpy(b, &x, sizeof(T));
    std::reverse(b, b + sizeof(T));
    T y;
    std::memcpy(&y, b, sizeof(T));
    return y;
}

struct Response {
    uint32_t dtype;
    std::vector<u64> shape;
    std::vector<uint8_t> body;
    std::vector<i64> count;
};

template <class T>
void push_value(std::vector<uint8_t> &body, T v) {
    const size_t at = body.size();
    body.resize(at + sizeof(T));
    std::memcpy(body.data() + at, &v, sizeof(T));
}

// Array of (value, count) pairs with a C-order shape, as produced by fold_axis/map.
template <class V>
struct Owned {
    std::vector<u64> dim;
    std::vector<V> data;  // C order
};

// ndarray fold_axis: result = from_elem(dim without axis, init); for each subview along axis
// (index order) zip_mut_with -> each output is a sequential fold along `axis`.
template <class V, class Src, class F>
Owned<V> fold_axis(const std::vector<u64> &dim, size_t axis, Src &&at, V init, F &&fold) {
    Owned<V> r;
    for (size_t k = 0; k < dim.size(); ++k)
        if (k != axis) r.dim.push_back(dim[k]);
    u64 outer = 1, inner = 1;
    for (size_t k = 0; k < axis; ++k) outer *= dim[k];
    for (size_t k = axis + 1; k < dim.size(); ++k) inner *= dim[k];
    r.data.assign(outer * inner, init);
    for (u64 i = 0; i < dim[axis]; ++i)
        for (u64 o = 0; o < outer; ++o)
            for (u64 n = 0; n < inner; ++n) {
                V &x = r.data[o * inner + n];
                x = fold(x, at((o * dim[axis] + i) * inner + n));
            }
    return r;
}

// Materialise a view's elements in C (logical) order.
template <class T>
std::vector<T> logical_values(const View &v, const T *data) {
    std::vector<T> out;
    out.reserve(v.len());
    for_each_logical(v, [&](i64 off) { out.push_back(data[off]); });
    return out;
}

// src/operations.rs:188-210 reduction_over_zero_axes
template <class T>
std::vector<std::pair<T, i64>> zero_axes(const View &sliced, const T *data, const Missing<T> &m,
                                         uint32_t order) {
    View it = order == RDX_ORDER_F ? transpose(sliced) : sliced;
    std::vector<std::pair<T, i64>> r;
    for_each_logical(it, [&](i64 off) {
        T v = data[off];
        r.push_back({v, (m.present() && m.is_missing(v)) ? 0 : 1});
    });
    return r;
}

enum class RedKind { Sum, Max, Min };

// src/operations.rs:213-268 / 361-416 / 532-583 *_array_multi_axis (axes non-empty)
template <class T>
Owned<std::pair<T, i64>> multi_axis(const View &sliced, const T *data, const std::vector<u64> &axes,
                                    const Missing<T> &m, RedKind kind) {
    const std::vector<T> vals = logical_values(sliced, data);
    const T init = kind == RedKind::Sum ? T(0)
                   : kind == RedKind::Max ? std::numeric_limits<T>::lowest()
                                          : std::numeric_limits<T>::max();
    // NOTE: num_traits Bounded::min_value for floats is f32::MIN / f64::MIN == lowest() (finite).
    auto step = [&](T acc, T v) -> T {
        switch (kind) {
            case RedKind::Sum: return add(acc, v);
            case RedKind::Max: return max_by(acc, v);
            default: return min_by(acc, v);
        }
    };
    using P = std::pair<T, i64>;
    Owned<P> res = fold_axis<P>(
        sliced.dim, axes[0], [&](u64 i) { return vals[i]; }, P{init, 0},
        [&](const P &acc, T v) -> P {
            if (m.present() && m.is_missing(v)) return acc;
            return P{step(acc.first, v), acc.second + 1};
        });
    for (size_t n = 0; n + 1 < axes.size(); ++n) {
        const size_t ax = axes[n + 1] - n - 1;
        const Owned<P> prev = res;
        res = fold_axis<P>(
            prev.dim, ax, [&](u64 i) { return prev.data[i]; }, P{init, 0},
            [&](const P &acc, const P &x) -> P { return P{step(acc.first, x.first), acc.second + x.second}; });
    }
    return res;
}

template <class T>
Missing<T> typed_missing(const rdx_request &req) {
    Missing<T> m;
    m.kind = req.missing.kind;
    if (m.kind != RDX_MISSING_NONE) {
        u64 n = req.missing.n_values;
        if (m.kind == RDX_MISSING_VALUE || m.kind == RDX_MISSING_VALID_MIN || m.kind == RDX_MISSING_VALID_MAX) n = 1;
        if (m.kind == RDX_MISSING_VALID_RANGE) n = 2;
        if (n > 0 && !req.missing.values) throw OracleError{RDX_E_INVALID_ARGUMENT};
        m.values.resize(n);
        if (n) std::memcpy(m.values.data(), req.missing.values, n * sizeof(T));
    }
    return m;
}

std::vector<u64> axes_of(const rdx_request &req) {
    std::vector<u64> ax;
    if (req.axes_kind == RDX_AXES_ONE) ax.push_back(req.axes[0]);
    if (req.axes_kind == RDX_AXES_MULTI)
        for (uint32_t i = 0; i < req.n_axes; ++i) ax.push_back(req.axes[i]);
    return ax;
}

// src/operation.rs:78-96 execute -> execute_t::<T>; src/array.rs:188-208 build_array;
// src/operations.rs Count/Max/Min/Select/Sum::execute_t.
template <class T>
Response execute_t(const rdx_request &req, std::vector<uint8_t> &bytes) {
    // array.rs:18-27 from_bytes (the copy below is 8-byte aligned, so only the length can fail)
    if (bytes.size() % sizeof(T) != 0) throw OracleError{RDX_E_FROM_BYTES};
    const u64 n = bytes.size() / sizeof(T);
    T *data = reinterpret_cast<T *>(bytes.data());
    // array.rs:35-47 get_shape, :58-63 from_shape (OutOfBounds when prod(shape) > n)
    View base;
    if (req.ndim == 0) base.dim = {n};
    else base.dim.assign(req.shape, req.shape + req.ndim);
    const bool fortran = req.order == RDX_ORDER_F;
    base.strides = default_strides(base.dim, fortran);
    if (base.len() > n) throw OracleError{RDX_E_SHAPE_INVALID};
    // array.rs:197-204 non-native byte order: reverse in place, only inside the selection
    if (req.byte_order == RDX_BYTE_ORDER_BIG) {
        View sel = slice_view(base, req.selection);
        for_each_logical(sel, [&](i64 off) { data[off] = bswap_value(data[off]); });
    }
    const View sliced = slice_view(base, req.selection);
    const Missing<T> m = typed_missing<T>(req);
    const std::vector<u64> axes = axes_of(req);
    // ndarray asserts axis.index() < ndim (operations.rs:1112-1118 should_panic) and the
    // `axis - n - 1` arithmetic needs ascending unique axes; models.rs:264-296 rejects all of
    // these at request validation, which is the status reported here.  Select ignores `axis`.
    if (req.op != RDX_OP_SELECT) {
        for (size_t i = 0; i < axes.size(); ++i)
            if (axes[i] >= base.dim.size() || (i && axes[i] <= axes[i - 1])) throw OracleError{RDX_E_REQUEST_VALIDATION};
    }
    Response r;
    r.dtype = req.dtype;

    if (req.op == RDX_OP_SELECT) {  // operations.rs:487-526
        i64 count = 0;
        if (m.present()) {
            for_each_logical(sliced, [&](i64 off) { count += m.filter_keep(data[off]) ? 1 : 0; });
        } else {
            count = (i64)sliced.len();
        }
        const View it = is_standard_layout(base) ? sliced : transpose(sliced);
        for_each_logical(it, [&](i64 off) { push_value(r.body, data[off]); });
        r.shape = sliced.dim;
        r.count = {count};
        return r;
    }

    if (req.op == RDX_OP_COUNT) {  // operations.rs:103-161
        r.dtype = RDX_DTYPE_INT64;
        if (req.axes_kind == RDX_AXES_ALL) {
            i64 count = 0;
            if (m.present()) {  // count_non_missing: iter().filter(missing_filter).count()
                for_each_logical(sliced, [&](i64 off) { count += m.filter_keep(data[off]) ? 1 : 0; });
            } else {
                count = (i64)sliced.len();
            }
            push_value(r.body, count);
            r.count = {count};
            return r;
        }
        // count_array_multi_axis (operations.rs:51-100)
        if (axes.empty()) {
            for_each_logical(sliced, [&](i64 off) {
                const i64 c = (m.present() && m.is_missing(data[off])) ? 0 : 1;
                push_value(r.body, c);
                r.count.push_back(c);
            });
            r.shape = sliced.dim;
            return r;
        }
        const std::vector<T> vals = logical_values(sliced, data);
        Owned<i64> res = fold_axis<i64>(
            sliced.dim, axes[0], [&](u64 i) { return vals[i]; }, 0,
            [&](i64 acc, T v) -> i64 { return (m.present() && m.is_missing(v)) ? acc : acc + 1; });
        for (size_t k = 0; k + 1 < axes.size(); ++k) {
            const Owned<i64> prev = res;
            res = fold_axis<i64>(
                prev.dim, axes[k + 1] - k - 1, [&](u64 i) { return prev.data[i]; }, 0,
                [](i64 acc, i64 c) { return acc + c; });
        }
        for (i64 c : res.data) { push_value(r.body, c); r.count.push_back(c); }
        r.shape = res.dim;
        return r;
    }

    const RedKind kind = req.op == RDX_OP_SUM ? RedKind::Sum : req.op == RDX_OP_MAX ? RedKind::Max : RedKind::Min;
    if (req.axes_kind == RDX_AXES_ALL) {
        // sliced.fold((init, 0_i64), ...) — operations.rs:303-318 / 457-473 / 622-632
        T acc = kind == RedKind::Sum ? T(0)
                : kind == RedKind::Max ? std::numeric_limits<T>::lowest()
                                       : std::numeric_limits<T>::max();
        i64 count = 0;
        for_each_fold_order(sliced, [&](i64 off) {
            const T v = data[off];
            if (m.present() && m.is_missing(v)) return;
            switch (kind) {
                case RedKind::Sum: acc = add(acc, v); break;
                case RedKind::Max: acc = max_by(acc, v); break;
                case RedKind::Min: acc = min_by(acc, v); break;
            }
            ++count;
        });
        push_value(r.body, acc);
        r.count = {count};
        return r;
    }
    if (axes.empty()) {  // reduction_over_zero_axes
        for (const auto &p : zero_axes(sliced, data, m, req.order)) {
            push_value(r.body, p.first);
            r.count.push_back(p.second);
        }
        r.shape = sliced.dim;
        return r;
    }
    Owned<std::pair<T, i64>> res = multi_axis(sliced, data, axes, m, kind);
    for (const auto &p : res.data) {
        push_value(r.body, p.first);
        r.count.push_back(p.second);
    }
    r.shape = res.dim;
    return r;
}

// src/models.rs:214-239 validate_raw_size
void validate_raw_size(u64 raw_size, uint32_t dtype, const rdx_request &req) {
    const u64 ds = dtype_size(dtype);
    if (req.ndim > 0) {
        u64 expected = 1;
        for (uint32_t k = 0; k < req.ndim; ++k) expected *= req.shape[k];
        if (raw_size != expected * ds) throw OracleError{RDX_E_REQUEST_VALIDATION};
    } else if (raw_size % ds != 0) {
        throw OracleError{RDX_E_REQUEST_VALIDATION};
    }
}

thread_local uint32_t g_inflate_error = 0;

// src/app.rs:163-183 operation<T>
Response execute_dtype(const rdx_request &req, std::vector<uint8_t> &data);

Response operation(const rdx_request &req, const uint8_t *chunk, u64 len) {
    std::vector<uint8_t> data;
    // filter_pipeline.rs:19-34: decompress (compression.rs:18-27, oracle_inflate.cpp), then the
    // filters in reverse
    g_inflate_error = 0;
    if (req.compression == RDX_COMPRESSION_GZIP || req.compression == RDX_COMPRESSION_ZLIB) {
        u64 cap = 4 * len + 4096, got = 0;
        for (;;) {
            data.resize(cap);
            const uint32_t e = oracle_decompress(req.compression, chunk, len, data.data(), cap, &got);
            if (e == RDX_INFLATE_OUTPUT_OVERFLOW) {
                cap *= 4;
                continue;
            }
            if (e != RDX_INFLATE_OK) {
                g_inflate_error = e;
                throw OracleError{RDX_E_DECOMPRESSION};
            }
            data.resize(got);
            break;
        }
    } else if (req.compression == RDX_COMPRESSION_BLOSC2) {   // compression.rs:29-57, oracle_blosc2.cpp
        u64 nbytes = 0, cbytes = 0, bsize = 0, got = 0;
        oracle_blosc2_sizes(chunk, len, &nbytes, &cbytes, &bsize);
        data.resize(nbytes ? nbytes : 1);
        const uint32_t e = nbytes ? oracle_blosc2_decompress(chunk, len, data.data(), nbytes, &got) : RDX_BLOSC2_INVALID;
        if (e != RDX_INFLATE_OK) {
            g_inflate_error = e;
            throw OracleError{e == RDX_BLOSC2_UNSUPPORTED ? RDX_E_UNSUPPORTED : RDX_E_DECOMPRESSION};
        }
        data.resize(got);
    } else if (req.compression != RDX_COMPRESSION_NONE) {
        throw OracleError{RDX_E_INVALID_ARGUMENT};
    } else {
        data.assign(chunk, chunk + len);
    }
    for (uint32_t k = req.n_filters; k-- > 0;) data = deshuffle(data, req.filters[k].element_size);
    // app.rs:169-172: the raw size is validated when compressed or when `size` was not given
    if (req.compression != RDX_COMPRESSION_NONE || !req.has_size) validate_raw_size(data.size(), req.dtype, req);
    return execute_dtype(req, data);
}

// operation.rs:78-96: runtime dtype -> NumOperation::execute_t::<T> (data owned, may be mutated)
Response execute_dtype(const rdx_request &req, std::vector<uint8_t> &data) {
    switch (req.dtype) {
        case RDX_DTYPE_INT32: return execute_t<int32_t>(req, data);
        case RDX_DTYPE_INT64: return execute_t<int64_t>(req, data);
        case RDX_DTYPE_UINT32: return execute_t<uint32_t>(req, data);
        case RDX_DTYPE_UINT64: return execute_t<uint64_t>(req, data);
        case RDX_DTYPE_FLOAT32: return execute_t<float>(req, data);
        case RDX_DTYPE_FLOAT64: return execute_t<double>(req, data);
        default: throw OracleError{RDX_E_INVALID_ARGUMENT};
    }
}

// ----------------------------------------------------------------------------------------------
// src/models.rs:179-313 request validation and src/types/missing.rs:47-80 / dvalue.rs:43-83
template <class T>
bool range_ok(const rdx_missing &m) {
    T lo, hi;
    std::memcpy(&lo, (const uint8_t *)m.values, sizeof(T));
    std::memcpy(&hi, (const uint8_t *)m.values + sizeof(T), sizeof(T));
    return lo < hi;  // `min >= max` is an error (missing.rs:58-68)
}

void validate_request(const rdx_request &req) {
    if (req.op > RDX_OP_SUM || req.dtype > RDX_DTYPE_FLOAT64) throw OracleError{RDX_E_INVALID_ARGUMENT};
    if (req.ndim > 0) {
        for (uint32_t k = 0; k < req.ndim; ++k)
            if (req.shape[k] == 0) throw OracleError{RDX_E_REQUEST_VALIDATION};  // validate_shape
    }
    if (req.selection) {
        if (req.ndim == 0) throw OracleError{RDX_E_REQUEST_VALIDATION};  // selection requires shape
        for (uint32_t k = 0; k < req.ndim; ++k)
            if (req.selection[k].stride == 0) throw OracleError{RDX_E_REQUEST_VALIDATION};
    }
    if (req.has_size) {
        if (req.size < 1) throw OracleError{RDX_E_REQUEST_VALIDATION};
        if (req.compression == RDX_COMPRESSION_NONE) validate_raw_size(req.size, req.dtype, req);
    }
    if (req.axes_kind == RDX_AXES_ONE || req.axes_kind == RDX_AXES_MULTI) {
        if (req.ndim == 0) throw OracleError{RDX_E_REQUEST_VALIDATION};
        const std::vector<u64> ax = axes_of(req);
        if (req.axes_kind == RDX_AXES_ONE) {
            if (ax[0] > req.ndim - 1) throw OracleError{RDX_E_REQUEST_VALIDATION};
        } else {
            if (ax.size() > req.ndim) throw OracleError{RDX_E_REQUEST_VALIDATION};
            std::vector<u64> sorted = ax;
            std::sort(sorted.begin(), sorted.end());
            if (sorted != ax) throw OracleError{RDX_E_REQUEST_VALIDATION};
            for (u64 a : ax)
                if (a > req.ndim - 1) throw OracleError{RDX_E_REQUEST_VALIDATION};
            for (size_t i = 1; i < ax.size(); ++i)
                if (ax[i] == ax[i - 1]) throw OracleError{RDX_E_REQUEST_VALIDATION};
        }
    }
    if (req.missing.kind == RDX_MISSING_VALID_RANGE) {
        bool ok = true;
        switch (req.dtype) {
            case RDX_DTYPE_INT32: ok = range_ok<int32_t>(req.missing); break;
            case RDX_DTYPE_INT64: ok = range_ok<int64_t>(req.missing); break;
            case RDX_DTYPE_UINT32: ok = range_ok<uint32_t>(req.missing); break;
            case RDX_DTYPE_UINT64: ok = range_ok<uint64_t>(req.missing); break;
            case RDX_DTYPE_FLOAT32: ok = range_ok<float>(req.missing); break;
            case RDX_DTYPE_FLOAT64: ok = range_ok<double>(req.missing); break;
        }
        if (!ok) throw OracleError{RDX_E_REQUEST_VALIDATION};
    }
}

}  // namespace

// ================================ exported (tests only) =========================================
extern "C" {

int oracle_execute(const rdx_request *req, const void *chunk, uint64_t len, void *body, uint64_t body_cap,
                   int64_t *counts, uint64_t counts_cap, rdx_response_info *info) {
    try {
        if (!req || (!chunk && len) || !info) return RDX_E_INVALID_ARGUMENT;
        Response r = operation(*req, static_cast<const uint8_t *>(chunk), len);
        std::memset(info, 0, sizeof(*info));
        info->dtype = r.dtype;
        info->ndim = (uint32_t)r.shape.size();
        for (size_t k = 0; k < r.shape.size() && k < RDX_MAX_NDIM; ++k) info->shape[k] = r.shape[k];
        info->body_bytes = r.body.size();
        info->n_counts = r.count.size();
        if (r.body.size() > body_cap || r.count.size() > counts_cap) return RDX_E_BUFFER_TOO_SMALL;
        if (!r.body.empty()) std::memcpy(body, r.body.data(), r.body.size());
        if (!r.count.empty()) std::memcpy(counts, r.count.data(), r.count.size() * sizeof(int64_t));
        return RDX_OK;
    } catch (const OracleError &e) {
        return e.status;
    } catch (...) {
        return RDX_E_OUT_OF_MEMORY;
    }
}

// Timing helper for bench.py's cpu_baseline legs: `reps` executions of one request over one chunk on
// the calling thread; *ns = elapsed wall nanoseconds.  clone = 1 copies the chunk into a fresh buffer
// every iteration, as the reference's criterion bench does (`data.clone()` inside the timed closure,
// benches/operations.rs:63); clone = 0 runs Operation::execute on one buffer prepared outside the loop
// (only for requests that do not mutate it: no filter, no compression, native byte order).
int oracle_bench(const rdx_request *req, const void *chunk, uint64_t len, uint64_t reps, int clone, uint64_t *ns) {
    try {
        if (!req || (!chunk && len) || !ns) return RDX_E_INVALID_ARGUMENT;
        if (!clone && (req->n_filters || req->compression != RDX_COMPRESSION_NONE ||
                       req->byte_order == RDX_BYTE_ORDER_BIG))
            return RDX_E_INVALID_ARGUMENT;
        const uint8_t *src = static_cast<const uint8_t *>(chunk);
        std::vector<uint8_t> once(src, src + len);
        volatile u64 sink = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t i = 0; i < reps; ++i) {
            Response r = clone ? operation(*req, src, len) : execute_dtype(*req, once);
            sink = sink + r.body.size();
        }
        *ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        return RDX_OK;
    } catch (const OracleError &e) {
        return e.status;
    } catch (...) {
        return RDX_E_OUT_OF_MEMORY;
    }
}

uint32_t oracle_inflate_last_error(void) { return g_inflate_error; }

int oracle_validate_request(const rdx_request *req) {
    try {
        validate_request(*req);
        return RDX_OK;
    } catch (const OracleError &e) {
        return e.status;
    }
}

void oracle_shuffle(const uint8_t *in, uint64_t len, uint64_t es, uint8_t *out) {
    std::vector<uint8_t> v(in, in + len);
    std::vector<uint8_t> r = shuffle(v, es);
    std::memcpy(out, r.data(), r.size());
}

int oracle_deshuffle(const uint8_t *in, uint64_t len, uint64_t es, uint8_t *out) {
    try {
        std::vector<uint8_t> v(in, in + len);
        std::vector<uint8_t> r = deshuffle(v, es);
        if (!r.empty()) std::memcpy(out, r.data(), r.size());
        return RDX_OK;
    } catch (const OracleError &e) {
        return e.status;
    }
}

// src/types/dvalue.rs:43-83 TryFromDValue.  `kind`: 0 = JSON integer stored as i64,
// 1 = JSON integer stored as u64 (> i64::MAX), 2 = JSON float.  serde_json::Number::as_i64/as_u64
// return None for floats; as_f64 always succeeds.
int oracle_missing_convert(uint32_t dtype, uint32_t kind, int64_t iv, uint64_t uv, double fv, void *out) {
    auto as_i64 = [&](int64_t &r) {
        if (kind == 0) { r = iv; return true; }
        return false;  // u64 > i64::MAX or float
    };
    auto as_u64 = [&](uint64_t &r) {
        if (kind == 0) { if (iv < 0) return false; r = (uint64_t)iv; return true; }
        if (kind == 1) { r = uv; return true; }
        return false;
    };
    auto as_f64 = [&]() -> double { return kind == 0 ? (double)iv : kind == 1 ? (double)uv : fv; };
    switch (dtype) {
        case RDX_DTYPE_INT32: {
            int64_t v;
            if (!as_i64(v) || v < INT32_MIN || v > INT32_MAX) return RDX_E_INCOMPATIBLE_MISSING;
            int32_t x = (int32_t)v; std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_INT64: {
            int64_t v;
            if (!as_i64(v)) return RDX_E_INCOMPATIBLE_MISSING;
            std::memcpy(out, &v, 8); return RDX_OK;
        }
        case RDX_DTYPE_UINT32: {
            uint64_t v;
            if (!as_u64(v) || v > UINT32_MAX) return RDX_E_INCOMPATIBLE_MISSING;
            uint32_t x = (uint32_t)v; std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_UINT64: {
            uint64_t v;
            if (!as_u64(v)) return RDX_E_INCOMPATIBLE_MISSING;
            std::memcpy(out, &v, 8); return RDX_OK;
        }
        case RDX_DTYPE_FLOAT32: {
            float x = (float)as_f64();
            if (!std::isfinite(x)) return RDX_E_INCOMPATIBLE_MISSING;
            std::memcpy(out, &x, 4); return RDX_OK;
        }
        case RDX_DTYPE_FLOAT64: {
            double x = as_f64();
            std::memcpy(out, &x, 8); return RDX_OK;
        }
    }
    return RDX_E_INVALID_ARGUMENT;
}

}  // extern "C"
