// Response serialisation, host side: the fixed segments of the CBOR body (rdx_cbor.hpp) and the
// host-buffer encoder rdx_cbor_encode.  The device encoder (rdx_cbor_encode_device) is in
// rdx_runtime.cpp / k_cbor.hip and writes the same bytes.
#include "rdx_cbor.hpp"

#include <cstring>

namespace rdx {
namespace {

void head(std::vector<uint8_t> &o, uint8_t major, uint64_t u) {
    uint8_t tmp[9];
    if (u < 24) {
        o.push_back((uint8_t)((major << 5) | u));
        return;
    }
    const int n = u <= 0xffu ? 1 : u <= 0xffffu ? 2 : u <= 0xffffffffull ? 4 : 8;
    tmp[0] = (uint8_t)((major << 5) | (n == 1 ? 24 : n == 2 ? 25 : n == 4 ? 26 : 27));
    for (int i = 0; i < n; ++i) tmp[1 + i] = (uint8_t)(u >> (8 * (n - 1 - i)));
    o.insert(o.end(), tmp, tmp + 1 + n);
}

void text(std::vector<uint8_t> &o, const char *s) {
    const size_t n = std::strlen(s);
    head(o, 3, n);
    o.insert(o.end(), s, s + n);
}

// DType's Display, lower-cased (models.rs:403: response.dtype.to_string().to_lowercase())
const char *dtype_name(uint32_t d) {
    switch (d) {
        case RDX_DTYPE_INT32: return "int32";
        case RDX_DTYPE_INT64: return "int64";
        case RDX_DTYPE_UINT32: return "uint32";
        case RDX_DTYPE_UINT64: return "uint64";
        case RDX_DTYPE_FLOAT32: return "float32";
        case RDX_DTYPE_FLOAT64: return "float64";
        default: return nullptr;
    }
}

}  // namespace

rdx_status cbor_layout(const rdx_response_info &info, uint32_t flags, CborLayout &L) {
    const char *dn = dtype_name(info.dtype);
    if (!dn || info.ndim > RDX_MAX_NDIM || (flags & ~(RDX_CBOR_SHAPE_AS_BYTES | RDX_CBOR_COUNT_AS_BYTES)))
        return RDX_E_INVALID_ARGUMENT;
    L = CborLayout{};
    L.body_len = info.body_bytes;
    L.n_counts = info.n_counts;
    const bool shape_bytes = flags & RDX_CBOR_SHAPE_AS_BYTES, count_bytes = flags & RDX_CBOR_COUNT_AS_BYTES;
    // A: CBORResponse has 7 fields (models.rs:355-370)
    head(L.a, 5, 7);
    text(L.a, "bytes");
    head(L.a, 2, info.body_bytes);
    // B
    text(L.b, "dtype");
    text(L.b, dn);
    text(L.b, "shape");
    if (shape_bytes) {
        head(L.b, 4, 0);
        text(L.b, "shape_as_bytes");
        head(L.b, 2, 8ull * info.ndim);
        for (uint32_t k = 0; k < info.ndim; ++k) {   // (s as u64).to_ne_bytes(): little-endian on x86
            const uint64_t s = info.shape[k];
            for (int i = 0; i < 8; ++i) L.b.push_back((uint8_t)(s >> (8 * i)));
        }
    } else {
        head(L.b, 4, info.ndim);
        for (uint32_t k = 0; k < info.ndim; ++k) head(L.b, 0, info.shape[k]);   // usize -> serialize_u64
        text(L.b, "shape_as_bytes");
        head(L.b, 2, 0);
    }
    text(L.b, "count");
    head(L.b, 4, count_bytes ? 0 : info.n_counts);
    L.count_array = !count_bytes && info.n_counts > 0;
    L.count_raw = count_bytes && info.n_counts > 0;
    // D
    text(L.d, "count_as_bytes");
    head(L.d, 2, count_bytes ? 8 * info.n_counts : 0);
    // F: NATIVE_BYTE_ORDER (types/byte_order.rs) is little on every host this engine runs on
    text(L.f, "byte_order");
    text(L.f, "little");
    return RDX_OK;
}

}  // namespace rdx

using namespace rdx;

extern "C" uint64_t rdx_cbor_bound(const rdx_response_info *info, uint32_t flags) {
    CborLayout L;
    if (!info || cbor_layout(*info, flags, L)) return 0;
    return L.fixed() + (L.count_array ? 9 * L.n_counts : 0);
}

extern "C" rdx_status rdx_cbor_encode(const rdx_response_info *info, const void *body, const int64_t *counts,
                                      uint32_t flags, void *out, uint64_t out_cap, uint64_t *out_len) {
    if (!info || !out_len) return RDX_E_INVALID_ARGUMENT;
    CborLayout L;
    if (rdx_status st = cbor_layout(*info, flags, L)) return st;
    if ((L.body_len && !body) || (L.n_counts && !counts)) return RDX_E_INVALID_ARGUMENT;
    uint64_t clen = 0;
    if (L.count_array)
        for (uint64_t i = 0; i < L.n_counts; ++i) clen += cbor_int_len(counts[i]);
    const uint64_t total = L.fixed() + clen;
    *out_len = total;
    if (out_cap < total || !out) return RDX_E_BUFFER_TOO_SMALL;
    uint8_t *p = static_cast<uint8_t *>(out);
    auto put = [&](const void *src, uint64_t n) {
        if (n) std::memcpy(p, src, n);
        p += n;
    };
    put(L.a.data(), L.a.size());
    put(body, L.body_len);
    put(L.b.data(), L.b.size());
    if (L.count_array)
        for (uint64_t i = 0; i < L.n_counts; ++i) p += cbor_put_int(p, counts[i]);
    put(L.d.data(), L.d.size());
    if (L.count_raw) put(counts, 8 * L.n_counts);   // c.to_ne_bytes() (models.rs:383-385)
    put(L.f.data(), L.f.size());
    return RDX_OK;
}
