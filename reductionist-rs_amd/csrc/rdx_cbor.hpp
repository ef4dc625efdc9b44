// Response serialisation (include/rdx.h rdx_cbor_*): the byte layout of
// serde_cbor::to_vec(&CBORResponse::new(&response)) (src/app.rs:33-40, src/models.rs:355-416).
//
// serde_cbor 0.11.2 writes a #[derive(Serialize)] struct as a definite-length map keyed by the field
// names (text strings) in declaration order; `Bytes` through serialize_bytes (major type 2), `String` /
// `&str` as text (major 3), `Vec<usize>` / `Vec<i64>` as definite arrays (major 4) of integers; every
// integer head in its shortest form (value < 24 in the initial byte, else 1 / 2 / 4 / 8 following bytes,
// big-endian), a negative i64 v as major 1 with -1 - v.
//
// Layout of one response, in order:
//   A  map(7), "bytes", bstr head(body_len)                    host-known
//      body bytes                                               copied
//   B  "dtype", tstr, "shape", array | [], "shape_as_bytes", bstr(shape u64s) | h'', "count",
//      array head(n) | []                                       host-known
//   C  the count array's integers                               variable: encoded per count
//   D  "count_as_bytes", bstr head(8n) | h''                    host-known
//   E  the counts' native-endian i64 bytes (count_as_bytes)    copied
//   F  "byte_order", "little"                                   host-known
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/rdx.h"

namespace rdx {

// Encoded length of one i64 as a CBOR integer (major 0 / 1, shortest head).
inline uint32_t cbor_int_len(int64_t v) {
    const uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) : (uint64_t)v;
    return u < 24 ? 1u : u <= 0xffu ? 2u : u <= 0xffffu ? 3u : u <= 0xffffffffull ? 5u : 9u;
}

// Writes one i64 as a CBOR integer at p; returns the bytes written.
inline uint32_t cbor_put_int(uint8_t *p, int64_t v) {
    const uint8_t major = v < 0 ? 0x20 : 0x00;
    const uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) : (uint64_t)v;
    if (u < 24) {
        p[0] = (uint8_t)(major | u);
        return 1;
    }
    const int n = u <= 0xffu ? 1 : u <= 0xffffu ? 2 : u <= 0xffffffffull ? 4 : 8;
    p[0] = (uint8_t)(major | (n == 1 ? 24 : n == 2 ? 25 : n == 4 ? 26 : 27));
    for (int i = 0; i < n; ++i) p[1 + i] = (uint8_t)(u >> (8 * (n - 1 - i)));
    return 1u + (uint32_t)n;
}

struct CborLayout {
    std::vector<uint8_t> a, b, d, f;   // the host-known segments
    uint64_t body_len = 0;
    uint64_t n_counts = 0;
    bool count_array = false;          // C present (count not as bytes)
    bool count_raw = false;            // E present (count as bytes)
    uint64_t body_off() const { return a.size(); }
    uint64_t b_off() const { return a.size() + body_len; }
    uint64_t c_off() const { return b_off() + b.size(); }
    // size of everything but C
    uint64_t fixed() const { return a.size() + body_len + b.size() + d.size() + (count_raw ? 8 * n_counts : 0) + f.size(); }
};

// RDX_E_INVALID_ARGUMENT for an info that no plan produces (dtype out of range, ndim > RDX_MAX_NDIM).
rdx_status cbor_layout(const rdx_response_info &info, uint32_t flags, CborLayout &L);

}  // namespace rdx
