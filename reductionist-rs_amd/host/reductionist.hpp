// C++ host mirror of reductionist-rs's operation/plugin interface, above the C ABI (include/rdx.h).
//
// The reference is Rust and its toolchain is not available here, so the host side of the drop-in is
// written in C++ with the reference's names, argument meaning and error behaviour:
//   RequestData / DType / Order / Slice / Filter / Compression / ReductionAxes  src/models.rs:14-176
//   RequestData::validate()                                                     src/models.rs:179-313
//   Missing + DValue (serde_json::Number) + TryFromDValue                       src/types/missing.rs,
//                                                                               src/types/dvalue.rs
//   Response                                                                    src/models.rs:316-351
//   ActiveStorageError (+ http_status)                                          src/error.rs:30-376
//   Operation<...>::execute(const RequestData&, std::vector<uint8_t>)           src/operation.rs:53-66
//   Count / Max / Min / Select / Sum                                            src/operations.rs
//   operation<Op>(RequestData, data)                                            src/app.rs:163-183
// Header-only; link with librdx.so.  All compute runs on the MI355X through rdx_execute().
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <variant>
#include <vector>

#include "../../include/rdx.h"

namespace reductionist {

enum class DType { Int32, Int64, Uint32, Uint64, Float32, Float64 };
enum class Order { C, F };
enum class ByteOrder { Big, Little };
enum class Compression { Blosc2, Gzip, Zlib };

inline size_t size_of(DType d) {  // models.rs:29-40
    return (d == DType::Int64 || d == DType::Uint64 || d == DType::Float64) ? 8 : 4;
}
inline const char *dtype_name(DType d) {
    static const char *n[] = {"int32", "int64", "uint32", "uint64", "float32", "float64"};
    return n[static_cast<int>(d)];
}

struct Slice {  // numpy [start, end, stride], models.rs:77-92
    int64_t start, end, stride;
};

struct Filter {  // models.rs:111-117
    enum class Id { Shuffle, ShuffleSimd } id;
    uint64_t element_size;
};

struct ReductionAxes {  // models.rs:122-127 (untagged: absent = All, n = One, [..] = Multi)
    enum class Kind { All, One, Multi } kind = Kind::All;
    std::vector<uint64_t> axes;
    static ReductionAxes all() { return {}; }
    static ReductionAxes one(uint64_t a) { return {Kind::One, {a}}; }
    static ReductionAxes multi(std::vector<uint64_t> a) { return {Kind::Multi, std::move(a)}; }
};

// serde_json::Number: PosInt/NegInt/Float (dvalue.rs:23)
using DValue = std::variant<int64_t, uint64_t, double>;

struct Missing {  // missing.rs:31-42
    enum class Kind { MissingValue, MissingValues, ValidMin, ValidMax, ValidRange } kind;
    std::vector<DValue> values;  // 1 value, a list, or {min, max}
};

// error.rs:30-130 — only the variants this path can raise, with error.rs:242-376's status.
class ActiveStorageError : public std::runtime_error {
  public:
    enum class Kind {
        RequestDataValidation,  // 400
        FromBytes,              // 500
        ShapeInvalid,           // 400
        IncompatibleMissing,    // 400
        ReferencePanic,         // the reference panics (shuffle assert, NaN order): connection drops
        Unsupported,            // blosc2: decompress on the host first (not on the device)
        Decompression,          // DecompressionFlate2 / DecompressionZune: 400 (error.rs:247-249)
        Device                  // 500
    };
    ActiveStorageError(Kind k, const std::string &what, rdx_status st = RDX_OK)
        : std::runtime_error(what), kind(k), status(st) {}
    int http_status() const {
        switch (kind) {
            case Kind::RequestDataValidation: case Kind::ShapeInvalid: case Kind::IncompatibleMissing:
            case Kind::Decompression: return 400;
            default: return 500;
        }
    }
    Kind kind;
    rdx_status status;
};

inline void check(rdx_status st) {
    using K = ActiveStorageError::Kind;
    switch (st) {
        case RDX_OK: return;
        case RDX_E_REQUEST_VALIDATION: throw ActiveStorageError(K::RequestDataValidation, "request data is not valid", st);
        case RDX_E_FROM_BYTES: throw ActiveStorageError(K::FromBytes, "failed to convert from bytes", st);
        case RDX_E_SHAPE_INVALID: throw ActiveStorageError(K::ShapeInvalid, "failed to create array from shape", st);
        case RDX_E_INCOMPATIBLE_MISSING: throw ActiveStorageError(K::IncompatibleMissing, "Incompatible value for missing", st);
        case RDX_E_DECOMPRESSION:  // compression.rs:166-190 messages where the reference pins them
            throw ActiveStorageError(K::Decompression, rdx_inflate_error_string(rdx_inflate_last_error()), st);
        case RDX_E_SHUFFLE_LENGTH: throw ActiveStorageError(K::ReferencePanic, "assertion `left == right` failed", st);
        case RDX_E_NAN_UNORDERED: throw ActiveStorageError(K::ReferencePanic, "unexpected undefined order error for min", st);
        case RDX_E_UNSUPPORTED: throw ActiveStorageError(K::Unsupported, "unsupported by the device engine", st);
        default: throw ActiveStorageError(K::Device, rdx_status_string(st), st);
    }
}

// TryFromDValue (dvalue.rs:43-83) through the C ABI: JSON number -> raw T bytes.
inline std::vector<uint8_t> dvalue_bytes(const DValue &v, DType dt) {
    uint8_t out[8];
    rdx_status st;
    const uint32_t d = static_cast<uint32_t>(dt);
    if (auto *i = std::get_if<int64_t>(&v)) st = rdx_missing_from_i64(d, *i, out);
    else if (auto *u = std::get_if<uint64_t>(&v)) st = rdx_missing_from_u64(d, *u, out);
    else st = rdx_missing_from_f64(d, std::get<double>(v), out);
    check(st);
    return std::vector<uint8_t>(out, out + size_of(dt));
}

struct RequestData {  // models.rs:133-176
    std::string interface_type = "s3";
    std::string url;
    DType dtype = DType::Int32;
    std::optional<ByteOrder> byte_order;
    std::optional<uint64_t> offset, size;
    std::optional<std::vector<uint64_t>> shape;
    ReductionAxes axis;
    std::optional<Order> order;
    std::optional<std::vector<Slice>> selection;
    std::optional<Compression> compression;
    std::optional<std::vector<Filter>> filters;
    std::optional<Missing> missing;
    std::optional<bool> option_disable_chunk_cache, option_shape_as_bytes, option_count_as_bytes;

    // models.rs field validators + validate_request_data (:179-313); missing conversion errors
    // surface as validation errors like Missing::validate (missing.rs:47-80).
    void validate() const {
        using K = ActiveStorageError::Kind;
        if (interface_type.empty()) throw ActiveStorageError(K::RequestDataValidation, "interface type must not be empty");
        if (shape && shape->empty()) throw ActiveStorageError(K::RequestDataValidation, "shape length must be greater than 0");
        if (selection && selection->empty())
            throw ActiveStorageError(K::RequestDataValidation, "selection length must be greater than 0");
        if (shape && selection && shape->size() != selection->size())
            throw ActiveStorageError(K::RequestDataValidation, "Shape and selection must have the same length");
        Marshalled m;
        try {
            m = marshal(RDX_OP_SUM);
        } catch (const ActiveStorageError &e) {
            if (e.kind == K::IncompatibleMissing)
                throw ActiveStorageError(K::RequestDataValidation, std::string("Missing data descriptor is invalid: ") + e.what());
            throw;
        }
        check(rdx_validate_request(&m.req));
    }

    // Plain-C view of this request for the ABI (owns the arrays rdx_request points into).
    struct Marshalled {
        rdx_request req{};
        std::vector<rdx_slice> sel;
        std::vector<rdx_filter> fl;
        std::vector<uint8_t> miss;
        std::vector<uint64_t> axes;
    };
    Marshalled marshal(rdx_op op) const {
        Marshalled m;
        rdx_request &r = m.req;
        r.abi_version = RDX_ABI_VERSION;
        r.op = op;
        r.dtype = static_cast<uint32_t>(dtype);
        r.byte_order = !byte_order ? RDX_BYTE_ORDER_UNSET : *byte_order == ByteOrder::Big ? RDX_BYTE_ORDER_BIG
                                                                                            : RDX_BYTE_ORDER_LITTLE;
        r.order = !order ? RDX_ORDER_UNSET : *order == Order::F ? RDX_ORDER_F : RDX_ORDER_C;
        if (shape) {
            r.ndim = static_cast<uint32_t>(shape->size());
            r.shape = shape->data();
        }
        if (selection) {
            for (const Slice &s : *selection) m.sel.push_back({s.start, s.end, s.stride});
            r.selection = m.sel.data();
        }
        m.axes = axis.axes;
        r.axes_kind = axis.kind == ReductionAxes::Kind::All ? RDX_AXES_ALL
                      : axis.kind == ReductionAxes::Kind::One ? RDX_AXES_ONE : RDX_AXES_MULTI;
        r.n_axes = static_cast<uint32_t>(m.axes.size());
        r.axes = m.axes.empty() ? nullptr : m.axes.data();
        if (filters) {
            for (const Filter &f : *filters)
                m.fl.push_back({f.id == Filter::Id::Shuffle ? (uint32_t)RDX_FILTER_SHUFFLE : (uint32_t)RDX_FILTER_SHUFFLE_SIMD, 0,
                                f.element_size});
            r.n_filters = static_cast<uint32_t>(m.fl.size());
            r.filters = m.fl.data();
        }
        r.compression = !compression ? RDX_COMPRESSION_NONE
                        : *compression == Compression::Gzip ? RDX_COMPRESSION_GZIP
                        : *compression == Compression::Zlib ? RDX_COMPRESSION_ZLIB : RDX_COMPRESSION_BLOSC2;
        if (missing) {
            static const uint32_t kinds[] = {RDX_MISSING_VALUE, RDX_MISSING_VALUES, RDX_MISSING_VALID_MIN,
                                             RDX_MISSING_VALID_MAX, RDX_MISSING_VALID_RANGE};
            r.missing.kind = kinds[static_cast<int>(missing->kind)];
            for (const DValue &v : missing->values) {
                std::vector<uint8_t> b = dvalue_bytes(v, dtype);
                m.miss.insert(m.miss.end(), b.begin(), b.end());
            }
            r.missing.n_values = missing->values.size();
            r.missing.values = m.miss.empty() ? nullptr : m.miss.data();
        }
        if (size) {
            r.has_size = 1;
            r.size = *size;
        }
        return m;
    }
};

struct Response {  // models.rs:316-351
    std::vector<uint8_t> body;
    DType dtype;
    std::vector<uint64_t> shape;
    std::vector<int64_t> count;
    bool option_shape_as_bytes = false;
    bool option_count_as_bytes = false;
};

// The device pool (rdx_context).  One per process; thread-safe.
class Engine {
  public:
    explicit Engine(const std::vector<int> &devices = {}) {
        check(rdx_context_create(devices.empty() ? nullptr : devices.data(), (int)devices.size(), &ctx_));
    }
    ~Engine() { rdx_context_destroy(ctx_); }
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;
    rdx_context *get() const { return ctx_; }

    static Engine &global() {
        static std::once_flag once;
        static std::unique_ptr<Engine> eng;
        std::call_once(once, [] { eng = std::make_unique<Engine>(); });
        return *eng;
    }

  private:
    rdx_context *ctx_ = nullptr;
};

// src/operation.rs:53-66 — `execute(request_data, data) -> Result<Response>`; errors are thrown.
// Unlike the reference's trait (which receives filter-decoded bytes from operation<T>()), this
// executes the whole synchronous pipeline on the device: pass the chunk as downloaded (gzip/zlib
// compressed or not, shuffled or not).
template <rdx_op OP>
struct Operation {
    static Response execute(const RequestData &rd, const std::vector<uint8_t> &data, Engine &eng = Engine::global()) {
        RequestData::Marshalled m = rd.marshal(OP);
        rdx_response_info info{};
        if (rd.compression) {
            // the response size depends on the decompressed length: a call without output capacity
            // inflates on the device and reports it (RDX_E_BUFFER_TOO_SMALL with `info` filled)
            const rdx_status st = rdx_execute(eng.get(), &m.req, data.data(), data.size(), nullptr, 0, nullptr, 0, &info);
            if (st != RDX_E_BUFFER_TOO_SMALL) check(st);
        } else {
            check(rdx_plan(&m.req, data.size(), &info));
        }
        Response r;
        r.body.resize(info.body_bytes);
        r.count.resize(info.n_counts);
        check(rdx_execute(eng.get(), &m.req, data.data(), data.size(), r.body.data(), r.body.size(), r.count.data(),
                          r.count.size(), &info));
        r.dtype = static_cast<DType>(info.dtype);
        r.shape.assign(info.shape, info.shape + info.ndim);
        r.option_shape_as_bytes = rd.option_shape_as_bytes.value_or(false);
        r.option_count_as_bytes = rd.option_count_as_bytes.value_or(false);
        return r;
    }
};

using Count = Operation<RDX_OP_COUNT>;
using Max = Operation<RDX_OP_MAX>;
using Min = Operation<RDX_OP_MIN>;
using Select = Operation<RDX_OP_SELECT>;
using Sum = Operation<RDX_OP_SUM>;

// src/app.rs:163-183 operation<T>(request_data, data): validate_raw_size / filters / execute.
template <class Op>
Response operation(const RequestData &rd, const std::vector<uint8_t> &data, Engine &eng = Engine::global()) {
    return Op::execute(rd, data, eng);
}

}  // namespace reductionist
