// Tests of the C++ host mirror (reductionist-rs_amd/host/reductionist.hpp), written like the
// reference's own unit tests.  `test_host cpu` needs no device; `test_host gpu` runs operations.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>

#include "../../reductionist-rs_amd/host/reductionist.hpp"

using namespace reductionist;

static int failures = 0;
#define EXPECT(c)                                                             \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

template <class F>
static ActiveStorageError::Kind error_kind(F &&f) {
    try {
        f();
    } catch (const ActiveStorageError &e) {
        return e.kind;
    }
    return static_cast<ActiveStorageError::Kind>(-1);
}

template <class T>
static std::vector<uint8_t> bytes_of(std::initializer_list<T> v) {
    std::vector<uint8_t> b(v.size() * sizeof(T));
    std::memcpy(b.data(), v.begin(), b.size());
    return b;
}

template <class T>
static T scalar(const Response &r) {
    T v;
    std::memcpy(&v, r.body.data(), sizeof(T));
    return v;
}

static void cpu_tests() {
    using K = ActiveStorageError::Kind;
    RequestData ok;
    ok.dtype = DType::Float32;
    ok.shape = std::vector<uint64_t>{2, 3};
    ok.selection = std::vector<Slice>{{0, 2, 1}, {0, 3, 2}};
    ok.axis = ReductionAxes::multi({0, 1});
    ok.size = 24;
    ok.missing = Missing{Missing::Kind::ValidRange, {DValue(-1.0), DValue(1.0)}};
    ok.validate();

    // models.rs validators
    RequestData r = ok;
    r.shape = std::vector<uint64_t>{0, 3};
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // validate_shape
    r = ok;
    r.size = 12;
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // validate_raw_size
    r = ok;
    r.axis = ReductionAxes::multi({1, 0});
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // ascending order
    r = ok;
    r.axis = ReductionAxes::one(2);
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // within shape
    r = ok;
    r.selection = std::vector<Slice>{{0, 2, 1}, {0, 3, 0}};
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // stride 0
    r = ok;
    r.missing = Missing{Missing::Kind::ValidRange, {DValue(42.0), DValue(42.0)}};
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // missing.rs:163-171
    r = ok;
    r.dtype = DType::Uint32;
    r.size = 24;
    r.missing = Missing{Missing::Kind::MissingValue, {DValue(int64_t(-1))}};
    EXPECT(error_kind([&] { r.validate(); }) == K::RequestDataValidation);  // missing.rs:144-149

    // models.rs:741-911 request-level validation (test_utils.rs:7-29 defaults: int32, nothing else)
    auto invalid = [](RequestData q) { return error_kind([&] { q.validate(); }) == K::RequestDataValidation; };
    RequestData d;
    d.validate();
    r = d;
    r.size = 1;
    EXPECT(invalid(r));                                                    // test_invalid_size_for_dtype
    r = d;
    r.size = 4;
    r.shape = std::vector<uint64_t>{1, 2};
    EXPECT(invalid(r));                                                    // test_invalid_size_for_shape
    r = d;
    r.shape = std::vector<uint64_t>{1, 2};
    r.selection = std::vector<Slice>{{1, 2, 1}};
    EXPECT(invalid(r));                                                    // test_shape_selection_mismatch
    r = d;
    r.selection = std::vector<Slice>{{1, 2, 1}};
    EXPECT(invalid(r));                                                    // test_selection_without_shape
    r = d;
    r.axis = ReductionAxes::one(1);
    EXPECT(invalid(r));                                                    // test_axis_without_shape
    r = d;
    r.shape = std::vector<uint64_t>{1, 2};
    r.axis = ReductionAxes::multi({1, 1});
    EXPECT(invalid(r));                                                    // test_axis_duplicates
    r = d;
    r.missing = Missing{Missing::Kind::MissingValue, {DValue(std::numeric_limits<int64_t>::max())}};
    EXPECT(invalid(r));                                                    // test_missing_invalid_value_for_dtype
    r = d;
    r.interface_type.clear();
    EXPECT(invalid(r));                                                    // test_invalid_interface_type
    for (Slice sl : {Slice{1, 0, 1}, Slice{1, 0, -1}, Slice{5, 5, 1}, Slice{-5, 5, 1}, Slice{1, -5, 1}}) {
        r = d;                                                             // models.rs:724-803: valid numpy slices
        r.shape = std::vector<uint64_t>{4};
        r.selection = std::vector<Slice>{sl};
        r.validate();
    }

    // dvalue.rs conversions
    EXPECT(dvalue_bytes(DValue(int64_t(42)), DType::Int32) == bytes_of<int32_t>({42}));
    EXPECT(error_kind([&] { dvalue_bytes(DValue(int64_t(1) << 31), DType::Int32); }) == K::IncompatibleMissing);
    EXPECT(error_kind([&] { dvalue_bytes(DValue(uint64_t(1) << 63), DType::Int64); }) == K::IncompatibleMissing);
    EXPECT(error_kind([&] { dvalue_bytes(DValue(1.0), DType::Int64); }) == K::IncompatibleMissing);
    EXPECT(dvalue_bytes(DValue(int64_t(42)), DType::Float32) == bytes_of<float>({42.0f}));
    EXPECT(error_kind([&] { dvalue_bytes(DValue(std::numeric_limits<float>::max() * 2.0), DType::Float32); }) ==
           K::IncompatibleMissing);
    EXPECT(ActiveStorageError(K::ShapeInvalid, "x").http_status() == 400);
    EXPECT(ActiveStorageError(K::FromBytes, "x").http_status() == 500);
}

static void gpu_tests() {
    using K = ActiveStorageError::Kind;
    RequestData rd;  // test_utils.rs:7-29
    // operations.rs:662-674 count_i32_1d
    Response c = Count::execute(rd, {1, 2, 3, 4, 5, 6, 7, 8});
    EXPECT(scalar<int64_t>(c) == 2 && c.dtype == DType::Int64 && c.shape.empty() && c.count == std::vector<int64_t>{2});
    // operations.rs:694-710 max_i64_1d
    rd.dtype = DType::Int64;
    EXPECT(scalar<int64_t>(Max::execute(rd, {1, 2, 3, 4, 5, 6, 7, 8})) == 0x0807060504030201);
    // operations.rs:964-975 sum_u32_1d
    rd.dtype = DType::Uint32;
    EXPECT(scalar<uint32_t>(Sum::execute(rd, {1, 2, 3, 4, 5, 6, 7, 8})) == 0x04030201u + 0x08070605u);
    // operations.rs:942-961 select_f32_2d_with_selection
    RequestData s;
    s.dtype = DType::Float32;
    s.shape = std::vector<uint64_t>{2, 2};
    s.selection = std::vector<Slice>{{0, 2, 1}, {1, 2, 1}};
    std::vector<uint8_t> d16;
    for (int i = 1; i <= 16; ++i) d16.push_back((uint8_t)i);
    Response sel = Select::execute(s, d16);
    EXPECT((sel.body == std::vector<uint8_t>{5, 6, 7, 8, 13, 14, 15, 16}) && (sel.shape == std::vector<uint64_t>{2, 1}));
    // operations.rs:829-842 min_f32_1d_nan (should_panic -> ReferencePanic)
    RequestData f;
    f.dtype = DType::Float32;
    EXPECT(error_kind([&] { Min::execute(f, bytes_of<float>({1.0f, NAN})); }) == K::ReferencePanic);
    // operations.rs:1032-1050 sum_u32_1d_axis_0
    RequestData ax;
    ax.dtype = DType::Uint32;
    ax.shape = std::vector<uint64_t>{2, 4};
    ax.axis = ReductionAxes::one(0);
    Response sa = Sum::execute(ax, bytes_of<uint32_t>({1, 2, 3, 4, 5, 6, 7, 8}));
    EXPECT(sa.body == bytes_of<uint32_t>({6, 8, 10, 12}) && (sa.count == std::vector<int64_t>{2, 2, 2, 2}));
    // filter pipeline + byte order through app.rs operation<T>
    RequestData p;
    p.dtype = DType::Uint32;
    p.byte_order = ByteOrder::Big;
    p.filters = std::vector<Filter>{{Filter::Id::Shuffle, 4}};
    std::vector<uint8_t> be = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 2, 3, 4};  // shuffle of BE [1,2,3,4]
    Response ps = operation<Sum>(p, be);
    EXPECT(scalar<uint32_t>(ps) == 10u);
    // array.rs:271-273 from_bytes_u32_too_small (size given -> FromBytes)
    RequestData fb;
    fb.dtype = DType::Uint32;
    fb.size = 3;
    EXPECT(error_kind([&] { Sum::execute(fb, {1, 2, 3}); }) == K::FromBytes);
    // filter_pipeline.rs:70-77: a gzip chunk is inflated on the device (stream of bytes 1..8, frozen)
    RequestData gz;
    gz.dtype = DType::Uint32;
    gz.compression = Compression::Gzip;
    const std::vector<uint8_t> gzs = {0x1f, 0x8b, 0x08, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x03, 0x63, 0x64, 0x62, 0x66, 0x61, 0x65, 0x63, 0xe7, 0x00, 0x00, 0xc5, 0x88, 0xca, 0x3f, 0x08, 0x00, 0x00, 0x00};
    EXPECT(scalar<uint32_t>(Sum::execute(gz, gzs)) == 0x04030201u + 0x08070605u);
    // compression.rs:165-176: b"invalid format" -> DecompressionFlate2 "invalid gzip header" (400)
    const std::string bad = "invalid format";
    try {
        Sum::execute(gz, std::vector<uint8_t>(bad.begin(), bad.end()));
        EXPECT(false);
    } catch (const ActiveStorageError &e) {
        EXPECT(e.kind == K::Decompression && e.http_status() == 400 && std::string(e.what()) == "invalid gzip header");
    }
}

int main(int argc, char **argv) {
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    cpu_tests();
    if (gpu) gpu_tests();
    std::printf("%s: %d failure(s)\n", gpu ? "cpu+gpu" : "cpu", failures);
    return failures ? 1 : 0;
}
