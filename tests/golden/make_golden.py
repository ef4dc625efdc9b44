#!/usr/bin/env python3
"""Generate tests/golden/kats.json: known-answer vectors TRANSCRIBED from reductionist-rs's own
#[cfg(test)] modules (the reference is Rust and cannot be built or run here; these inputs and
expected outputs are the data those tests assert).  Each vector cites the reference test it comes
from.  Re-run:  python tests/golden/make_golden.py

Conventions for turning a unit-level assertion into an end-to-end request:
  * function-level tests on an ndarray (operations.rs *_multi_axis tests) become requests whose raw
    chunk is the array's memory image (i64 little-endian; `(0..n).collect()` in those tests), shape
    and axes as in the test.  The *_f_order variants pass order=F to the function but build a C-order
    array, so the equivalent request ships the F-order memory image of the same logical array.
  * array.rs view/slicing tests become Select requests (Select returns the view's elements in logical
    order for standard-layout arrays) or axis reductions that expose the logical layout.
  * "should_panic" tests expect the status the C ABI returns instead of the panic.
"""
import json
import struct
from pathlib import Path

import numpy as np

OUT = Path(__file__).with_name("kats.json")

FMT = {"int32": "<i4", "int64": "<i8", "uint32": "<u4", "uint64": "<u8", "float32": "<f4", "float64": "<f8"}


def b(x, dtype):
    return np.asarray(x, dtype=FMT[dtype]).tobytes().hex()


def raw(seq):
    return bytes(seq).hex()


KATS = []


def op(name, ref, opname, data_hex, expect, **req):
    KATS.append({"kind": "op", "name": name, "ref": ref, "op": opname, "request": req, "data": data_hex,
                 "expect": expect})


def ok(body_hex, dtype, shape, count):
    return {"status": "ok", "body": body_hex, "dtype": dtype, "shape": shape, "count": count}


def err(status):
    return {"status": status}


# ---- filters/shuffle.rs, shuffle_simd.rs, filters.rs, filter_pipeline.rs --------------------------
for src in ("src/filters/shuffle.rs", "src/filters/shuffle_simd.rs"):
    base = 92 if "simd" not in src else 33
    KATS.append({"kind": "deshuffle", "name": f"{src}:deshuffle_2", "ref": f"{src}:{base}-98", "es": 2,
                 "input": [0, 2, 4, 6, 1, 3, 5, 7], "output": [0, 1, 2, 3, 4, 5, 6, 7]})
    KATS.append({"kind": "deshuffle", "name": f"{src}:deshuffle_4", "ref": f"{src}:{base + 9}-107", "es": 4,
                 "input": [0, 4, 1, 5, 2, 6, 3, 7], "output": [0, 1, 2, 3, 4, 5, 6, 7]})
    KATS.append({"kind": "deshuffle", "name": f"{src}:deshuffle_8", "ref": f"{src}:{base + 18}-116", "es": 8,
                 "input": [0, 8, 1, 9, 2, 10, 3, 11, 4, 12, 5, 13, 6, 14, 7, 15], "output": list(range(16))})
KATS.append({"kind": "shuffle", "name": "shuffle_4", "ref": "src/filters/shuffle.rs:138-144", "es": 4,
             "input": list(range(8)), "output": [0, 4, 1, 5, 2, 6, 3, 7]})
KATS.append({"kind": "shuffle", "name": "shuffle_8", "ref": "src/filters/shuffle.rs:147-153", "es": 8,
             "input": list(range(16)), "output": [0, 8, 1, 9, 2, 10, 3, 11, 4, 12, 5, 13, 6, 14, 7, 15]})

# decode / pipeline round trips, observed through Select on uint8-compatible data: [1..8] as 2 x u32
one_to_8 = list(range(1, 9))
shuf4 = [1, 5, 2, 6, 3, 7, 4, 8]                      # shuffle([1..8], 4)
shuf4_2 = [1, 2, 3, 4, 5, 6, 7, 8]
# shuffle(shuffle([1..8],4),2): shuffle([1,5,2,6,3,7,4,8],2) = even bytes then odd bytes
shuf4_2 = [1, 2, 3, 4, 5, 6, 7, 8]
_s = [1, 5, 2, 6, 3, 7, 4, 8]
shuf4_2 = _s[0::2] + _s[1::2]
for fid, ref in (("shuffle", "src/filters.rs:32-39"), ("shuffle_simd", "src/filters.rs:42-50")):
    op(f"decode_{fid}", ref, "select", raw(shuf4), ok(raw(one_to_8), "uint32", [2], [2]), dtype="uint32",
       filters=[{"id": fid, "element_size": 4}])
op("filter_pipeline_noop", "src/filter_pipeline.rs:61-67", "select", raw([1, 2, 3, 4]),
   ok(raw([1, 2, 3, 4]), "uint32", [1], [1]), dtype="uint32")
op("filter_pipeline_shuffle", "src/filter_pipeline.rs:80-88", "select", raw(shuf4),
   ok(raw(one_to_8), "uint32", [2], [2]), dtype="uint32", filters=[{"id": "shuffle", "element_size": 4}])
# Compressed pipelines.  The reference compresses with flate2 Compression::fast() inside the test; any
# valid DEFLATE encoder's stream of the same bytes must decode identically, so the streams below come
# from CPython's zlib (level 1) and are FROZEN in kats.json as data (hex) — re-running this script
# with another zlib may change the stream bytes, never the decoded result.
import zlib  # noqa: E402


def _gz(data):
    c = zlib.compressobj(1, zlib.DEFLATED, 31)
    return c.compress(bytes(data)) + c.flush()


def _zl(data):
    c = zlib.compressobj(1, zlib.DEFLATED, 15)
    return c.compress(bytes(data)) + c.flush()


op("filter_pipeline_gzip", "src/filter_pipeline.rs:70-77", "select", _gz([1, 2, 3, 4]).hex(),
   ok(raw([1, 2, 3, 4]), "uint32", [1], [1]), dtype="uint32", compression="gzip", size=4)
op("filter_pipeline_shuffle_zlib", "src/filter_pipeline.rs:91-101", "select", _zl(shuf4).hex(),
   ok(raw(one_to_8), "uint32", [2], [2]), dtype="uint32", compression="zlib",
   filters=[{"id": "shuffle", "element_size": 4}])
op("filter_pipeline_shuffle_x2_zlib", "src/filter_pipeline.rs:104-120", "select", _zl(shuf4_2).hex(),
   ok(raw(one_to_8), "uint32", [2], [2]), dtype="uint32", compression="zlib",
   filters=[{"id": "shuffle", "element_size": 4}, {"id": "shuffle", "element_size": 2}])
# compression.rs:136-162 decompress b"hello world": the API has no 8-bit dtype, so the 11 decoded
# bytes are observed through validate_raw_size (11 is not a multiple of 4 -> 400) and, repeated 4
# times (44 bytes), through Select as 11 u32 words
op("decompress_gzip_hello_world -> raw size 11", "src/compression.rs:143-150 + src/app.rs:169-172", "count",
   _gz(b"hello world").hex(), err("E_REQUEST_VALIDATION"), dtype="uint32", compression="gzip")
op("decompress_zlib_hello_world_x4 (44 bytes = 11 x u32)", "src/compression.rs:152-159", "select",
   _zl(b"hello world" * 4).hex(), ok((b"hello world" * 4).hex(), "uint32", [11], [11]), dtype="uint32",
   compression="zlib")
# compression.rs:166-190: b"invalid format" -> DecompressionFlate2 "invalid gzip header" /
# DecompressionZune "Unknown zlib compression method 9" (both HTTP 400)
op("decompress_invalid_gzip", "src/compression.rs:165-176", "count", b"invalid format".hex(),
   {"status": "E_DECOMPRESSION", "inflate_error": "INFLATE_GZIP_HEADER"}, dtype="uint32", compression="gzip")
op("decompress_invalid_zlib", "src/compression.rs:178-190", "count", b"invalid format".hex(),
   {"status": "E_DECOMPRESSION", "inflate_error": "INFLATE_ZLIB_METHOD"}, dtype="uint32", compression="zlib")

# ---- array.rs ----------------------------------------------------------------------------------------
for dt, val, ref in (("uint32", 42, "216-221"), ("uint64", 2 ** 64 - 1, "224-229"), ("int32", -42, "232-237"),
                     ("int64", -2 ** 63, "240-245"), ("float32", float(np.finfo(np.float32).min), "248-253"),
                     ("float64", float(np.finfo(np.float64).max), "256-261")):
    op(f"from_bytes_{dt}", f"src/array.rs:{ref}", "select", b([val], dt), ok(b([val], dt), dt, [1], [1]), dtype=dt)
op("from_bytes_u32_too_small", "src/array.rs:271-273", "select", raw([1, 2, 3]), err("E_FROM_BYTES"),
   dtype="uint32", size=3)
op("from_bytes_u32_too_big", "src/array.rs:276-278", "select", raw([1, 2, 3, 4, 5]), err("E_FROM_BYTES"),
   dtype="uint32", size=5)
op("build_array_from_shape_err", "src/array.rs:352-361", "select", b([1, 2, 3], "int32"),
   err("E_SHAPE_INVALID"), dtype="int32", shape=[4], size=12)
# logical layouts (array.rs:304-350): expose via select (standard layout: C order) and per-axis sums
layouts = [
    ("1d", [3], "C", [1, 2, 3], [1, 2, 3]),
    ("1d_fortran", [3], "F", [1, 2, 3], [1, 2, 3]),
    ("2d", [2, 3], "C", [1.0, 2.1, 3.2, 4.3, 5.4, 6.5], [[1.0, 2.1, 3.2], [4.3, 5.4, 6.5]]),
    ("2d_fortran", [2, 3], "F", [1.0, 2.1, 3.2, 4.3, 5.4, 6.5], [[1.0, 3.2, 5.4], [2.1, 4.3, 6.5]]),
    ("3d", [2, 2, 2], "C", list(range(1, 9)), [[[1, 2], [3, 4]], [[5, 6], [7, 8]]]),
    ("3d_fortran", [2, 2, 2], "F", list(range(1, 9)), [[[1, 5], [3, 7]], [[2, 6], [4, 8]]]),
]
lines = {"1d": "304-309", "1d_fortran": "312-317", "2d": "320-325", "2d_fortran": "328-333", "3d": "336-341",
         "3d_fortran": "344-349"}
for name, shape, order, data, logical in layouts:
    dt = "float64"
    L = np.asarray(logical, dtype=np.float64)
    for ax in range(len(shape)):
        mx = L.max(axis=ax)
        op(f"build_array_from_shape_{name}_max_axis{ax}", f"src/array.rs:{lines[name]}", "max", b(data, dt),
           ok(b(mx.ravel(), dt), dt, list(mx.shape), [shape[ax]] * int(mx.size)), dtype=dt, shape=shape,
           order=order, axis=[ax])
    std = order == "C" or sum(s != 1 for s in shape) <= 1
    sel = L.ravel(order="C" if std else "F")
    op(f"build_array_from_shape_{name}_select", f"src/array.rs:{lines[name]}", "select", b(data, dt),
       ok(b(sel, dt), dt, shape, [L.size]), dtype=dt, shape=shape, order=order)
op("reverse_array_byte_order_u32", "src/array.rs:486-495", "select", b([0, 42, 2 ** 32 - 1], "uint32"),
   ok(b([0, 42 << 24, 2 ** 32 - 1], "uint32"), "uint32", [3], [3]), dtype="uint32", byte_order="big")
op("build_array_1d_u32", "src/array.rs:498-504", "select", raw(one_to_8),
   ok(b([0x04030201, 0x08070605], "uint32"), "uint32", [2], [2]), dtype="uint32")
op("build_array_2d_i64", "src/array.rs:507-514", "select", raw([1, 2, 3, 4, 0, 0, 0, 0, 5, 6, 7, 8, 0, 0, 0, 0]),
   ok(b([0x04030201, 0x08070605], "int64"), "int64", [2, 1], [2]), dtype="int64", shape=[2, 1])
A, B = 0x04030201, 0x08070605
sel_cases = [  # array.rs:529-636 test_selection(slice, expected) on [A, B], shape [2]
    ("all", (0, 2, 1), [A, B], "529-534"), ("negative_start", (-2, 2, 1), [A, B], "537-542"),
    ("start_lt_negative_length", (-3, 2, 1), [A, B], "545-550"), ("start_eq_length", (2, 2, 1), [], "553-555"),
    ("start_gt_length", (3, 2, 1), [], "558-560"), ("negative_end", (0, -1, 1), [A], "563-565"),
    ("end_lt_negative_length", (0, -3, 1), [], "568-570"), ("end_gt_length", (0, 3, 1), [A, B], "573-578"),
    ("all_negative_stride", (1, -3, -1), [B, A], "581-588"),
    ("negative_start_negative_stride", (-1, -3, -1), [B, A], "591-597"),
    ("start_lt_negative_length_negative_stride", (-3, 0, -1), [], "600-603"),
    ("start_eq_length_negative_stride", (2, 1, -1), [], "606-609"),
    ("start_gt_length_negative_stride", (3, 1, -1), [], "612-615"),
    ("negative_end_negative_stride", (2, -1, -1), [], "618-621"),
    ("end_lt_negative_length_negative_stride", (1, -3, -1), [B, A], "624-630"),
    ("end_gt_length_negative_stride", (3, 0, -1), [B], "633-636"),
]
for name, s, exp, lines_ in sel_cases:
    op(f"build_array_with_selection_{name}", f"src/array.rs:{lines_}", "select", raw(one_to_8),
       ok(b(exp, "uint32"), "uint32", [len(exp)], [len(exp)]), dtype="uint32", shape=[2], selection=[list(s)])

# ---- operations.rs ------------------------------------------------------------------------------------
op("count_i32_1d", "src/operations.rs:662-674", "count", raw(one_to_8), ok(b([2], "int64"), "int64", [], [2]),
   dtype="int32")
op("count_u32_1d_missing_value", "src/operations.rs:677-691", "count", raw(one_to_8),
   ok(b([1], "int64"), "int64", [], [1]), dtype="uint32", missing={"missing_value": 0x04030201})
op("max_i64_1d", "src/operations.rs:694-710", "max", raw(one_to_8), ok(b([0x0807060504030201], "int64"), "int64", [], [1]),
   dtype="int64")
op("max_i64_1d_missing_values", "src/operations.rs:713-730", "max", raw(range(1, 17)),
   ok(b([0x100f0e0d0c0b0a09], "int64"), "int64", [], [1]), dtype="int64",
   missing={"missing_values": [0x0807060504030201]})
inf = float("inf")
op("max_f32_1d_infinity", "src/operations.rs:733-745", "max", b([1.0, inf], "float32"),
   ok(b([inf], "float32"), "float32", [], [2]), dtype="float32")
op("max_f32_1d_infinity_first", "src/operations.rs:748-760", "max", b([inf, 1.0], "float32"),
   ok(b([inf], "float32"), "float32", [], [2]), dtype="float32")
op("min_u64_1d", "src/operations.rs:763-774", "min", raw(one_to_8), ok(b([0x0807060504030201], "uint64"), "uint64", [], [1]),
   dtype="uint64")
op("min_i64_1d_valid_min", "src/operations.rs:777-795", "min", raw(range(1, 17)),
   ok(b([0x100f0e0d0c0b0a09], "int64"), "int64", [], [1]), dtype="int64", missing={"valid_min": 0x0807060504030202})
op("min_f32_1d_infinity", "src/operations.rs:798-810", "min", b([1.0, inf], "float32"),
   ok(b([1.0], "float32"), "float32", [], [2]), dtype="float32")
op("min_f32_1d_infinity_first", "src/operations.rs:813-825", "min", b([inf, 1.0], "float32"),
   ok(b([1.0], "float32"), "float32", [], [2]), dtype="float32")
nan = float("nan")
op("min_f32_1d_nan", "src/operations.rs:829-842 (should_panic)", "min", b([1.0, nan], "float32"),
   err("E_NAN_UNORDERED"), dtype="float32")
op("min_f32_1d_nan_first", "src/operations.rs:845-858 (should_panic)", "min", b([nan, 1.0], "float32"),
   err("E_NAN_UNORDERED"), dtype="float32")
op("min_f32_1d_nan_missing_value", "src/operations.rs:861-875 (should_panic)", "min", b([1.0, nan], "float32"),
   err("E_NAN_UNORDERED"), dtype="float32", missing={"missing_value": 42.0})
op("min_f32_1d_nan_first_missing_value", "src/operations.rs:878-892 (should_panic)", "min",
   b([nan, 1.0], "float32"), err("E_NAN_UNORDERED"), dtype="float32", missing={"missing_value": 42.0})
op("select_f32_1d", "src/operations.rs:895-906", "select", raw(one_to_8), ok(raw(one_to_8), "float32", [2], [2]),
   dtype="float32")
op("select_f32_1d_1ax (axis ignored)", "src/operations.rs:909-924", "select", raw(one_to_8),
   ok(raw(one_to_8), "float32", [2], [2]), dtype="float32", axis=[0])
op("select_f64_2d", "src/operations.rs:927-939", "select", raw(range(1, 17)), ok(raw(range(1, 17)), "float64", [2, 1], [2]),
   dtype="float64", shape=[2, 1])
op("select_f32_2d_with_selection", "src/operations.rs:942-961", "select", raw(range(1, 17)),
   ok(raw([5, 6, 7, 8, 13, 14, 15, 16]), "float32", [2, 1], [2]), dtype="float32", shape=[2, 2],
   selection=[[0, 2, 1], [1, 2, 1]])
op("sum_u32_1d", "src/operations.rs:964-975", "sum", raw(one_to_8), ok(b([0x04030201 + 0x08070605], "uint32"), "uint32", [], [2]),
   dtype="uint32")
op("sum_u32_1d_valid_max", "src/operations.rs:978-990", "sum", raw(one_to_8), ok(b([0x04030201], "uint32"), "uint32", [], [1]),
   dtype="uint32", missing={"valid_max": 0x08070605 - 1})
op("sum_f32_1d_infinity", "src/operations.rs:993-1005", "sum", b([1.0, inf], "float32"),
   ok(b([inf], "float32"), "float32", [], [2]), dtype="float32")
op("sum_f64_1d_nan (f64::NAN bits)", "src/operations.rs:1008-1020", "sum",
   struct.pack("<Qd", 0x7FF8000000000000, 1.0).hex(), ok(struct.pack("<Q", 0x7FF8000000000000).hex(), "float64", [], [2]),
   dtype="float64")
d = np.arange(1, 9, dtype=np.uint32)
op("sum_u32_1d_axis_0", "src/operations.rs:1032-1050", "sum", d.tobytes().hex(),
   ok(b(d.reshape(2, 4).sum(axis=0), "uint32"), "uint32", [4], [2, 2, 2, 2]), dtype="uint32", shape=[2, 4], axis=0)
d = np.array([0, 2, 3, 4, 5, 6, 7, 8], dtype=np.uint32)
op("sum_u32_1d_axis_1_missing", "src/operations.rs:1053-1072", "sum", d.tobytes().hex(),
   ok(b(d.reshape(2, 4).sum(axis=1), "uint32"), "uint32", [2], [3, 4]), dtype="uint32", shape=[2, 4], axis=1,
   missing={"missing_value": 0})
d = np.array([0, 2, 3, 4, 5, 6, 7, 8], dtype=np.float64)
op("sum_f64_1d_axis_1_missing", "src/operations.rs:1075-1095", "sum", d.tobytes().hex(),
   ok(b(d.reshape(2, 2, 2).sum(axis=1), "float64"), "float64", [2, 2], [1, 2, 2, 2]), dtype="float64",
   shape=[2, 2, 2], axis=1, missing={"missing_value": 0})

# *_multi_axis function tests (arrays from (0..n); i64 element type)
def arr(n):
    return np.arange(n, dtype=np.int64).tobytes().hex()


def i64(x):
    return b(x, "int64")


MA = [  # (name, lines, op, n, shape, axes, missing, body, count, shape_out)
    ("sum_multi_axis_2d_wrong_axis", "1112-1118", "sum", 4, [2, 2], [2], None, None, None, None),
    ("sum_multi_axis_2d_2ax", "1121-1130", "sum", 4, [2, 2], [0, 1], None, [6], [4], []),
    ("sum_multi_axis_2d_2ax_missing", "1133-1143", "sum", 4, [2, 2], [0, 1], {"missing_value": 1}, [5], [3], []),
    ("sum_multi_axis_2d_no_ax_some_missing", "1146-1159", "sum", 6, [2, 3], [], {"valid_max": 2},
     list(range(6)), [1, 1, 1, 0, 0, 0], [2, 3]),
    ("sum_multi_axis_4d_1ax", "1180-1189", "sum", 12, [2, 3, 2, 1], [2], None, [1, 5, 9, 13, 17, 21], [2] * 6,
     [2, 3, 1]),
    ("sum_multi_axis_4d_3ax", "1192-1201", "sum", 12, [2, 3, 2, 1], [0, 1, 3], None, [30, 36], [6, 6], [2]),
    ("min_multi_axis_2d_wrong_axis", "1205-1211", "min", 4, [2, 2], [2], None, None, None, None),
    ("min_multi_axis_2d_2ax", "1214-1227", "min", 6, [2, 3], [0, 1], None, [0], [6], []),
    ("min_multi_axis_2d_no_ax_some_missing", "1230-1243", "min", 6, [2, 3], [], {"valid_max": 2}, list(range(6)),
     [1, 1, 1, 0, 0, 0], [2, 3]),
    ("min_multi_axis_2d_1ax_missing", "1264-1277", "min", 6, [2, 3], [1], {"missing_value": 0}, [1, 3], [2, 3], [2]),
    ("min_multi_axis_4d_3ax_missing", "1280-1292", "min", 12, [2, 3, 2, 1], [0, 1, 3], {"missing_value": 1}, [0, 3],
     [6, 5], [2]),
    ("max_multi_axis_2d_wrong_axis", "1295-1303", "max", 4, [2, 2], [2], None, None, None, None),
    ("max_multi_axis_2d_2ax", "1306-1319", "max", 6, [2, 3], [0, 1], None, [5], [6], []),
    ("max_multi_axis_2d_no_ax_some_missing", "1322-1335", "max", 6, [2, 3], [], {"valid_max": 2}, list(range(6)),
     [1, 1, 1, 0, 0, 0], [2, 3]),
    ("max_multi_axis_2d_1ax_missing", "1356-1369", "max", 6, [2, 3], [1], {"missing_value": 0}, [2, 5], [2, 3], [2]),
    ("max_multi_axis_4d_3ax_missing", "1372-1386", "max", 12, [2, 3, 2, 1], [0, 1, 3], {"missing_value": 10}, [8, 11],
     [5, 6], [2]),
    ("count_multi_axis_2d_wrong_axis", "1389-1397", "count", 4, [2, 2], [2], None, None, None, None),
    ("count_multi_axis_2d_2ax", "1400-1412", "count", 6, [2, 3], [0, 1], None, [6], [6], []),
    ("count_multi_axis_2d_no_ax", "1415-1427", "count", 6, [2, 3], [], None, [1] * 6, [1] * 6, [2, 3]),
    ("count_multi_axis_2d_1ax_missing", "1430-1442", "count", 6, [2, 3], [1], {"missing_value": 0}, [2, 3], [2, 3],
     [2]),
    ("count_multi_axis_4d_3ax_multi_missing", "1445-1457", "count", 12, [2, 3, 2, 1], [0, 1, 3],
     {"missing_values": [9, 10, 11]}, [5, 4], [5, 4], [2]),
    ("count_multi_axis_4d_3ax_missing", "1460-1472", "count", 12, [2, 3, 2, 1], [0, 1, 3], {"missing_value": 10},
     [5, 6], [5, 6], [2]),
]
for name, lines_, opn, n, shape, axes, missing, body, count, shape_out in MA:
    req = dict(dtype="int64", shape=shape, axis=axes)
    if missing:
        req["missing"] = missing
    exp = err("E_REQUEST_VALIDATION") if body is None else ok(i64(body), "int64", shape_out, count)
    op(name, f"src/operations.rs:{lines_}", opn, arr(n), exp, **req)
# *_no_ax_some_missing_f_order: logical [[0,1,2],[3,4,5]] shipped as its F-order memory image
f_img = np.arange(6, dtype=np.int64).reshape(2, 3).ravel(order="F")
for opn, lines_ in (("sum", "1162-1177"), ("min", "1246-1261"), ("max", "1338-1353")):
    op(f"{opn}_multi_axis_2d_no_ax_some_missing_f_order", f"src/operations.rs:{lines_}", opn, f_img.tobytes().hex(),
       ok(i64([0, 3, 1, 4, 2, 5]), "int64", [2, 3], [1, 0, 1, 0, 1, 0]), dtype="int64", shape=[2, 3], order="F",
       axis=[], missing={"valid_max": 2})

# ---- types/missing.rs is_missing truth tables (via Count over axis=(), per-element 0/1) --------------
for name, lines_, missing, data, exp in (
        ("is_missing_value", "247-252", {"missing_value": 1}, [0, 1, 2], [1, 0, 1]),
        ("is_missing_values", "255-261", {"missing_values": [1, 2]}, [0, 1, 2, 3], [1, 0, 0, 1]),
        ("is_missing_valid_min", "264-269", {"valid_min": 1}, [0, 1, 2], [0, 1, 1]),
        ("is_missing_valid_max", "272-277", {"valid_max": 1}, [0, 1, 2], [1, 1, 0]),
        ("is_missing_valid_range", "280-286", {"valid_range": [1, 2]}, [0, 1, 2, 3], [0, 1, 1, 0])):
    op(name, f"src/types/missing.rs:{lines_}", "count", b(data, "int32"), ok(i64(exp), "int64", [len(data)], exp),
       dtype="int32", shape=[len(data)], axis=[], missing=missing)

# ---- types/dvalue.rs + missing.rs conversion (TryFromDValue) ------------------------------------------
CONV = [  # (dtype, json value, expected bytes-or-None, ref)
    ("int32", 42, b([42], "int32"), "src/types/dvalue.rs:102-106"),
    ("int32", 2 ** 31, None, "src/types/dvalue.rs:109-112"),
    ("int32", -2 ** 31 - 1, None, "src/types/dvalue.rs:115-117"),
    ("int64", -42, b([-42], "int64"), "src/types/dvalue.rs:120-124"),
    ("int64", 2 ** 63, None, "src/types/dvalue.rs:127-130"),
    ("int64", 1.0, None, "src/types/dvalue.rs:133-135"),
    ("uint32", 42, b([42], "uint32"), "src/types/dvalue.rs:138-142"),
    ("uint32", 2 ** 32, None, "src/types/dvalue.rs:145-148"),
    ("uint32", -1, None, "src/types/dvalue.rs:151-153"),
    ("uint64", 42, b([42], "uint64"), "src/types/dvalue.rs:156-160"),
    ("uint64", -1, None, "src/types/dvalue.rs:163-166"),
    ("uint64", -1.0, None, "src/types/dvalue.rs:169-171"),
    ("float32", 42.0, b([42.0], "float32"), "src/types/dvalue.rs:174-177"),
    ("float32", 42, b([42.0], "float32"), "src/types/dvalue.rs:180-184"),
    ("float32", float(np.finfo(np.float32).max) * 2.0, None, "src/types/dvalue.rs:187-189"),
    ("float64", -42.0, b([-42.0], "float64"), "src/types/dvalue.rs:192-195"),
    ("float64", 42, b([42.0], "float64"), "src/types/dvalue.rs:198-201"),
    ("int32", 42, b([42], "int32"), "src/types/missing.rs:130-133"),
    ("int32", 2 ** 31, None, "src/types/missing.rs:174-179"),
    ("int64", 2 ** 63, None, "src/types/missing.rs:193-199"),
    ("uint32", 42, b([42], "uint32"), "src/types/missing.rs:202-206"),
    ("uint32", 2 ** 32, None, "src/types/missing.rs:209-212"),
    ("uint64", 42, b([42], "uint64"), "src/types/missing.rs:215-219"),
    ("uint64", -1, None, "src/types/missing.rs:222-224"),
    ("float32", -42.0, b([-42.0], "float32"), "src/types/missing.rs:227-235"),
    ("float32", float(np.finfo(np.float32).max) * 2.0, None, "src/types/missing.rs:238-244"),
]
for dt, v, exp, ref in CONV:
    KATS.append({"kind": "convert", "name": f"{dt}<-{v!r}", "ref": ref, "dtype": dt,
                 "value": v, "value_is_float": isinstance(v, float), "expect": exp})

# missing validation (missing.rs:136-170): ok, u32 negative -> invalid, range min >= max -> invalid
VAL = [
    ("validate_i32", "src/types/missing.rs:136-141", "int32", {"missing_value": 42}, "ok"),
    ("validate_u32_negative", "src/types/missing.rs:144-149", "uint32", {"missing_value": -1}, "E_REQUEST_VALIDATION"),
    ("validate_f32_range_min_gt_max", "src/types/missing.rs:152-160", "float32", {"valid_range": [42.0, -42.0]},
     "E_REQUEST_VALIDATION"),
    ("validate_f32_range_min_eq_max", "src/types/missing.rs:163-171", "float32", {"valid_range": [42.0, 42.0]},
     "E_REQUEST_VALIDATION"),
]
for name, ref, dt, missing, st in VAL:
    KATS.append({"kind": "validate_missing", "name": name, "ref": ref, "dtype": dt, "missing": missing,
                 "expect": st})

OUT.write_text(json.dumps(KATS, indent=1) + "\n")
print(f"wrote {len(KATS)} vectors to {OUT}")
