"""Parity of the MI355X engine (through the C ABI) with the oracle and the reference's KATs.

Bar: bit-exact for count, select, every integer op and min/max (incl. the ±0 tie rule); float sums
bit-exact on exactly-summable data and within the stated tolerance on real-valued data:
    f32: |gpu - exact| <= 1 ulp_f32(exact) + 2^-45 * sum|x|      (f64 accumulation, one rounding)
    f64: |gpu - exact| <= 2 ulp_f64(exact) + 2^-100 * n * sum|x|   (Neumaier-compensated f64)
where `exact` is math.fsum of the included values.  NaN results compare by NaN-ness (x86 and gfx950
produce different default-NaN bit patterns for inf - inf).
"""
import math
import struct

import numpy as np
import pytest

from helpers import NP, check_kat_result, encode_filters, load_kats, make_request, product_convert, random_case
from oracle import py_oracle as oracle
from reductionist_amd import _abi

pytestmark = pytest.mark.gpu


def same_result(dtype, body_a, body_b):
    if body_a == body_b:
        return True
    if not dtype.startswith("float") or len(body_a) != len(body_b):
        return False
    a = np.frombuffer(body_a, dtype=NP[dtype])
    b = np.frombuffer(body_b, dtype=NP[dtype])
    ua = a.view(np.uint32 if dtype == "float32" else np.uint64)
    ub = b.view(np.uint32 if dtype == "float32" else np.uint64)
    return bool(np.all((ua == ub) | (np.isnan(a) & np.isnan(b))))


def run_both(engine, op, req, data):
    creq = make_request(op, req, oracle.convert)
    ost, oinfo, obody, ocounts = oracle.execute(creq, data)
    pst, pinfo, pbody, pcounts = engine.execute_raw(creq, data)
    return (ost, oinfo, obody, ocounts), (pst, pinfo, pbody, pcounts)


def assert_parity(engine, op, req, data):
    (ost, oinfo, obody, ocounts), (pst, pinfo, pbody, pcounts) = run_both(engine, op, req, data)
    assert pst == ost, (op, req, pst, ost)
    if ost != 0:
        return
    resp_dtype = _abi.DTYPE_NAMES[oinfo.dtype]
    assert pinfo.shape_list() == oinfo.shape_list(), (op, req)
    assert pcounts == ocounts, (op, req, pcounts, ocounts)
    assert same_result(resp_dtype, pbody, obody), (op, req, pbody.hex(), obody.hex())


@pytest.mark.parametrize("kat", load_kats("op"), ids=lambda k: k["name"])
def test_reference_kats_on_device(engine, kat):
    creq = make_request(kat["op"], kat["request"], product_convert)
    st, info, body, counts = engine.execute_raw(creq, bytes.fromhex(kat["data"]))
    check_kat_result(kat, st, info, body, counts, _abi.lib().rdx_inflate_last_error())


@pytest.mark.parametrize("seed", range(8))
def test_random_differential(engine, seed):
    rng = np.random.default_rng(1000 + seed)
    n = 0
    for _ in range(300):
        op, req, raw = random_case(rng, allow_nan=True)
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        try:
            assert_parity(engine, op, req, data)
        except ValueError:
            continue
        n += 1
    assert n > 200


@pytest.mark.parametrize("dtype", list(NP))
@pytest.mark.parametrize("op", ["count", "max", "min", "sum", "select"])
def test_larger_strided_views(engine, dtype, op):
    """Multi-workgroup paths (cross-workgroup finalisation, slices) on mid-size hyperslabs."""
    rng = np.random.default_rng(sum(map(ord, dtype + op)))
    for shape, sel, axis, order in (
        ([64, 48, 40], [[3, 60, 1], [0, 48, 2], [5, 37, 1]], None, "C"),
        ([64, 48, 40], [[60, 3, -1], [1, 47, 3], [-1, -41, -2]], None, "F"),
        ([64, 48, 40], [[3, 60, 1], [0, 48, 2], [5, 37, 1]], [1], "C"),
        ([64, 48, 40], None, [0, 2], "C"),
        ([64, 48, 40], [[3, 60, 1], [0, 48, 2], [8, 40, 1]], None, "C"),     # 16-B vector lanes
        ([64, 48, 40], [[3, 60, 1], [0, 48, 2], [8, 40, 1]], [], "C"),
        ([64, 48, 40], [[3, 60, 1], [0, 48, 2], [8, 40, 1]], [], "F"),
        ([64, 48, 40], None, [2], "F"),
        ([300, 500], None, 0, "C"),
        ([300, 500], [[0, 300, 1], [10, 490, 7]], 1, "C"),
        ([7, 9000], None, 1, "C"),
        ([9000, 7], None, 0, "C"),
        ([9000, 7], None, [], "F"),
        ([16, 8, 128], None, [2], "C"),          # rows mode, 16-B lanes
        ([4, 20000], None, 1, "C"),              # rows mode, few outputs -> slices
        ([20000, 8], None, 0, "C"),              # cols mode, 16-B lanes, slices
        ([8, 20000], None, 0, "F"),              # F order: kept dim contiguous
        ([32, 64, 24], [[0, 32, 1], [8, 64, 2], [0, 24, 1]], [0, 1], "C"),
    ):
        n = int(np.prod(shape))
        vals = rng.integers(-100, 100, n).astype(NP[dtype]) if dtype.startswith("float") else \
            rng.integers(0, 100, n).astype(NP[dtype])
        req = {"dtype": dtype, "shape": shape, "order": order}
        if sel:
            req["selection"] = sel
        if axis is not None:
            req["axis"] = axis
        if rng.random() < 0.5:
            req["missing"] = {"valid_range": [-50, 60] if not dtype.startswith("u") else [5, 60]}
        assert_parity(engine, op, req, vals.tobytes())


def test_pm0_tie_rule(engine):
    """max_by keeps the LAST equal element, min_by the FIRST (operations.rs:229-241, 459-469)."""
    rng = np.random.default_rng(7)
    for dtype in ("float32", "float64"):
        for _ in range(200):
            n = int(rng.integers(1, 4000))
            v = np.where(rng.random(n) < 0.5, -0.0, 0.0).astype(NP[dtype])
            v[rng.random(n) < 0.3] = -1.0
            shape = None
            req = {"dtype": dtype}
            if rng.random() < 0.6 and n >= 4:
                a = int(rng.integers(1, 5))
                n = (n // a) * a
                v = v[:n]
                req["shape"] = shape = [a, n // a]
                req["order"] = "F" if rng.random() < 0.5 else "C"
                r = rng.random()
                if r < 0.3:
                    req["selection"] = [[0, a, 1], [int(rng.integers(0, 3)), n // a, int(rng.choice([1, 2, -1, -3]))]]
                elif r < 0.6:
                    req["axis"] = int(rng.integers(0, 2))
                elif r < 0.8:
                    req["axis"] = [0, 1]
            for op in ("max", "min"):
                assert_parity(engine, op, req, v.tobytes())


@pytest.mark.parametrize("dtype", ["float32", "float64"])
@pytest.mark.parametrize("per", [3, 4, 5, 7])
def test_minmax_long_contiguous_ranges(engine, dtype, per):
    """Float min/max over whole chunks long enough that every workgroup of k_all_contig folds `per`
    4096-element tiles (the software-pipelined loop's even/odd exits and its single-tile remainder),
    plus a ragged tail; ±0 planted everywhere incl. the last tile, so the value is a zero whose sign
    comes from the fold-order ranks (min_by keeps the FIRST equal, max_by the LAST); plain, and
    byte-shuffled + big-endian (the fused path)."""
    rng = np.random.default_rng(100 * per + (dtype == "float64"))
    n = 4096 * 256 * per + int(rng.integers(1, 4096))
    base = (np.abs(rng.standard_normal(n)) + 1.0).astype(NP[dtype])
    pos = np.concatenate([rng.integers(0, n, 48), rng.integers(n - 5000, n, 16)])
    zeros = np.where(rng.random(pos.size) < 0.5, -0.0, 0.0).astype(NP[dtype])
    es = np.dtype(NP[dtype]).itemsize
    for op, sign in (("min", 1.0), ("max", -1.0)):
        v = (base * sign).astype(NP[dtype])
        v[pos] = zeros
        for req in ({"dtype": dtype},
                    {"dtype": dtype, "byte_order": "big", "filters": [{"id": "shuffle", "element_size": es}]}):
            raw = v.astype(v.dtype.newbyteorder(">")).tobytes() if req.get("byte_order") == "big" else v.tobytes()
            assert_parity(engine, op, req, encode_filters(raw, req.get("filters"), oracle.shuffle))


def test_nan_raises_like_reference_panic(engine):
    for dtype in ("float32", "float64"):
        v = np.arange(4096, dtype=NP[dtype])
        v[1234] = np.nan
        for op in ("max", "min"):
            for req in ({"dtype": dtype}, {"dtype": dtype, "shape": [64, 64], "axis": 1},
                        {"dtype": dtype, "shape": [64, 64], "selection": [[0, 64, 2], [0, 64, 1]]}):
                assert_parity(engine, op, req, v.tobytes())
                creq = make_request(op, req, oracle.convert)
                st = engine.execute_raw(creq, v.tobytes())[0]
                if req.get("selection") and 1234 // 64 % 2 == 1:
                    continue
                assert st == _abi.E_NAN_UNORDERED
            # axis=() never compares: NaN passes through (operations.rs:188-210)
            assert_parity(engine, op, {"dtype": dtype, "shape": [64, 64], "axis": []}, v.tobytes())


@pytest.mark.parametrize("shape,axis,dtype,op", [
    ([65536, 32], 0, "float64", "min"),       # narrow tile: 16 lanes x 2 per row, 4 rows per access, long fold
    ([4096, 48], 0, "float32", "sum"),        # 12 vectors -> 16-lane tile
    ([3000, 130], 0, "int32", "max"),         # 130 % 4 != 0 -> 8-byte lanes
    ([2048, 1024], 0, "float32", "sum"),      # narrower lanes chosen to bound the fold
    ([64, 512, 96], 1, "uint64", "count"),    # cols over a middle axis, missing filter
    ([8, 4096, 3], 1, "float32", "max"),      # odd inner width, scalar lanes
    ([40000, 2], 0, "int64", "sum"),          # 2 outputs
    ([50001, 6], 0, "float32", "max"),        # 1-lane tile, ragged slices
    ([30000, 64], 0, "int32", "sum"),         # 16-B lanes, many slices per tile
])
def test_cols_tilings(engine, shape, axis, dtype, op):
    """Column-mode tile shapes (k_axis_cols): W lanes x VW outputs, several rows per wave access,
    sliced reductions folded by the last slice; bit-exact vs the oracle."""
    rng = np.random.default_rng(11)
    n = int(np.prod(shape))
    real = dtype.startswith("float") and op != "sum"   # float sums: exactly summable values (bit-exact)
    v = (rng.standard_normal(n) * 100 if real else rng.integers(-1000, 1000, n)).astype(NP[dtype])
    req = {"dtype": dtype, "shape": shape, "axis": axis}
    if op == "count":
        req["missing"] = {"valid_min": 0}
    if dtype.startswith("float") and op in ("min", "max"):
        v[rng.integers(0, n, 50)] = 0.0
        v[rng.integers(0, n, 50)] = -0.0           # ±0 ties across slices
    assert_parity(engine, op, req, v.tobytes())


@pytest.mark.parametrize("case", range(12))
def test_row_batch(engine, case):
    """Few long contiguous rows (>= 64 KiB reduced per output) go to the batched all-axes kernel,
    one chunk per output (rdx_runtime.cpp, Mode::Axis): selections on the kept and reduced dims,
    reversed reduced axis, F order, shuffle + big-endian, missing data, ±0 ties, NaN."""
    dtype, op, shape, sel, axis, order, extra = [
        ("float32", "sum", [6, 40000], None, 1, "C", {}),
        ("float64", "max", [5, 16411], None, 1, "C", {}),                         # unaligned rows
        ("float32", "min", [7, 30001], [[1, 7, 2], [3, 29990, 1]], 1, "C", {}),    # strided kept, offset rows
        ("int32", "max", [4, 50000], [[0, 4, 1], [49999, 10, -1]], 1, "C", {}),    # reversed reduced axis
        ("int64", "sum", [20000, 3], None, 0, "F", {}),
        ("uint32", "count", [3, 70000], None, 1, "C", {"missing": {"valid_min": 40}}),
        ("float32", "max", [4, 65536], None, 1, "C", {"byte_order": "big",
                                                     "filters": [{"id": "shuffle", "element_size": 4}]}),
        ("uint64", "min", [2, 3, 20000], None, 2, "C", {"missing": {"missing_values": [7, 9]}}),
        ("float64", "min", [3, 9000], None, 1, "C", {}),                          # NaN -> status
        ("float32", "select", [4, 40000], None, 1, "C", {}),
        ("float32", "sum", [3, 20001], None, 1, "C", {"byte_order": "big",               # unaligned fused rows
                                                      "filters": [{"id": "shuffle", "element_size": 4}]}),
        ("int64", "max", [5, 9001], [[0, 5, 2], [1, 9000, 1]], 1, "C",
         {"filters": [{"id": "shuffle", "element_size": 8}], "missing": {"valid_max": 90}}),
    ][case]
    rng = np.random.default_rng(100 + case)
    n = int(np.prod(shape))
    v = rng.integers(-100, 100, n).astype(NP[dtype]) if not dtype.startswith("u") else \
        rng.integers(0, 100, n).astype(NP[dtype])
    if dtype.startswith("float") and op in ("min", "max"):
        v[rng.integers(0, n, 200)] = 0.0
        v[rng.integers(0, n, 200)] = -0.0
        if case == 8:
            v[n // 2 + 17] = np.nan
    req = {"dtype": dtype, "shape": shape, "axis": axis, "order": order, **extra}
    if sel:
        req["selection"] = sel
    raw = v.astype(NP[dtype]).tobytes()
    if req.get("byte_order") == "big":
        raw = v.astype(np.dtype(NP[dtype]).newbyteorder(">")).tobytes()
    data = encode_filters(raw, req.get("filters"), oracle.shuffle)
    assert_parity(engine, op, req, data)


def test_long_missing_values_list(engine):
    rng = np.random.default_rng(3)
    for dtype in NP:
        v = rng.integers(0, 200, 20000).astype(NP[dtype])
        lst = sorted({int(x) for x in rng.integers(0, 200, 60)})
        if dtype.startswith("float"):
            lst = [float(x) for x in lst] + [-0.0]
        for op in ("count", "sum", "max", "select"):
            assert_parity(engine, op, {"dtype": dtype, "missing": {"missing_values": lst}}, v.tobytes())


def test_unfused_filters_and_chains(engine):
    rng = np.random.default_rng(5)
    raw = rng.integers(-1000, 1000, 6 * 4096).astype(np.int32).tobytes()
    for filters in ([2], [8], [3], [1], [4, 2], [2, 4], [8, 4, 2], [24], [len(raw) // 2], [len(raw)]):
        fl = [{"id": "shuffle", "element_size": e} for e in filters]
        data = encode_filters(raw, fl, oracle.shuffle)
        for op in ("sum", "select", "max"):
            assert_parity(engine, op, {"dtype": "int32", "filters": fl}, data)
    # odd lengths that the shuffle assert rejects
    assert_parity(engine, "sum", {"dtype": "int32", "filters": [{"id": "shuffle", "element_size": 3}]}, raw[:-4])


def test_c2_f32_sum_64mib(engine):
    """BASELINE config 2: 16 Mi f32, big-endian + shuffle(es=4).  D-int (exactly summable) is
    bit-exact with the sequential oracle; D-real meets the stated f32 tolerance."""
    n = 16 * 1024 * 1024
    req = {"dtype": "float32", "byte_order": "big", "filters": [{"id": "shuffle", "element_size": 4}]}
    for seed, real in ((0x5EED0003, False), (0x5EED0004, True)):
        rng = np.random.default_rng(seed)
        vals = rng.random(n, dtype=np.float32) if real else rng.integers(-8, 9, n).astype(np.float32)
        data = oracle.shuffle(vals.astype(">f4").tobytes(), 4)
        creq = make_request("sum", req, oracle.convert)
        st, info, body, counts = engine.execute_raw(creq, data)
        assert st == 0 and counts == [n]
        gpu = struct.unpack("<f", body)[0]
        ost, _, obody, _ = oracle.execute(creq, data, body_cap=64, counts_cap=8)
        cpu = struct.unpack("<f", obody)[0]
        exact = math.fsum(vals.astype(np.float64))
        if not real:
            assert gpu == cpu == exact
        else:
            tol = float(np.spacing(np.float32(abs(exact)))) + 2.0 ** -45 * float(np.abs(vals).sum(dtype=np.float64))
            assert abs(gpu - exact) <= tol, (gpu, exact, cpu)
            assert abs(gpu - exact) <= abs(cpu - exact) + tol


def test_f64_sum_tolerance(engine):
    rng = np.random.default_rng(0x5EED0002)
    for n in (1000, 1 << 20, 3 * (1 << 20) + 7):
        vals = rng.standard_normal(n) * 1e3
        creq = make_request("sum", {"dtype": "float64"}, oracle.convert)
        st, info, body, counts = engine.execute_raw(creq, vals.tobytes())
        gpu = struct.unpack("<d", body)[0]
        exact = math.fsum(vals)
        tol = 2 * float(np.spacing(abs(exact))) + 2.0 ** -100 * n * float(np.abs(vals).sum())
        assert abs(gpu - exact) <= tol, (n, gpu, exact)


def test_c3_f64_minmax_hyperslab_missing(engine):
    """BASELINE config 3: f64 [128,128,128], selection, missing_value -9999 at 5 %, min and max,
    plus a valid_range variant — bit-exact with the oracle."""
    rng = np.random.default_rng(0x5EED0005)
    vals = rng.standard_normal(128 ** 3) * 100
    vals[rng.random(vals.size) < 0.05] = -9999.0
    sel = [[8, 120, 1], [0, 128, 2], [16, 112, 1]]
    for missing in ({"missing_value": -9999.0}, {"valid_range": [-250.0, 250.0]}):
        for op in ("min", "max", "count", "sum"):
            req = {"dtype": "float64", "shape": [128, 128, 128], "selection": sel, "missing": missing}
            if op == "sum":
                creq = make_request(op, req, oracle.convert)
                st, info, body, counts = engine.execute_raw(creq, vals.tobytes())
                ost, _, obody, ocounts = oracle.execute(creq, vals.tobytes(), body_cap=64, counts_cap=8)
                assert counts == ocounts
                v = vals.reshape(128, 128, 128)[8:120, 0:128:2, 16:112].ravel()
                v = v[v != -9999.0] if "missing_value" in missing else v[(v >= -250) & (v <= 250)]
                exact = math.fsum(v)
                gpu = struct.unpack("<d", body)[0]
                assert abs(gpu - exact) <= 2 * float(np.spacing(abs(exact))) + 2.0 ** -100 * v.size * float(np.abs(v).sum())
            else:
                assert_parity(engine, op, req, vals.tobytes())


def test_c5_i64_select_256mib(engine):
    """BASELINE config 5: i64 [512,256,256] select with a hyperslab (128 MiB out)."""
    rng = np.random.default_rng(0x5EED0006)
    vals = rng.integers(-2 ** 63, 2 ** 63 - 1, 512 * 256 * 256, dtype=np.int64)
    req = {"dtype": "int64", "shape": [512, 256, 256], "selection": [[0, 512, 1], [64, 192, 1], [0, 256, 1]]}
    creq = make_request("select", req, oracle.convert)
    st, info, body, counts = engine.execute_raw(creq, vals.tobytes())
    assert st == 0 and counts == [16777216] and info.shape_list() == [512, 128, 256]
    expect = vals.reshape(512, 256, 256)[:, 64:192, :]
    assert np.array_equal(np.frombuffer(body, dtype=np.int64), expect.ravel())


def test_device_resident_and_batch_paths(engine):
    """rdx_execute_device / rdx_execute_batch_device agree with the host path."""
    import torch
    rng = np.random.default_rng(11)
    n_chunks, n = 48, 1 << 18
    req = {"dtype": "float32", "filters": [{"id": "shuffle", "element_size": 4}]}
    creq = make_request("sum", req, oracle.convert)
    chunks = [oracle.shuffle(rng.integers(-8, 9, n).astype(np.float32).tobytes(), 4) for _ in range(n_chunks)]
    dev = [torch.frombuffer(bytearray(c), dtype=torch.uint8).cuda() for c in chunks]
    bodies = torch.zeros(n_chunks, dtype=torch.float32, device="cuda")
    counts = torch.zeros(n_chunks, dtype=torch.int64, device="cuda")
    status = torch.zeros(n_chunks, dtype=torch.int32, device="cuda")
    ws = engine.workspace(0)
    stream = torch.cuda.current_stream().cuda_stream
    ws.execute_batch_device(creq, [d.data_ptr() for d in dev], 4 * n, bodies.data_ptr(), counts.data_ptr(),
                            status.data_ptr(), stream)
    torch.cuda.synchronize()
    for i, c in enumerate(chunks):
        st, info, body, cnt = engine.execute_raw(creq, c)
        assert st == 0 and struct.unpack("<f", body)[0] == float(bodies[i]) and cnt == [int(counts[i])]
    assert int(status.abs().sum()) == 0
    one_b = torch.zeros(1, dtype=torch.float32, device="cuda")
    one_c = torch.zeros(1, dtype=torch.int64, device="cuda")
    ws.execute_device(creq, dev[3].data_ptr(), 4 * n, one_b.data_ptr(), one_c.data_ptr(), None, stream)
    torch.cuda.synchronize()
    assert float(one_b[0]) == float(bodies[3]) and int(one_c[0]) == n
    ws.close()
