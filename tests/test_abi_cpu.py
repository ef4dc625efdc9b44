"""CPU-side checks of the product boundary: the C-ABI library loads and exports every symbol the
header declares; the host logic (validation, planning, missing conversion) agrees with the oracle
and the reference's KATs.  No kernel is launched here."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from helpers import STATUS, encode_filters, load_kats, make_request, product_convert, random_case
from oracle import py_oracle as oracle
from reductionist_amd import _abi
from reductionist_amd.models import RequestData, typed_missing
from reductionist_amd.errors import RequestDataValidation, IncompatibleMissing

HEADER = Path(__file__).resolve().parent.parent / "include" / "rdx.h"


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(rdx_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = _abi.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"librdx.so does not export {n}"
    assert set(names) == set(_abi.EXPORTED)
    assert lib.rdx_abi_version() == _abi.RDX_ABI_VERSION
    assert _abi.status_string(_abi.E_NAN_UNORDERED) == "unexpected undefined order error for min"


def test_plan_matches_oracle_random():
    rng = np.random.default_rng(1234)
    lib = _abi.lib()
    checked = 0
    for _ in range(600):
        op, req, raw = random_case(rng)
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        try:
            creq = make_request(op, req, oracle.convert)
        except ValueError:
            continue
        ost, oinfo, _, _ = oracle.execute(creq, data)
        info = _abi.rdx_response_info()
        pst = lib.rdx_plan(creq.ref, len(data), C.byref(info))
        if ost == _abi.E_NAN_UNORDERED:   # data dependent: planning succeeds
            assert pst == 0
            continue
        assert pst == ost, (op, req, pst, ost)
        if ost == 0:
            assert info.dtype == oinfo.dtype and info.shape_list() == oinfo.shape_list()
            assert info.body_bytes == oinfo.body_bytes and info.n_counts == oinfo.n_counts, (op, req)
            checked += 1
    assert checked > 300


def test_plan_error_order_matches_oracle():
    """operation<T>() raises its first error in a fixed order (app.rs:163-183)."""
    cases = [
        ("sum", {"dtype": "int32", "filters": [{"id": "shuffle", "element_size": 3}]}, 8, _abi.E_SHUFFLE_LENGTH),
        ("sum", {"dtype": "int32", "filters": [{"id": "shuffle", "element_size": 0}]}, 8, _abi.E_SHUFFLE_LENGTH),
        ("sum", {"dtype": "int32"}, 6, _abi.E_REQUEST_VALIDATION),              # validate_raw_size
        ("sum", {"dtype": "int32", "size": 6}, 6, _abi.E_FROM_BYTES),
        ("sum", {"dtype": "int32", "shape": [3], "size": 8}, 8, _abi.E_SHAPE_INVALID),
        ("sum", {"dtype": "int32", "shape": [1], "size": 8}, 8, 0),              # ndarray views may be shorter
        ("sum", {"dtype": "int64", "shape": [2, 2], "axis": [1, 0]}, 32, _abi.E_REQUEST_VALIDATION),
        ("select", {"dtype": "int64", "axis": [5]}, 32, 0),                      # select ignores axis
    ]
    lib = _abi.lib()
    for op, req, n, exp in cases:
        creq = make_request(op, req, oracle.convert)
        ost = oracle.execute(creq, bytes(n))[0]
        info = _abi.rdx_response_info()
        assert ost == exp, (req, ost)
        assert lib.rdx_plan(creq.ref, n, C.byref(info)) == exp, req
    # a compressed request is decompressed first (filter_pipeline.rs:23-25): 8 zero bytes are not a
    # zlib stream; rdx_plan takes the DECOMPRESSED length and plans it like an uncompressed chunk
    creq = make_request("sum", {"dtype": "int32", "compression": "zlib", "size": 8}, oracle.convert)
    assert oracle.execute(creq, bytes(8))[0] == _abi.E_DECOMPRESSION
    assert lib.rdx_plan(creq.ref, 8, C.byref(_abi.rdx_response_info())) == 0
    assert lib.rdx_plan(creq.ref, 6, C.byref(_abi.rdx_response_info())) == _abi.E_REQUEST_VALIDATION
    # blosc2 (compression.rs:29-57): 8 zero bytes are no blosc2 header -> "invalid blosc2 compressed data"
    creq = make_request("sum", {"dtype": "int32", "compression": "blosc2", "size": 8}, oracle.convert)
    assert oracle.execute(creq, bytes(8))[0] == _abi.E_DECOMPRESSION
    assert oracle.lib().oracle_inflate_last_error() == _abi.BLOSC2_INVALID
    assert lib.rdx_plan(creq.ref, 8, C.byref(_abi.rdx_response_info())) == 0


def _random_validation_case(rng):
    op, req, raw = random_case(rng)
    r = rng.random()
    if "shape" in req:
        if r < 0.1:
            req["shape"] = [0] + req["shape"][1:]
        elif r < 0.2 and "selection" in req:
            req["selection"][0][2] = 0
        elif r < 0.3 and isinstance(req.get("axis"), list) and len(req["axis"]) > 1:
            req["axis"] = req["axis"][::-1]
        elif r < 0.4 and req.get("axis") is not None:
            req["axis"] = len(req["shape"]) + 1
    if rng.random() < 0.3:
        req["size"] = len(raw) + (0 if rng.random() < 0.7 else 4)
    return op, req, raw


def test_validate_matches_oracle_random():
    rng = np.random.default_rng(99)
    lib = _abi.lib()
    n = 0
    for _ in range(800):
        op, req, _ = _random_validation_case(rng)
        try:
            creq = make_request(op, req, oracle.convert)
        except ValueError:
            continue
        assert lib.rdx_validate_request(creq.ref) == oracle.validate(creq), (op, req)
        n += 1
    assert n > 500


@pytest.mark.parametrize("kat", load_kats("convert"), ids=lambda k: k["name"])
def test_product_convert_kats(kat):
    st, out = product_convert(kat["dtype"], kat["value"])
    if kat["expect"] is None:
        assert st != 0
    else:
        assert st == 0 and out.hex() == kat["expect"]


@pytest.mark.parametrize("kat", load_kats("validate_missing"), ids=lambda k: k["name"])
def test_request_data_validate_missing_kats(kat):
    rd = RequestData(dtype=kat["dtype"], missing=kat["missing"])
    if kat["expect"] == "ok":
        rd.validate()
    else:
        with pytest.raises(RequestDataValidation):
            rd.validate()


def test_request_data_validation_mirror():
    """models.rs validators (models.rs:179-313) on the Python host mirror."""
    ok = RequestData.from_json({"interface_type": "s3", "url": "http://x/b/o", "dtype": "float32",
                                "shape": [2, 3], "selection": [[0, 2, 1], [0, 3, 2]], "axis": [0, 1],
                                "filters": [{"id": "shuffle", "element_size": 4}], "size": 24,
                                "missing": {"valid_range": [-1.0, 1.0]}})
    ok.validate()
    bad = [
        {"shape": [0, 3]}, {"size": 0}, {"selection": [[0, 1, 0]], "shape": [2]}, {"selection": [[0, 1, 1]]},
        {"shape": [2, 3], "selection": [[0, 1, 1]]}, {"axis": 0}, {"shape": [2], "axis": 1},
        {"shape": [2, 3], "axis": [1, 0]}, {"shape": [2, 3], "axis": [0, 0]}, {"shape": [2], "axis": [0, 1]},
        {"shape": [2], "size": 12}, {"missing": {"valid_range": [2, 1]}}, {"missing": {"missing_value": 1.5}},
    ]
    for b in bad:
        rd = RequestData(dtype="int32", **b)
        with pytest.raises(RequestDataValidation):
            rd.validate()
    with pytest.raises(RequestDataValidation):
        RequestData.from_json({"interface_type": "s3", "url": "u", "dtype": "int32", "bogus": 1})
    with pytest.raises(IncompatibleMissing):
        typed_missing({"missing_value": -1}, "uint32")


def test_no_device_fails_loudly():
    lib = _abi.lib()
    if lib.rdx_device_count() > 0:
        pytest.skip("a device is present")
    from reductionist_amd import Engine
    from reductionist_amd.errors import DeviceError
    with pytest.raises(DeviceError):
        Engine()


def test_host_decompressed_request_runs_validate_raw_size():
    """app.rs:169-172: a compressed request has its DECOMPRESSED length checked against the shape, whatever
    `size` says (for a compressed request `size` is the compressed length, models.rs:244-249).  The Rust
    plugin that inflates a lone gzip/zlib chunk on the host hands it to the engine with `compression` and
    `size` both cleared (integration/app_gpu.rs host_decompressed); the engine runs validate_raw_size
    exactly when `size` is absent, so the mismatch is still a 400."""
    import gzip

    lib = _abi.lib()
    raw = np.arange(6, dtype=np.int32).tobytes()          # 6 elements behind a shape of 4
    stream = gzip.compress(raw)
    as_sent = _abi.CRequest("sum", "int32", shape=[4], compression="gzip", size=len(stream))
    assert oracle.execute(as_sent, stream)[0] == _abi.E_REQUEST_VALIDATION   # the reference's answer
    cleared = _abi.CRequest("sum", "int32", shape=[4])
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(cleared.ref, len(raw), C.byref(info)) == _abi.E_REQUEST_VALIDATION
    # keeping `size` would skip the check and reduce the first 4 elements (round-2 shim defect)
    kept = _abi.CRequest("sum", "int32", shape=[4], size=len(stream))
    assert lib.rdx_plan(kept.ref, len(raw), C.byref(info)) == 0
    # a decompressed length that matches passes either way
    assert lib.rdx_plan(cleared.ref, 16, C.byref(info)) == 0 and info.shape_list() == []


def test_unsupported_carries_its_reason():
    """RDX_E_UNSUPPORTED says why (rdx_last_unsupported_reason): only a blosc2 codec sends the plugin to host
    decompression; a rank above 32 or a view of 2^32 elements sends it to the reference CPU path."""
    lib = _abi.lib()
    info = _abi.rdx_response_info()
    deep = _abi.CRequest("sum", "int32", shape=[1] * 33)
    assert lib.rdx_plan(deep.ref, 4, C.byref(info)) == _abi.E_UNSUPPORTED
    assert lib.rdx_last_unsupported_reason() == _abi.UNSUPPORTED_RANK
    # planning only (no data): a strided view of 2^32 f32 elements over a 32 GiB chunk
    big = _abi.CRequest("sum", "float32", shape=[1 << 31, 4], selection=[[0, 1 << 31, 1], [0, 4, 2]])
    assert lib.rdx_plan(big.ref, (1 << 31) * 16, C.byref(info)) == _abi.E_UNSUPPORTED
    assert lib.rdx_last_unsupported_reason() == _abi.UNSUPPORTED_VIEW_SIZE
    # the reason is per thread and only read after E_UNSUPPORTED: a good plan leaves it alone
    ok = _abi.CRequest("sum", "int32")
    assert lib.rdx_plan(ok.ref, 16, C.byref(info)) == 0
    assert lib.rdx_last_unsupported_reason() == _abi.UNSUPPORTED_VIEW_SIZE
