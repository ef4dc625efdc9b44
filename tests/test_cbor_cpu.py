"""Response serialisation (rdx_cbor_*, models.rs:355-416 CBORResponse through serde_cbor, app.rs:33-40):
the oracle pinned by RFC 7049 Appendix A and the reference's response tests, and the engine's host encoder
(rdx_cbor_encode: host code, no device needed) byte-identical to the oracle.  The device encoder is
checked against the same oracle in test_gpu_cbor.py."""
import ctypes as C
import json
import struct
from pathlib import Path

import numpy as np
import pytest

from oracle import cbor_oracle as cb
from reductionist_amd import _abi

GOLDEN = Path(__file__).resolve().parent / "golden"
RFC = json.loads((GOLDEN / "cbor_rfc7049.json").read_text())
MODELS = json.loads((GOLDEN / "cbor_models.json").read_text())


def _encode_value(v):
    """Generic encoder for the RFC table's value forms (ints, text, bytes, arrays, ordered maps)."""
    if isinstance(v, bool):
        raise TypeError
    if isinstance(v, int):
        return cb.enc_int(v) if v < (1 << 63) else cb.head(0, v)
    if isinstance(v, str):
        return cb.enc_text(v)
    if isinstance(v, list):
        return cb.head(4, len(v)) + b"".join(_encode_value(x) for x in v)
    if "bytes" in v:
        return cb.enc_bytes(bytes.fromhex(v["bytes"]))
    return cb.head(5, len(v["map"])) + b"".join(_encode_value(k) + _encode_value(x) for k, x in v["map"])


def _plain(v, is_map=False):
    """Decoded value -> the fixture's value form (maps decode to ordered (key, value) pairs)."""
    if isinstance(v, bytes):
        return {"bytes": v.hex()}
    if is_map:
        return {"map": [[k, _plain(x)] for k, x in v]}
    if isinstance(v, list):
        return [_plain(x) for x in v]
    return v


def buf_major(hexstr):
    return bytes.fromhex(hexstr)[0] >> 5


@pytest.mark.parametrize("row", RFC, ids=[r["diagnostic"] for r in RFC])
def test_oracle_primitives_match_rfc7049(row):
    enc = _encode_value(row["value"])
    assert enc.hex() == row["hex"]
    dec, used = cb.decode(bytes.fromhex(row["hex"]))
    assert used == len(enc)
    want = row["value"]
    if isinstance(want, dict) and "map" in want:
        assert buf_major(row["hex"]) == 5 and _plain(dec, is_map=True) == want
    elif isinstance(want, dict):
        assert dec == bytes.fromhex(want["bytes"])
    else:
        assert dec == want


def _fields(buf):
    dec, used = cb.decode(buf)
    assert used == len(buf)
    assert isinstance(dec, list) and len(dec) == 7
    return dec


@pytest.mark.parametrize("case", MODELS, ids=[m["source"] for m in MODELS])
def test_oracle_matches_reference_response_tests(case):
    r = case["response"]
    buf = cb.cbor_response(bytes(r["body"]), r["dtype"], r["shape"], r["count"],
                           r["option_shape_as_bytes"], r["option_count_as_bytes"])
    dec = _fields(buf)
    names = [k for k, _ in dec]
    assert names == ["bytes", "dtype", "shape", "shape_as_bytes", "count", "count_as_bytes", "byte_order"]
    if "field_order" in case:
        assert names == case["field_order"]
    got = dict(dec)
    e = case["expect"]
    assert list(got["bytes"]) == e["bytes"]
    assert got["dtype"] == e["dtype"] and got["byte_order"] == e["byte_order"]
    assert got["shape"] == e["shape"] and got["count"] == e["count"]
    if "shape_as_bytes_u64" in e:   # convert_shape_from_bytes (models.rs:1050-1055): u64 native-endian
        assert list(struct.unpack(f"<{len(got['shape_as_bytes']) // 8}Q", got["shape_as_bytes"])) == e["shape_as_bytes_u64"]
    else:
        assert list(got["shape_as_bytes"]) == e["shape_as_bytes"]
    if "count_as_bytes_i64" in e:   # convert_count_from_bytes (models.rs:1080-1085)
        assert list(struct.unpack(f"<{len(got['count_as_bytes']) // 8}q", got["count_as_bytes"])) == e["count_as_bytes_i64"]
    else:
        assert list(got["count_as_bytes"]) == e["count_as_bytes"]


def _info(dtype, shape, body_bytes, n_counts):
    info = _abi.rdx_response_info()
    info.dtype = _abi.DTYPES[dtype]
    info.ndim = len(shape)
    for i, s in enumerate(shape):
        info.shape[i] = s
    info.body_bytes = body_bytes
    info.n_counts = n_counts
    return info


def host_encode(info, body: bytes, counts: np.ndarray, flags: int) -> bytes:
    lib = _abi.lib()
    bound = lib.rdx_cbor_bound(C.byref(info), flags)
    out = (C.c_uint8 * max(1, bound))()
    n = C.c_uint64()
    cts = np.ascontiguousarray(counts, dtype=np.int64)
    st = lib.rdx_cbor_encode(C.byref(info), body, cts.ctypes.data if cts.size else None, flags, out, bound,
                             C.byref(n))
    assert st == 0, _abi.status_string(st)
    assert n.value <= bound
    return C.string_at(out, n.value)


def random_counts(rng, n):
    """Counts covering every CBOR integer length class and sign (engine counts are >= 0; the encoder
    handles any i64)."""
    cls = rng.integers(0, 7, n)
    lim = np.array([23, 255, 65535, 2 ** 32 - 1, 2 ** 62, 24, 2 ** 31], dtype=np.int64)
    v = (rng.random(n) * lim[cls].astype(np.float64)).astype(np.int64)
    edges = np.array([0, 23, 24, 255, 256, 65535, 65536, 2 ** 32 - 1, 2 ** 32, 2 ** 63 - 1, -1, -24, -25,
                      -256, -257, -65536, -65537, -(2 ** 32), -(2 ** 32) - 1, -(2 ** 63)], dtype=np.int64)
    v[rng.random(n) < 0.1] *= -1
    if n:
        k = min(n, edges.size)
        v[rng.choice(n, k, replace=False)] = edges[:k]
    return v


def test_host_encoder_matches_reference_tests():
    for case in MODELS:
        r = case["response"]
        flags = (_abi.CBOR_SHAPE_AS_BYTES if r["option_shape_as_bytes"] else 0) | \
                (_abi.CBOR_COUNT_AS_BYTES if r["option_count_as_bytes"] else 0)
        info = _info(r["dtype"], r["shape"], len(r["body"]), len(r["count"]))
        got = host_encode(info, bytes(r["body"]), np.array(r["count"]), flags)
        assert got == cb.cbor_response(bytes(r["body"]), r["dtype"], r["shape"], r["count"],
                                       r["option_shape_as_bytes"], r["option_count_as_bytes"])


def test_host_encoder_random_matches_oracle():
    rng = np.random.default_rng(0xCB0)
    dtypes = list(_abi.DTYPES)
    for it in range(300):
        dtype = dtypes[it % len(dtypes)]
        nd = int(rng.integers(0, 6))
        shape = [int(x) for x in rng.integers(0, 70000 if nd < 3 else 300, nd)]
        if it % 7 == 0 and nd:
            shape[0] = int(rng.integers(0, 2 ** 40))   # long shape heads
        n = int(rng.integers(0, 3000))
        counts = random_counts(rng, n)
        body = rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
        flags = int(rng.integers(0, 4))
        info = _info(dtype, shape, len(body), n)
        got = host_encode(info, body, counts, flags)
        want = cb.cbor_response(body, dtype, shape, counts.tolist(), bool(flags & 1), bool(flags & 2))
        assert got == want, (it, dtype, shape, n, flags)


def test_host_encoder_sizes_and_errors():
    lib = _abi.lib()
    info = _info("float32", [4], 16, 4)
    counts = np.array([1, 2, 3, 1000000], dtype=np.int64)
    body = bytes(16)
    exact = len(cb.cbor_response(body, "float32", [4], counts.tolist()))
    n = C.c_uint64()
    out = (C.c_uint8 * exact)()
    assert lib.rdx_cbor_encode(C.byref(info), body, counts.ctypes.data, 0, out, exact - 1, C.byref(n)) == \
        _abi.E_BUFFER_TOO_SMALL
    assert n.value == exact
    assert lib.rdx_cbor_encode(C.byref(info), body, counts.ctypes.data, 0, out, exact, C.byref(n)) == 0
    assert lib.rdx_cbor_bound(C.byref(info), 0) == exact - (1 + 1 + 1 + 5) + 4 * 9
    bad = _info("float32", [4], 16, 4)
    bad.dtype = 9
    assert lib.rdx_cbor_encode(C.byref(bad), body, counts.ctypes.data, 0, out, exact, C.byref(n)) == \
        _abi.E_INVALID_ARGUMENT
    assert lib.rdx_cbor_encode(C.byref(info), body, counts.ctypes.data, 4, out, exact, C.byref(n)) == \
        _abi.E_INVALID_ARGUMENT
