"""CPU tests of the decompression oracle (oracle/oracle_inflate.cpp, a restatement of
src/compression.rs:18-82 through RFC 1950/1951/1952) — the checker the device inflate kernel is
compared against in tests/test_gpu_inflate.py.

Pinning: the reference's own tests (compression.rs:136-190, filter_pipeline.rs:56-120) give decoded
bytes for gzip/zlib streams of b"hello world" and [1, 2, 3, 4] (flate2 Compression::fast(); any valid
encoder's stream must decode to the same bytes) and the two error messages for b"invalid format";
for valid streams CPython's zlib (an independent DEFLATE implementation) is the cross-check over
every block type (stored / fixed / dynamic), strategy and level.
"""
import zlib

import numpy as np
import pytest

from oracle import py_oracle as oracle
from reductionist_amd import _abi

GZIP, ZLIB = 1, 2


def gz(b, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, 31, 9, strategy)
    return c.compress(b) + c.flush()


def zl(b, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, 15, 9, strategy)
    return c.compress(b) + c.flush()


STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FILTERED]


def payload(rng, kind, n):
    if kind == 0:
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()          # incompressible: stored blocks
    if kind == 1:
        return rng.integers(0, 4, n, dtype=np.uint8).tobytes()            # short codes, long matches
    if kind == 2:
        return (np.arange(n) % 251).astype(np.uint8).tobytes()            # periodic: far matches
    return rng.standard_normal(n // 4 + 1).astype(np.float32).tobytes()  # float chunk


@pytest.mark.parametrize("comp", [GZIP, ZLIB])
def test_reference_kats(comp):
    # compression.rs:136-150 / filter_pipeline.rs:56-64
    for data in (b"hello world", bytes([1, 2, 3, 4])):
        stream = gz(data, 1) if comp == GZIP else zl(data, 1)
        e, out = oracle.decompress(comp, stream, len(data))
        assert e == 0 and out == data


def test_reference_error_messages():
    # compression.rs:166-190: b"invalid format" -> "invalid gzip header" / "Unknown zlib compression method 9"
    e, _ = oracle.decompress(GZIP, b"invalid format")
    assert e == _abi.INFLATE_GZIP_HEADER
    e, _ = oracle.decompress(ZLIB, b"invalid format")
    assert e == _abi.INFLATE_ZLIB_METHOD


def test_matches_cpython_zlib_all_block_types():
    rng = np.random.default_rng(1)
    for trial in range(60):
        b = payload(rng, trial % 4, int(rng.integers(0, 200000)))
        level = int(rng.integers(0, 10))
        strategy = STRATEGIES[trial % 5]
        for comp, f in ((GZIP, gz), (ZLIB, zl)):
            stream = f(b, level, strategy)
            e, out = oracle.decompress(comp, stream, len(b) + 16)
            assert e == 0 and out == b, (trial, comp, e)
            if b:  # one byte short of the output -> overflow, never a wrong answer
                e2, _ = oracle.decompress(comp, stream, len(b) - 1)
                assert e2 == _abi.INFLATE_OUTPUT_OVERFLOW


def test_corrupt_streams():
    b = bytes(range(256)) * 1000
    s = bytearray(zl(b))
    s[-1] ^= 1
    assert oracle.decompress(ZLIB, bytes(s), len(b))[0] == _abi.INFLATE_CHECKSUM
    s = bytearray(gz(b))
    s[-6] ^= 1
    assert oracle.decompress(GZIP, bytes(s), len(b))[0] == _abi.INFLATE_CHECKSUM
    s = bytearray(gz(b))
    s[-2] ^= 1                                           # ISIZE
    assert oracle.decompress(GZIP, bytes(s), len(b))[0] == _abi.INFLATE_CHECKSUM
    assert oracle.decompress(ZLIB, zl(b)[:100], len(b))[0] == _abi.INFLATE_TRUNCATED
    assert oracle.decompress(GZIP, gz(b)[:-3], len(b))[0] == _abi.INFLATE_TRUNCATED
    # zlib header checks: CINFO > 7, FCHECK, FDICT
    assert oracle.decompress(ZLIB, bytes([0x88, 0x1c]) + zl(b)[2:], len(b))[0] == _abi.INFLATE_ZLIB_HEADER
    assert oracle.decompress(ZLIB, bytes([0x78, 0x9d]) + zl(b)[2:], len(b))[0] == _abi.INFLATE_ZLIB_HEADER
    assert oracle.decompress(ZLIB, bytes([0x78, 0xbb]) + zl(b)[2:], len(b))[0] == _abi.INFLATE_ZLIB_HEADER
    # reserved block type 3 right after a valid zlib header
    assert oracle.decompress(ZLIB, bytes([0x78, 0x9c, 0x07]), 16)[0] == _abi.INFLATE_BLOCK_TYPE
    # stored block with LEN != ~NLEN
    assert oracle.decompress(ZLIB, bytes([0x78, 0x9c, 0x01, 0x05, 0x00, 0x00, 0x00]), 16)[0] == \
        _abi.INFLATE_STORED_LENGTH


def test_gzip_header_fields_and_trailing_bytes():
    data = b"reductionist " * 50
    body = zlib.compressobj(6, zlib.DEFLATED, -15)
    raw = body.compress(data) + body.flush()
    crc = zlib.crc32(data).to_bytes(4, "little")
    size = len(data).to_bytes(4, "little")
    # FLG = FEXTRA | FNAME | FCOMMENT | FHCRC
    hdr = bytes([0x1F, 0x8B, 8, 4 | 8 | 16 | 2, 0, 0, 0, 0, 0, 3]) + (3).to_bytes(2, "little") + b"xyz" \
        + b"name\0" + b"comment\0" + b"\x00\x00"
    e, out = oracle.decompress(GZIP, hdr + raw + crc + size + b"trailing garbage", len(data))
    assert e == 0 and out == data
    bad_cm = hdr[:2] + bytes([7]) + hdr[3:]
    assert oracle.decompress(GZIP, bad_cm + raw + crc + size, len(data))[0] == _abi.INFLATE_GZIP_HEADER


def test_operation_with_compression_and_filters():
    # filter_pipeline.rs:66-120: zlib + shuffle chains; app.rs:169-172 raw-size validation afterwards
    vals = np.arange(1, 4097, dtype=np.int32)
    sh = oracle.shuffle(vals.tobytes(), 4)
    creq = _abi.CRequest("sum", "int32", compression="zlib", filters=[{"id": "shuffle", "element_size": 4}])
    st, info, body, counts = oracle.execute(creq, zl(sh))
    assert st == 0 and int(np.frombuffer(body, np.int32)[0]) == int(vals.sum()) and counts == [4096]
    # a shape that does not match the decompressed size -> validation error (400), even with `size`
    creq = _abi.CRequest("sum", "int32", compression="gzip", shape=[4095], size=123)
    st, *_ = oracle.execute(creq, gz(vals.tobytes()))
    assert st == _abi.E_REQUEST_VALIDATION
    creq = _abi.CRequest("sum", "int32", compression="gzip")
    st, *_ = oracle.execute(creq, b"invalid format")
    assert st == _abi.E_DECOMPRESSION
    assert oracle.lib().oracle_inflate_last_error() == _abi.INFLATE_GZIP_HEADER
    creq = _abi.CRequest("sum", "int32", compression="blosc2")
    st, *_ = oracle.execute(creq, b"\0" * 64)
    assert st == _abi.E_DECOMPRESSION and oracle.lib().oracle_inflate_last_error() == _abi.BLOSC2_INVALID


def test_oracle_decodes_gnu_gzip_members():
    """A second encoder pins the oracle: members written by GNU gzip 1.10 (its own deflate, not zlib;
    tests/golden/make_gnu_gzip.py) decode to the inputs' bytes (SHA-256 in the manifest), as CPython's
    zlib decodes them."""
    import hashlib
    import json
    from pathlib import Path
    d = Path(__file__).resolve().parent / "golden" / "gnu_gzip"
    man = json.loads((d / "manifest.json").read_text())
    for m in man["members"]:
        s = (d / m["file"]).read_bytes()
        err, out = oracle.decompress(GZIP, s, m["raw_bytes"] + 64)
        assert err == 0 and len(out) == m["raw_bytes"], m["file"]
        assert hashlib.sha256(out).hexdigest() == m["sha256"] == hashlib.sha256(zlib.decompress(s, 31)).hexdigest()
    # the inputs regenerate bit for bit from the committed script
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_gnu_gzip", d.parent / "make_gnu_gzip.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    ins = mod.inputs()
    for m in man["members"]:
        assert hashlib.sha256(ins[m["input"]]).hexdigest() == m["sha256"]
