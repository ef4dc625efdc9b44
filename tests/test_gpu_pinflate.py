"""MI355X parity of the single-stream parallel inflate (k_pinflate.hip): a lone gzip / zlib stream
(src/compression.rs:60-82, one request = one chunk, app.rs:163-183) decoded by the whole device, against
the original bytes and the oracle (oracle/oracle_inflate.cpp, pinned in tests/test_inflate_cpu.py), through
the C ABI (rdx_decompress_one_device, rdx_execute).

* valid streams of every kind the encoders write — zlib levels 0-9 and all five strategies over incompressible
  bytes (stored blocks), short-alphabet bytes, periodic bytes, float chunks, the BASELINE C4-shaped chunk
  (shuffled N(0,1) f32, zlib level 1), gzip headers with FNAME / FCOMMENT / FEXTRA / FHCRC, unaligned
  starts, empty and tiny streams — decode byte-identical, and the device says the parallel path produced
  them (rdx_inflate_last_path) wherever the stream's blocks are Huffman or stored ones;
* corrupt streams (random byte flips anywhere, truncations, trailer damage) give exactly the oracle's
  error: the parallel path never accepts a stream the sequential decoder rejects;
* the reference's own gzip / zlib KATs (filter_pipeline.rs:56-120) through rdx_decompress_one_device;
* compressed requests end to end through rdx_execute (decompress -> filters -> operation)."""
import gzip
import io
import json
import zlib
from pathlib import Path

import numpy as np
import pytest

from helpers import make_request, product_convert
from oracle import py_oracle as oracle
from reductionist_amd import _abi
from test_inflate_cpu import STRATEGIES, gz, payload, zl

pytestmark = pytest.mark.gpu

GZIP, ZLIB = 1, 2
NAMES = {GZIP: "gzip", ZLIB: "zlib"}
PATH_PARALLEL, PATH_FALLBACK = 2, 3
GOLDEN = Path(__file__).resolve().parent / "golden" / "kats.json"


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def one(torch, ws, comp, stream, cap=None, skew=0):
    """Decode one stream placed at a 256-byte boundary + skew; returns (err, bytes, path)."""
    host = np.zeros(skew + len(stream) + 16, dtype=np.uint8)
    host[skew:skew + len(stream)] = np.frombuffer(stream, dtype=np.uint8)
    d_in = torch.from_numpy(host).cuda()
    cap = cap if cap is not None else 4 * len(stream) + (1 << 20)
    d_out = torch.zeros(max(16, cap), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    err, n, path = ws.decompress_one_device(NAMES[comp], d_in.data_ptr() + skew, len(stream), d_out.data_ptr(), cap)
    out = d_out[:n].cpu().numpy().tobytes() if err == 0 else b""
    return err, out, path


def c4_chunk(seed):
    v = np.random.default_rng(seed).standard_normal(1 << 20).astype(np.float32)
    return v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()   # byte-shuffled (es = 4), as bench.py leg_inflate


@pytest.mark.parametrize("comp", [ZLIB, GZIP])
def test_bench_chunk_level1_parallel(torch, workspace, comp):
    """The bench's lone chunk: 4 MiB shuffled N(0,1) f32 at zlib level 1 (191 stored + 20 Huffman blocks)."""
    raw = c4_chunk(0x5EED2000)
    stream = (gz if comp == GZIP else zl)(raw, 1)
    err, out, path = one(torch, workspace, comp, stream)
    assert err == 0 and out == raw and path == PATH_PARALLEL


@pytest.mark.parametrize("comp", [ZLIB, GZIP])
@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_levels_strategies_kinds(torch, workspace, comp, kind):
    rng = np.random.default_rng(100 * comp + kind)
    for level in (0, 1, 3, 6, 9):
        for strategy in STRATEGIES:
            n = int(rng.integers(1, 600000))
            b = payload(rng, kind, n)
            s = (gz if comp == GZIP else zl)(b, level, strategy)
            skew = int(rng.integers(0, 4))
            err, out, path = one(torch, workspace, comp, s, skew=skew)
            oe, oout = oracle.decompress(comp, s, len(b) + 64)
            assert err == oe == 0 and out == b == oout, (level, strategy, n, err, oe)
            # Huffman / stored blocks decode on the parallel path; a stream of many fixed-Huffman blocks
            # (Z_FIXED) may exceed the host's per-block rounds and go to k_inflate, still byte-exact
            if strategy != zlib.Z_FIXED:
                assert path == PATH_PARALLEL, (level, strategy, n, path)
            else:
                assert path in (PATH_PARALLEL, PATH_FALLBACK)


@pytest.mark.parametrize("comp", [ZLIB, GZIP])
def test_shapes_of_data(torch, workspace, comp):
    """Highly compressible periodic chunks (long matches, few blocks, parses that keep apart), integer-
    valued floats, text, and sizes around the block / window edges."""
    rng = np.random.default_rng(5 + comp)
    datas = [
        (np.arange(1 << 20) % 1000).astype(np.float32).tobytes(),
        rng.integers(-8, 9, 1 << 20).astype(np.float32).tobytes(),
        b"".join(b"line %d of some text with words %d\n" % (i, i * 7 % 13) for i in range(60000)),
        bytes(1 << 22),
        bytes([7]) * 65536 + rng.integers(0, 256, 40000, dtype=np.uint8).tobytes() + bytes(300000),
        rng.integers(0, 256, 32768, dtype=np.uint8).tobytes() * 9,
    ]
    for b in datas:
        for level in (1, 6, 9):
            s = (gz if comp == GZIP else zl)(b, level)
            err, out, path = one(torch, workspace, comp, s, cap=len(b) + 64)
            assert err == 0 and out == b and path == PATH_PARALLEL, (len(b), level, err, path)


def test_gzip_header_fields(torch, workspace):
    b = np.random.default_rng(9).integers(0, 20, 300000, dtype=np.uint8).tobytes()
    body = gz(b, 6)[10:]                       # raw DEFLATE + trailer behind a 10-byte header
    heads = [
        bytes([0x1f, 0x8b, 8, 0x08, 0, 0, 0, 0, 0, 3]) + b"name.nc\x00",                         # FNAME
        bytes([0x1f, 0x8b, 8, 0x10, 0, 0, 0, 0, 0, 3]) + b"a comment\x00",                       # FCOMMENT
        bytes([0x1f, 0x8b, 8, 0x04, 0, 0, 0, 0, 0, 3]) + bytes([5, 0]) + b"extra",              # FEXTRA
        bytes([0x1f, 0x8b, 8, 0x1e, 0, 0, 0, 0, 0, 3]) + bytes([2, 0]) + b"xy" + b"n\x00" + b"c\x00" + b"\x12\x34",
    ]
    for h in heads:
        s = h + body
        err, out, path = one(torch, workspace, GZIP, s)
        oe, oout = oracle.decompress(GZIP, s, len(b) + 64)
        assert err == oe == 0 and out == b and path == PATH_PARALLEL
    # CPython's gzip module (mtime, FNAME) and trailing bytes after the member (ignored by GzDecoder)
    bio = io.BytesIO()
    with gzip.GzipFile("chunk.bin", "wb", 6, bio, mtime=1) as f:
        f.write(b)
    s = bio.getvalue() + b"trailing garbage"
    err, out, path = one(torch, workspace, GZIP, s)
    oe, _ = oracle.decompress(GZIP, s, len(b) + 64)
    assert err == oe == 0 and out == b and path == PATH_PARALLEL


@pytest.mark.parametrize("comp", [ZLIB, GZIP])
def test_tiny_and_empty(torch, workspace, comp):
    for b in (b"", b"a", b"hello world", bytes([1, 2, 3, 4]), bytes(range(256)) * 3):
        for level in (0, 1, 9):
            s = (gz if comp == GZIP else zl)(b, level)
            err, out, path = one(torch, workspace, comp, s)
            oe, oout = oracle.decompress(comp, s, len(b) + 64)
            assert err == oe == 0 and out == b == oout, (b[:8], level)
            assert path in (PATH_PARALLEL, PATH_FALLBACK)


def test_reference_kats(torch, workspace):
    """The reference's gzip / zlib pipeline KATs (filter_pipeline.rs:56-120, compression.rs:136-190): the
    streams decode to the bytes the reference's tests expect."""
    kats = [k for k in json.loads(GOLDEN.read_text()) if k.get("request", {}).get("compression") in ("gzip", "zlib")]
    assert kats
    for k in kats:
        comp = GZIP if k["request"]["compression"] == "gzip" else ZLIB
        s = bytes.fromhex(k["data"])
        err, out, _ = one(torch, workspace, comp, s)
        oe, oout = oracle.decompress(comp, s, 1 << 16)
        assert err == oe, k["name"]
        if err == 0:
            assert out == oout, k["name"]
    for comp, detail in ((GZIP, _abi.INFLATE_GZIP_HEADER), (ZLIB, _abi.INFLATE_ZLIB_METHOD)):
        err, _, _ = one(torch, workspace, comp, b"invalid format")
        assert err == detail


@pytest.mark.parametrize("comp", [ZLIB, GZIP])
def test_corruption_gives_the_oracle_error(torch, workspace, comp):
    """Never more lenient than the sequential decoder: flips anywhere (headers, Huffman bodies, stored data,
    the trailer), truncations; the error code equals the oracle's, and where the oracle decodes, the bytes."""
    rng = np.random.default_rng(77 + comp)
    b = c4_chunk(0x5EED2001)[: 1 << 20] + rng.integers(-8, 9, 1 << 18).astype(np.float32).tobytes()
    good = (gz if comp == GZIP else zl)(b, 1)
    cases = [good[:len(good) // 2], good[:-1], good[:-5], good[:-9]]
    for _ in range(40):
        c = bytearray(good)
        for _ in range(int(rng.integers(1, 4))):
            c[int(rng.integers(0, len(c)))] ^= int(rng.integers(1, 256))
        cases.append(bytes(c))
    for _ in range(10):                           # flips inside the Huffman-coded tail (the exponent plane)
        c = bytearray(good)
        c[int(rng.integers(len(c) * 3 // 4, len(c)))] ^= 1 << int(rng.integers(0, 8))
        cases.append(bytes(c))
    cap = len(b) + 4096
    for i, c in enumerate(cases):
        err, out, path = one(torch, workspace, comp, c, cap=cap)
        oe, oout = oracle.decompress(comp, c, cap)
        assert err == oe, (i, err, oe)
        if err == 0:
            assert out == oout
        else:
            assert path == PATH_FALLBACK, (i, path)


def test_output_capacity(torch, workspace):
    b = np.arange(300000, dtype=np.uint32).tobytes()
    s = zl(b, 6)
    err, _, _ = one(torch, workspace, ZLIB, s, cap=4096)
    assert err == _abi.INFLATE_OUTPUT_OVERFLOW
    err, out, path = one(torch, workspace, ZLIB, s, cap=len(b))
    assert err == 0 and out == b and path == PATH_PARALLEL


@pytest.mark.parametrize("comp", ["zlib", "gzip"])
def test_lone_request_end_to_end(engine, comp):
    """rdx_execute with a compressed lone request (C4's chunk: shuffled f32 sum), as the plugin sends it:
    the chunk is decoded by the whole device, then unshuffled and summed; the response equals the oracle's."""
    rng = np.random.default_rng(31)
    v = rng.integers(-8, 9, 1 << 20).astype(np.float32)
    raw = oracle.shuffle(v.tobytes(), 4)
    stream = (gz if comp == "gzip" else zl)(raw, 1)
    req = {"dtype": "float32", "compression": comp, "filters": [{"id": "shuffle", "element_size": 4}]}
    creq = make_request("sum", req, product_convert)
    st, info, body, counts = engine.execute_raw(creq, stream)
    ost, oinfo, obody, ocounts = oracle.execute(creq, stream)
    assert st == ost == 0 and body == obody and counts == ocounts
    assert _abi.lib().rdx_inflate_last_path() == PATH_PARALLEL
