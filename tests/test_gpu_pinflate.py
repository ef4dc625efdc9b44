"""MI355X parity of the single-stream parallel inflate (k_pinflate.hip): a lone gzip / zlib stream
(src/compression.rs:60-82, one request = one chunk, app.rs:163-183) decoded by the whole device, against
the original bytes and the oracle (oracle/oracle_inflate.cpp, pinned in tests/test_inflate_cpu.py), through
the C ABI (rdx_decompress_one_device, rdx_execute).

* valid streams of every kind the encoders write — zlib levels 0-9 and all five strategies over incompressible
  bytes (stored blocks), short-alphabet bytes, periodic bytes, float chunks, the BASELINE C4-shaped chunk
  (shuffled N(0,1) f32, zlib level 1), gzip headers with FNAME / FCOMMENT / FEXTRA / FHCRC, unaligned
  starts, empty and tiny streams — decode byte-identical, and the device says the parallel path produced
  them (rdx_inflate_last_path) wherever the stream's blocks are Huffman or stored ones;
* corrupt streams (random byte flips anywhere, truncations, trailer damage): the parallel path never accepts
  a stream the sequential decoder rejects — by default it declines them (RDX_UNSUPPORTED_INFLATE_DECLINED,
  the caller's host decoder answers), and with inflate_fallback the device's k_inflate gives exactly the
  oracle's error;
* streams written by GNU gzip (its own deflate, not zlib: tests/golden/gnu_gzip, make_gnu_gzip.py) decode on
  the parallel path;
* a declined lone stream costs little more than the parallel attempt (no one-wavefront k_inflate);
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
PATH_PARALLEL, PATH_FALLBACK, PATH_DECLINED = 2, 3, 4
GOLDEN = Path(__file__).resolve().parent / "golden" / "kats.json"
GNU = Path(__file__).resolve().parent / "golden" / "gnu_gzip"


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def serial_ws(torch):
    """A workspace of a context with inflate_fallback on: a stream k_pinflate declines is decoded by the
    device's sequential k_inflate (its bytes or its error) instead of going back to the caller."""
    from reductionist_amd import Engine
    eng = Engine()
    eng.configure(inflate_fallback=True)
    ws = eng.workspace(0)
    yield ws
    ws.close()
    eng.close()


def one(torch, ws, comp, stream, cap=None, skew=0):
    """Decode one stream placed at a 256-byte boundary + skew; returns (err, bytes, path) — err None when
    the stream was declined (path PATH_DECLINED)."""
    host = np.zeros(skew + len(stream) + 16, dtype=np.uint8)
    host[skew:skew + len(stream)] = np.frombuffer(stream, dtype=np.uint8)
    d_in = torch.from_numpy(host).cuda()
    cap = cap if cap is not None else 4 * len(stream) + (1 << 20)
    d_out = torch.zeros(max(16, cap), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    err, n, path = ws.decompress_one_device(NAMES[comp], d_in.data_ptr() + skew, len(stream), d_out.data_ptr(), cap)
    assert (err is None) == (path == PATH_DECLINED)
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
def test_levels_strategies_kinds(torch, workspace, serial_ws, comp, kind):
    rng = np.random.default_rng(100 * comp + kind)
    for level in (0, 1, 3, 6, 9):
        for strategy in STRATEGIES:
            n = int(rng.integers(1, 600000))
            b = payload(rng, kind, n)
            s = (gz if comp == GZIP else zl)(b, level, strategy)
            skew = int(rng.integers(0, 4))
            err, out, path = one(torch, workspace, comp, s, skew=skew)
            oe, oout = oracle.decompress(comp, s, len(b) + 64)
            assert oe == 0 and oout == b
            # Huffman / stored blocks decode on the parallel path; a stream of many fixed-Huffman blocks
            # (Z_FIXED) takes a host round trip per block start no candidate covers and is declined after a
            # few (or, up to 4 KiB, decoded by k_inflate) — byte-exact whichever decoder answers
            if strategy != zlib.Z_FIXED:
                assert path == PATH_PARALLEL and err == 0 and out == b, (level, strategy, n, err, path)
            elif path == PATH_DECLINED:
                assert len(s) > 4096
                err, out, path = one(torch, serial_ws, comp, s, skew=skew)
                assert err == 0 and out == b and path == PATH_FALLBACK
            else:
                assert path in (PATH_PARALLEL, PATH_FALLBACK) and err == 0 and out == b


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
def test_corruption_gives_the_oracle_error(torch, workspace, serial_ws, comp):
    """Never more lenient than the sequential decoder: flips anywhere (headers, Huffman bodies, stored data,
    the trailer), truncations.  Default context: a stream the oracle rejects is declined (the caller's host
    decoder answers), one it accepts decodes to its bytes.  inflate_fallback: the error code equals the
    oracle's, and where the oracle decodes, the bytes."""
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
        oe, oout = oracle.decompress(comp, c, cap)
        err, out, path = one(torch, workspace, comp, c, cap=cap)
        if oe != 0:
            assert path == PATH_DECLINED, (i, err, oe, path)
        else:
            assert err == 0 and out == oout and path in (PATH_PARALLEL, PATH_DECLINED), (i, err, path)
        err, out, path = one(torch, serial_ws, comp, c, cap=cap)
        assert err == oe, (i, err, oe)
        if err == 0:
            assert out == oout
        else:
            assert path == PATH_FALLBACK, (i, path)


def test_gnu_gzip_streams(torch, workspace):
    """Members written by GNU gzip 1.10 (its own deflate.c / trees.c: block boundaries, stored / fixed /
    dynamic choice and code-length headers of its own) — committed fixtures, tests/golden/make_gnu_gzip.py.
    Each decodes on the parallel path to the input's bytes (SHA-256 in the manifest) and the oracle's."""
    import hashlib
    man = json.loads((GNU / "manifest.json").read_text())
    assert len(man["members"]) >= 8
    for m in man["members"]:
        s = (GNU / m["file"]).read_bytes()
        err, out, path = one(torch, workspace, GZIP, s, cap=m["raw_bytes"] + 64)
        oe, oout = oracle.decompress(GZIP, s, m["raw_bytes"] + 64)
        assert oe == 0 and hashlib.sha256(oout).hexdigest() == m["sha256"], m["file"]
        assert err == 0 and out == oout, (m["file"], err, path)
        if m["gz_bytes"] > 4096:
            assert path == PATH_PARALLEL, (m["file"], path)


@pytest.mark.parametrize("comp", [ZLIB, GZIP])
def test_declined_stream_costs_little(torch, workspace, comp):
    """The cliff verdict r04 named: a lone 4 MiB stream the parallel path declines (Z_FIXED: a fixed-Huffman
    block per 16 K symbols, none of them a finder candidate; and a corrupt stream) must come back fast — it
    used to run the one-wavefront k_inflate, 100-220 ms.  Bound: 20 ms, far above the decline's cost
    (finder + block decode + a few host round trips) and far below the old route."""
    import time
    rng = np.random.default_rng(2024 + comp)
    b = rng.integers(-8, 9, 1 << 20).astype(np.float32).tobytes()
    fixed = (gz if comp == GZIP else zl)(b, 6, zlib.Z_FIXED)
    bad = bytearray((gz if comp == GZIP else zl)(b, 6))
    bad[-6] ^= 0x40                          # the trailer: every block decodes, the checksum fails
    for s in (fixed, bytes(bad)):
        one(torch, workspace, comp, s, cap=len(b) + 64)          # warm (allocations)
        t0 = time.perf_counter()
        err, _, path = one(torch, workspace, comp, s, cap=len(b) + 64)
        dt = time.perf_counter() - t0
        if path == PATH_DECLINED:
            assert dt < 0.020, dt
        else:
            assert s is fixed and err == 0 and path == PATH_PARALLEL


def test_candidate_overflow_declines(torch, workspace):
    """More block-start candidates than one stream's list holds (kPinfMaxCand, 4096): a Z_HUFFMAN_ONLY stream
    at memLevel 9 writes a block per 32 K literals, so 160 MiB is ~5100 blocks.  The parallel path declines it (the caller's
    host decoder answers) quickly instead of failing or taking the sequential decoder."""
    import time
    b = np.random.default_rng(77).integers(0, 16, 160 << 20, dtype=np.uint8).tobytes()
    s = zl(b, 1, zlib.Z_HUFFMAN_ONLY)
    t0 = time.perf_counter()
    err, _, path = one(torch, workspace, ZLIB, s, cap=len(b) + 64)
    dt = time.perf_counter() - t0
    assert path == PATH_DECLINED and err is None, (err, path)
    assert dt < 0.5, dt


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
    the chunk is decoded by the whole device, then unshuffled and summed; the response equals the oracle's.
    A declined stream (Z_FIXED) comes back as RDX_E_UNSUPPORTED / INFLATE_DECLINED, and the operations mirror
    (reductionist_amd.operations, as integration/app_gpu.rs) decompresses it on the host and runs it
    uncompressed: the same response."""
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
    from reductionist_amd import operations
    from reductionist_amd.models import RequestData
    fixed = (gz if comp == "gzip" else zl)(raw, 6, zlib.Z_FIXED)
    st, _, _, _ = engine.execute_raw(creq, fixed)
    if st == _abi.E_UNSUPPORTED:
        assert _abi.lib().rdx_last_unsupported_reason() == _abi.UNSUPPORTED_INFLATE_DECLINED
        assert _abi.lib().rdx_inflate_last_path() == PATH_DECLINED
    rd = RequestData.from_json({"interface_type": "s3", "url": "http://x/y", "dtype": "float32",
                                "compression": {"id": comp}, "filters": [{"id": "shuffle", "element_size": 4}]})
    resp = operations.Sum.execute(rd, fixed, engine)
    assert resp.body == obody and resp.count == ocounts
