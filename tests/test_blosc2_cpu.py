"""blosc2 decompression (src/compression.rs:29-57) — the oracle (oracle/oracle_blosc2.cpp) and the host
part of the C ABI (rdx_blosc2_cbuffer_sizes), no GPU.

Pinned by the reference's own tests where they exist (compression.rs:112-119 test_decompress_blosc:
b"hello world" compressed by blosc2_compress(clevel 5, BLOSC_SHUFFLE, typesize 1) — below the minimum
buffer size blosc stores it memcpy'ed behind a 32-byte header, rebuilt here from the published chunk
format; compression.rs:130-140 test_decompress_invalid_blosc: b"invalid format" ->
"invalid blosc2 compressed data").  Everything else is PARITY UNPINNED (no blosc2 library in the
image): chunks come from this repo's own writer (datagen/blosc2_chunk.py) and are checked for round
trips, the frozen fixtures in tests/golden/blosc2_chunks.json, and the error taxonomy."""
import hashlib
import itertools
import json
import struct
from pathlib import Path

import numpy as np
import pytest

from datagen import blosc2_chunk as B
from oracle import py_oracle as oracle
from reductionist_amd import _abi

GOLDEN = Path(__file__).parent / "golden" / "blosc2_chunks.json"


def payload(rng, n, kind):
    """Test data: smooth (compressible after shuffle), small integers, random bytes, constant."""
    if kind == "smooth":
        x = np.cumsum(rng.standard_normal(n // 4 + 1)).astype(np.float32)
        return x.tobytes()[:n]
    if kind == "ints":
        return rng.integers(0, 40, n // 4 + 1).astype(np.int32).tobytes()[:n]
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    return bytes([7]) * n


def test_reference_hello_world_and_invalid():
    # test_decompress_blosc (compression.rs:112-119): a memcpy'ed chunk, version 5, typesize 1
    c = B.build(b"hello world", typesize=1, codec=B.BLOSCLZ, filters=(0, 0, 0, 0, 0, B.SHUFFLE))
    assert len(c) == 32 + 11 and c[2] & 0x02
    assert oracle.blosc2_sizes(c) == (11, 43, 11) == _abi.blosc2_cbuffer_sizes(c)
    assert oracle.blosc2_decompress(c) == (0, b"hello world")
    # test_decompress_invalid_blosc (compression.rs:130-140)
    assert oracle.blosc2_sizes(b"invalid format") == (0, 0, 0) == _abi.blosc2_cbuffer_sizes(b"invalid format")
    assert oracle.blosc2_decompress(b"invalid format")[0] == _abi.BLOSC2_INVALID
    assert _abi.inflate_error_string(_abi.BLOSC2_INVALID) == "invalid blosc2 compressed data"
    assert _abi.inflate_error_string(_abi.BLOSC2_FAILED) == "failed to decompress blosc2 data"
    assert _abi.inflate_error_string(_abi.BLOSC2_SIZE) == "unexpected decompressed size for blosc2 data"


CASES = list(itertools.product(
    [B.BLOSCLZ, B.LZ4, B.SNAPPY, B.ZLIB],                         # codec
    [1, 4, 8],                                                    # typesize
    [None, 1000, 16384],                                          # blocksize (None: 64 KiB)
    [True, False],                                                # split streams
    [(0,) * 6, (0, 0, 0, 0, 0, B.SHUFFLE), (0, 0, 0, 0, 0, B.BITSHUFFLE), (0, 0, 0, 0, B.SHUFFLE, B.BITSHUFFLE)],
    [5, 2]))                                                      # version (2: 16-byte blosc1 header)


@pytest.mark.parametrize("kind", ["smooth", "ints", "random", "const"])
def test_roundtrip_every_layout(kind):
    rng = np.random.default_rng(len(kind))
    fails = []
    for n in (1, 13, 4096, 65536 + 13, 200000):
        d = payload(rng, n, kind)
        for codec, ts, bs, split, filt, ver in CASES:
            if ver == 2 and filt.count(0) < 5:
                continue   # the blosc1 header carries one shuffle flag
            c = B.build(d, ts, bs, codec, filt, split, ver)
            assert oracle.blosc2_sizes(c) == _abi.blosc2_cbuffer_sizes(c)
            e, out = oracle.blosc2_decompress(c)
            if e or out != d:
                fails.append((n, codec, ts, bs, split, filt, ver, e))
    assert not fails, fails[:5]


def test_stream_forms_and_specials():
    rng = np.random.default_rng(3)
    d = payload(rng, 50000, "ints")
    for mode in ("auto", "raw"):
        c = B.build(d, 4, 8192, B.LZ4, stream_mode=mode, memcpyed=False)
        assert oracle.blosc2_decompress(c) == (0, d)
    # zero and byte-run streams (csize 0 / -byte + token)
    z = bytes(4096) + bytes([9]) * 4096
    c = B.build(z, 4, 4096, B.BLOSCLZ, memcpyed=False)
    assert struct.unpack_from("<i", c, 32 + 8)[0] == 0
    assert oracle.blosc2_decompress(c) == (0, z)
    # special-value chunks
    assert oracle.blosc2_decompress(B.special(64, 4, 1)) == (0, bytes(64))
    assert oracle.blosc2_decompress(B.special(64, 4, 2)) == (0, np.full(16, np.nan, np.float32).tobytes())
    assert oracle.blosc2_decompress(B.special(64, 8, 2)) == (0, np.full(8, np.nan, np.float64).tobytes())
    assert oracle.blosc2_decompress(B.special(64, 4, 3, b"\1\2\3\4")) == (0, b"\1\2\3\4" * 16)


def test_error_taxonomy():
    rng = np.random.default_rng(4)
    d = payload(rng, 70000, "smooth")
    good = B.build(d, 4, 16384, B.BLOSCLZ, memcpyed=False)
    assert oracle.blosc2_decompress(good) == (0, d)
    F, I, U = _abi.BLOSC2_FAILED, _abi.BLOSC2_INVALID, _abi.BLOSC2_UNSUPPORTED
    bad = bytearray(good)
    bad[0] = 6                                              # version above 5
    assert oracle.blosc2_decompress(bytes(bad))[0] == I
    assert oracle.blosc2_decompress(good[:-1])[0] == F      # cbytes > length
    bad = bytearray(good)
    bad[2] = (bad[2] & 0x1F) | (6 << 5)                    # a user-defined codec
    assert oracle.blosc2_decompress(bytes(bad))[0] == U
    bad = bytearray(good)
    bad[2] = (bad[2] & 0x1F) | (B.ZSTD << 5)               # BloscLZ streams read as zstd frames
    assert oracle.blosc2_decompress(bytes(bad))[0] == F
    bad = bytearray(good)
    bad[21] = B.DELTA                                       # delta filter
    assert oracle.blosc2_decompress(bytes(bad))[0] == U
    bad = bytearray(good)
    struct.pack_into("<i", bad, 32, 3)                      # bstarts[0] inside the header
    assert oracle.blosc2_decompress(bytes(bad))[0] == F
    bad = bytearray(good)
    bad[-20] ^= 0xFF                                        # corrupt the last stream
    assert oracle.blosc2_decompress(bytes(bad))[0] in (0, F)
    nb = oracle.blosc2_sizes(good)[0]
    assert oracle.blosc2_decompress(good, cap=nb - 1)[0] == _abi.INFLATE_OUTPUT_OVERFLOW


def test_golden_chunks_frozen():
    """tests/golden/blosc2_chunks.json (make_blosc2_golden.py): chunks from this repo's writer with the
    SHA-256 of their decoded bytes, so a change to writer or decoder that breaks the format shows."""
    g = json.loads(GOLDEN.read_text())
    assert len(g["chunks"]) >= 10
    for case in g["chunks"]:
        c = bytes.fromhex(case["chunk"])
        e, out = oracle.blosc2_decompress(c)
        assert e == case["error"], case["name"]
        if e == 0:
            assert hashlib.sha256(out).hexdigest() == case["sha256"] and len(out) == case["nbytes"], case["name"]


def test_execute_blosc2_request_oracle():
    """operation<T>() with compression blosc2 (app.rs:163-183): decompress, then filters and the op."""
    rng = np.random.default_rng(9)
    vals = rng.integers(-20, 20, 30000).astype(np.float32)
    raw = oracle.shuffle(vals.astype(">f4").tobytes(), 4)
    c = B.build(raw, 4, 16384, B.LZ4, memcpyed=False)
    creq = _abi.CRequest("sum", "float32", byte_order="big", compression="blosc2",
                         filters=[{"id": "shuffle", "element_size": 4}])
    st, info, body, counts = oracle.execute(creq, c)
    assert st == 0 and struct.unpack("<f", body)[0] == float(vals.astype(np.float64).sum()) and counts == [30000]


def v2_bitshuffle_chunks():
    """Hand-built c-blosc 1.x chunks (header version 2, 16-byte header, BITSHUFFLE flag, BloscLZ codec id,
    every stream stored raw: csize == stream size) -> (chunk, decoded bytes).  c-blosc 1.x bitshuffles a
    block only when its element count is a multiple of 8 and stores any other block unshuffled; c-blosc2
    decodes version-2 chunks by the same rule (bitunshuffle(..., format_version)).  Version 3+ instead
    bitshuffles the first floor(n/8)*8 elements and leaves the tail."""
    rng = np.random.default_rng(0xB175)
    out = []
    # (a) one block of 1001 f32 elements, one stream (DONTSPLIT): stored as it is
    d = rng.integers(0, 1 << 31, 1001, dtype=np.uint32).tobytes()
    h = struct.pack("<BBBBiii", 2, 1, 0x04 | 0x10, 4, len(d), len(d), 16 + 4 + 4 + len(d))
    out.append((h + struct.pack("<i", 20) + struct.pack("<i", len(d)) + d, d))
    # (b) a 2000-element block (bitshuffled, split into 4 raw streams) + a 1001-element leftover block
    d = rng.integers(0, 1 << 31, 3001, dtype=np.uint32).tobytes()
    blk0 = B.bitshuffle_block(d[:8000], 4)
    assert blk0 != d[:8000]
    streams0 = b"".join(struct.pack("<i", 2000) + blk0[k * 2000:(k + 1) * 2000] for k in range(4))
    b0 = 16 + 8
    b1 = b0 + len(streams0)
    body = streams0 + struct.pack("<i", 4004) + d[8000:]
    h = struct.pack("<BBBBiii", 2, 1, 0x04, 4, len(d), 8000, b0 + len(body))
    out.append((h + struct.pack("<ii", b0, b1) + body, d))
    return out


def test_version2_bitshuffle_leftover_rule():
    for c, d in v2_bitshuffle_chunks():
        assert oracle.blosc2_decompress(c) == (0, d)
        # the writer follows the same rule for version 2
        assert B.bitshuffle_block(d[-4004:], 4, version=2) == d[-4004:]
        # the same bytes read as a version-3 chunk take the newer rule: the odd block is bit-unshuffled
        c3 = bytes([3]) + c[1:]
        e3, d3 = oracle.blosc2_decompress(c3)
        assert e3 == 0 and d3 != d and d3[-4:] == d[-4:]


SNAPPY_BAD = [bytes([20, 0x0C]) + b"abcd" + bytes([0x11, 0, 0x11, 4]),    # offset 0
              bytes([20, 0x0C]) + b"abcd" + bytes([0x11, 5, 0x11, 4]),    # offset past the output
              bytes([21, 0x0C]) + b"abcd" + bytes([0x11, 4, 0x11, 4]),    # preamble longer than the elements
              bytes([19, 0x0C]) + b"abcd" + bytes([0x11, 4, 0x11, 4]),    # elements overrun the preamble
              bytes([20, 0x0C]) + b"abc",                                 # truncated literal
              bytes([20, 0x0C]) + b"abcd" + bytes([0x11, 4, 0x11]),       # truncated copy
              bytes([20, 0x0C]) + b"abcd" + bytes([0x3F, 4, 0, 0]),       # truncated copy-4
              bytes([0x94, 0x80, 0x80, 0x80, 0x80, 0x00]) + b"abcd"]     # 6-byte varint


def snappy_chunk(stream: bytes, nbytes: int) -> bytes:
    """One block, one stream (typesize 1), codec Snappy, no filter: the stream wrapped in a chunk."""
    base = 32 + 4
    body = struct.pack("<i", len(stream)) + stream
    h = struct.pack("<BBBBiii", 5, 1, 0x05 | (B.SNAPPY << 5) | 0x10, 1, nbytes, nbytes, base + len(body))
    h += bytes(6) + bytes([0, 0]) + bytes(6) + bytes([0, 0])
    return h + struct.pack("<i", base) + body


def test_snappy_element_forms_and_errors():
    """Snappy (codec 2; blusc -> the snap crate, raw format of google/snappy format_description.txt).
    A hand-assembled known answer from the format description, each element form, and malformed streams
    (zero / too-far offsets, preamble mismatches, truncation) -> "failed to decompress blosc2 data"."""
    F = _abi.BLOSC2_FAILED
    want = b"abcd" * 5
    # varint 20; literal "abcd" (tag 3 << 2); two copy-1 of len 8 offset 4 (tag 1 | 4 << 2, offset byte)
    kat = bytes([20, 0x0C]) + b"abcd" + bytes([0x11, 4, 0x11, 4])
    assert oracle.blosc2_decompress(snappy_chunk(kat, 20)) == (0, want)
    # copy-2 (len 16 = (15 << 2) | 2, offset 4 LE16) and copy-4 (LE32) give the same bytes
    for tail in (bytes([0x3E, 4, 0]), bytes([0x3F, 4, 0, 0, 0])):
        assert oracle.blosc2_decompress(snappy_chunk(bytes([20, 0x0C]) + b"abcd" + tail, 20)) == (0, want)
    # a literal with a 1-byte length extension (tag 60 << 2, length - 1 = 99), then a copy
    lit = bytes(range(100))
    assert oracle.blosc2_decompress(snappy_chunk(bytes([150, 1, 60 << 2, 99]) + lit + bytes([0xC6, 100, 0]), 150)) == \
        (0, lit + lit[:50])
    for stream in SNAPPY_BAD:
        assert oracle.blosc2_decompress(snappy_chunk(stream, 20))[0] == F, stream.hex()
    # this repo's encoder: far copies (copy-4 beyond 64 KiB), long literals (2-3 extension bytes)
    rng = np.random.default_rng(21)
    motif = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    d = motif + rng.integers(0, 256, 300, dtype=np.uint8).tobytes() + motif
    st = B.lz(B.SNAPPY, d, max_dist=1 << 30)
    assert any(st[i] & 3 == 3 for i in range(len(st)))   # (loose: some byte looks like a copy-4 tag)
    c = B.build(d, 1, len(d), B.SNAPPY, (0,) * 6, memcpyed=False)
    assert oracle.blosc2_decompress(c) == (0, d)
