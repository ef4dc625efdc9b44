"""zstd — the ZSTD codec of the reference's blosc2 branch (src/compression.rs:29-57 -> blusc 0.0.2 -> the
`zstd` crate, zstd-sys 2.0.16 = libzstd 1.5.7, Cargo.lock) — and the real-encoder pinning of the blosc2
LZ4 / Snappy streams.  No GPU.

The oracle (oracle/oracle_zstd.cpp, RFC 8878 restated) is checked against the REAL libzstd, liblz4 and
libsnappy bundled with pyarrow: frames / blocks written by the libraries at every level decode to the
input bytes, and libzstd's own decoder (pa.decompress) is the comparator on corrupted frames."""
import struct

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
xxhash = pytest.importorskip("xxhash")

from datagen import blosc2_chunk as B  # noqa: E402
from oracle import py_oracle as oracle  # noqa: E402
from reductionist_amd import _abi  # noqa: E402


def payload(rng, n, kind):
    if kind == "smooth":
        return np.cumsum(rng.standard_normal(n // 4 + 1)).astype(np.float32).tobytes()[:n]
    if kind == "ints":
        return rng.integers(0, 40, n // 4 + 1).astype(np.int32).tobytes()[:n]
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "text":
        return (b"the quick brown fox jumps over the lazy dog %d " * (n // 40 + 1))[:n]
    return bytes([7]) * n


def zstd(data, level=3):
    return pa.Codec("zstd", compression_level=level).compress(data, asbytes=True)


def libzstd_decompress(frame, n):
    try:
        return 0, pa.decompress(frame, decompressed_size=n, codec="zstd", asbytes=True)
    except Exception:   # noqa: BLE001 — any libzstd error
        return -1, b""


def test_xxh64_matches_xxhash():
    rng = np.random.default_rng(1)
    for n in (0, 1, 3, 4, 7, 8, 31, 32, 33, 63, 64, 100, 1000, 12345):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.xxh64(d) == xxhash.xxh64(d).intdigest(), n


@pytest.mark.parametrize("kind", ["smooth", "ints", "random", "text", "const"])
def test_libzstd_frames_every_level(kind):
    """Frames written by libzstd (levels -7 .. 22: raw / RLE / compressed blocks, Huffman literals with 1 and
    4 streams and treeless repeats, predefined / RLE / FSE / repeat sequence tables, multi-block frames)."""
    rng = np.random.default_rng(len(kind))
    for n in (1, 10, 100, 1000, 5000, 65536, 131073, 200000, 1 << 20):
        d = payload(rng, n, kind)
        for level in (-7, -1, 1, 3, 6, 9, 15, 19, 22):
            e, out = oracle.zstd_decompress(zstd(d, level), n)
            assert e == 0 and out == d, (kind, n, level, e)


def test_frame_forms():
    """Content checksum (XXH64 low 32 bits), skippable frames, concatenated frames, header errors."""
    rng = np.random.default_rng(2)
    d = payload(rng, 70000, "smooth")
    f = bytearray(zstd(d))
    assert f[4] & 0x04 == 0
    ck = bytearray(f)
    ck[4] |= 0x04                                   # Content_Checksum_flag
    good = bytes(ck) + struct.pack("<I", xxhash.xxh64(d).intdigest() & 0xFFFFFFFF)
    assert oracle.zstd_decompress(good, len(d)) == (0, d) == libzstd_decompress(good, len(d))
    wrong = good[:-1] + bytes([good[-1] ^ 1])
    assert oracle.zstd_decompress(wrong, len(d))[0] == -1 == libzstd_decompress(wrong, len(d))[0]
    skip = struct.pack("<II", 0x184D2A53, 5) + b"12345"
    d2 = payload(rng, 3000, "text")
    both = skip + bytes(f) + zstd(d2, 9)
    assert oracle.zstd_decompress(both, len(d) + len(d2)) == (0, d + d2)
    assert oracle.zstd_decompress(bytes(f), len(d) - 1)[0] == -1            # output does not fit
    for pos, val in ((0, 0x29), (4, f[4] | 0x08), (4, (f[4] & ~3) | 1)):     # magic, reserved bit, a dictionary
        b = bytearray(f)
        b[pos] = val
        if pos == 4 and val & 3:
            b[5:5] = b"\x07"                                              # the 1-byte dictionary id
        assert oracle.zstd_decompress(bytes(b), len(d))[0] == -1, (pos, val)
    assert oracle.zstd_decompress(b"", 10)[0] == -1
    assert oracle.zstd_decompress(bytes(f)[:-3], len(d))[0] == -1           # truncated


def test_corrupted_frames_never_more_lenient_than_libzstd():
    """Single-byte corruptions of libzstd frames, compared with libzstd 's own decoder: whenever the oracle
    decodes, libzstd decodes the same bytes; whenever libzstd fails, the oracle fails.  (The other
    direction is PARITY UNPINNED: libzstd 1.5.x's fast 4-stream Huffman path returns bytes for some
    corrupted literal streams that the RFC's exact-consumption rule — kept here and on the device —
    rejects as "failed to decompress".)"""
    rng = np.random.default_rng(7)
    stricter = 0
    for kind in ("smooth", "ints", "text", "random"):
        n = int(rng.integers(100, 300000))
        d = payload(rng, n, kind)
        f = zstd(d, int(rng.integers(1, 20)))
        for _ in range(120):
            b = bytearray(f)
            b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
            e1, o1 = oracle.zstd_decompress(bytes(b), n)
            e2, o2 = libzstd_decompress(bytes(b), n)
            if e1 == 0:
                assert e2 == 0 and o1 == o2
            if e2 != 0:
                assert e1 != 0
            stricter += e1 != 0 and e2 == 0
    assert stricter < 120   # a minority (observed ~9 %)


@pytest.mark.parametrize("codec", [B.LZ4, B.SNAPPY, B.ZSTD])
def test_blosc2_real_encoder_streams(codec):
    """blosc2 chunks whose streams come from the real liblz4 / libsnappy / libzstd (B.build enc="lib"), across
    typesizes, block sizes, split / unsplit streams and filters: the oracle decodes the input bytes."""
    rng = np.random.default_rng(codec)
    fails = []
    for kind in ("smooth", "ints", "random", "const"):
        for n in (13, 4096, 65536 + 13, 200000):
            d = payload(rng, n, kind)
            for ts, bs, split, filt in ((1, None, True, (0,) * 6), (4, 16384, True, (0, 0, 0, 0, 0, B.SHUFFLE)),
                                        (8, 1000, False, (0, 0, 0, 0, 0, B.BITSHUFFLE)), (4, None, False, (0,) * 6)):
                c = B.build(d, ts, bs, codec, filt, split, enc="lib")
                e, out = oracle.blosc2_decompress(c)
                if e or out != d:
                    fails.append((kind, n, ts, bs, split, e))
    assert not fails, fails[:5]


def test_blosc2_zstd_stream_errors():
    """A zstd stream that fails or does not produce its share -> "failed to decompress blosc2 data"."""
    rng = np.random.default_rng(9)
    d = payload(rng, 50000, "ints")
    c = bytearray(B.build(d, 4, 16384, B.ZSTD, memcpyed=False))
    assert oracle.blosc2_decompress(bytes(c)) == (0, d)
    # the first stream's frame magic broken (a compressed stream: csize below the 4096-byte plane)
    first = struct.unpack_from("<i", c, 32)[0]
    assert 0 < struct.unpack_from("<i", c, first)[0] < 4096
    c2 = bytearray(c)
    c2[first + 4] ^= 0xFF
    assert oracle.blosc2_decompress(bytes(c2))[0] == _abi.BLOSC2_FAILED
