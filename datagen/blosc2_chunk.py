"""This repo's own blosc2 chunk WRITER — synthetic inputs for tests and bench (neither product nor oracle).

The reference only decompresses blosc2 (src/compression.rs:29-57, via the un-vendored blusc 0.0.2, a
pure-Rust port of c-blosc2); its one test compresses b"hello world" with blusc itself
(compression.rs:90-110).  With no blosc2 library in this image, chunks are assembled here from the
published c-blosc2 chunk format (README_CHUNK_FORMAT): header (16 bytes, or 32 with the extended
blosc2 fields when flags carry both shuffle bits), bstarts, per block `typesize` split streams (or one),
each a signed 32-bit csize followed by a BloscLZ / LZ4 / Snappy / zlib / zstd stream, a raw copy (csize == stream
size), a zero run (csize 0) or a byte run (csize = -byte, token byte 1); memcpy'ed and special-value
chunks.  Filters run forward per block (filters[0] first): byte shuffle, bitshuffle.  The LZ encoders
are datagen/blosc2_writer.cpp's (greedy, this repo's own); with enc="lib" the LZ4 / Snappy streams, and
always the zstd streams, come from the real liblz4 / libsnappy / libzstd bundled with pyarrow, so the
stream decoders are checked against the real encoders.  The chunk container itself is checked against the
format description only, not against c-blosc2's bytes ("parity unpinned").
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

import ctypes as C
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libblosc2w.so"
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
        L = C.CDLL(str(LIB_PATH))
        L.blosc2w_lz_compress.restype = C.c_int64
        L.blosc2w_lz_compress.argtypes = [C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                                C.c_uint64]
        _LIB = L
    return _LIB


def lz(codec: int, data: bytes, max_dist: int = 8191 + 65535) -> bytes:
    """One BloscLZ (codec 0) / LZ4 (codec 1) / Snappy (codec 2) stream by this repo's greedy encoder."""
    cap = 2 * len(data) + 64
    out = (C.c_uint8 * cap)()
    src = C.create_string_buffer(bytes(data), max(1, len(data)))
    n = lib().blosc2w_lz_compress(codec, src, len(data), max_dist, out, cap)
    assert n >= 0
    return bytes(out)[:n]

BLOSCLZ, LZ4, SNAPPY, ZLIB, ZSTD = 0, 1, 2, 3, 4
NOFILTER, SHUFFLE, BITSHUFFLE, DELTA, TRUNC = 0, 1, 2, 3, 4


def shuffle_block(b: bytes, ts: int) -> bytes:
    ne = len(b) // ts
    if ts <= 1 or ne == 0:
        return b
    a = np.frombuffer(b[: ne * ts], np.uint8).reshape(ne, ts)
    return a.T.tobytes() + b[ne * ts:]


def bitshuffle_block(b: bytes, ts: int, version: int = 5) -> bytes:
    size = len(b) // ts
    if version == 2 and size % 8:
        return b     # c-blosc 1.x (header version 2) stores such a block unshuffled
    size -= size % 8
    if size == 0:
        return b
    a = np.frombuffer(b[: size * ts], np.uint8).reshape(size, ts)
    bits = np.unpackbits(a[:, :, None], axis=2, bitorder="little")      # [elem][byte][bit]
    rows = np.packbits(bits.transpose(1, 2, 0), axis=2, bitorder="little")  # [byte][bit][elem / 8]
    return rows.tobytes() + b[size * ts:]


def lib_stream(codec: int, data: bytes, level: int = 3) -> bytes:
    """One stream by the REAL codec library (pyarrow's bundled liblz4 / libsnappy / libzstd): LZ4 raw block
    (c-blosc2 lz4_wrap_compress: LZ4_compress_fast), Snappy raw (c-blosc's snappy_compress), a zstd frame
    (c-blosc2 zstd_wrap_compress: ZSTD_compressCCtx).  These pin the stream decoders against the real
    encoders; the chunk container around them is still this repo's writer."""
    import pyarrow as pa
    name = {LZ4: "lz4_raw", SNAPPY: "snappy", ZSTD: "zstd"}[codec]
    if codec == ZSTD:
        return pa.Codec(name, compression_level=level).compress(bytes(data), asbytes=True)
    return pa.Codec(name).compress(bytes(data), asbytes=True)


def _stream(codec: int, s: bytes, mode: str, enc: str = "repo") -> bytes:
    n = len(s)
    if mode == "auto" and n and s.count(s[0]) == n:
        return struct.pack("<i", 0) if s[0] == 0 else struct.pack("<iB", -s[0], 1)
    if mode == "raw":
        return struct.pack("<i", n) + s
    if codec == ZSTD or (enc == "lib" and codec in (LZ4, SNAPPY)):
        c = lib_stream(codec, s) if n else b""
    elif codec in (BLOSCLZ, LZ4, SNAPPY):
        c = lz(codec, s)
    elif codec == ZLIB:
        c = zlib.compress(s, 6)
    else:
        raise ValueError(codec)
    if len(c) >= n:
        return struct.pack("<i", n) + s
    return struct.pack("<i", len(c)) + c


def build(data: bytes, typesize: int = 4, blocksize: int | None = None, codec: int = BLOSCLZ,
          filters=(0, 0, 0, 0, 0, SHUFFLE), split: bool = True, version: int = 5, memcpyed: bool | None = None,
          stream_mode: str = "auto", b2flags: int = 0, enc: str = "repo") -> bytes:
    """One chunk.  version 5: extended 32-byte header with the filter pipeline; version 2: the 16-byte
    blosc1 header (filters from the flag bits).  memcpyed None: only when compressing does not pay.
    enc "lib": LZ4 / Snappy streams by the real libraries (lib_stream); zstd streams always are."""
    nbytes = len(data)
    if blocksize is None:
        blocksize = min(nbytes, 64 * 1024) or 1
    blocksize = max(1, min(blocksize, max(nbytes, 1)))
    ext = version >= 3
    overhead = 32 if ext else 16
    flags = codec << 5
    fl = list(filters)
    if ext:
        flags |= 0x05
    else:
        if SHUFFLE in fl:
            flags |= 0x01
        if BITSHUFFLE in fl:
            flags |= 0x04
    if not split:
        flags |= 0x10

    def header(fl_, cbytes):
        h = struct.pack("<BBBBiii", version, 1, fl_, typesize, nbytes, blocksize, cbytes)
        if ext:
            h += bytes(fl[:6]) + bytes([0, 0]) + bytes(6) + bytes([0, b2flags])
        return h

    nblocks = (nbytes + blocksize - 1) // blocksize
    leftover = nbytes % blocksize
    body = bytearray()
    bstarts = []
    base = overhead + 4 * nblocks
    for j in range(nblocks):
        left = leftover and j == nblocks - 1
        blk = data[j * blocksize: j * blocksize + (leftover if left else blocksize)]
        for f in fl:
            if f == SHUFFLE:
                blk = shuffle_block(blk, typesize)
            elif f == BITSHUFFLE:
                blk = bitshuffle_block(blk, typesize, version)
        ns = typesize if (split and not left) else 1
        ne = len(blk) // ns
        bstarts.append(base + len(body))
        for k in range(ns):
            body += _stream(codec, blk[k * ne:(k + 1) * ne], stream_mode, enc)
    cbytes = base + len(body)
    if memcpyed is None:
        memcpyed = cbytes >= nbytes + overhead
    if memcpyed:
        return header(flags | 0x02, nbytes + overhead) + data
    return header(flags, cbytes) + struct.pack(f"<{nblocks}i", *bstarts) + bytes(body)


def special(nbytes: int, typesize: int, kind: int, value: bytes = b"") -> bytes:
    """A special-value chunk (blosc2_flags bits 4-6: 1 zeros, 2 NaN, 3 a repeated value, 4 uninit)."""
    cbytes = 32 + (len(value) if kind == 3 else 0)
    h = struct.pack("<BBBBiii", 5, 1, 0x05, typesize, nbytes, max(1, min(nbytes, 1 << 16)), cbytes)
    h += bytes(6) + bytes([0, 0]) + bytes(6) + bytes([0, kind << 4])
    return h + (value if kind == 3 else b"")
