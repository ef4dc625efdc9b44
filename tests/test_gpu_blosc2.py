"""MI355X parity of the device blosc2 decoder (k_blosc2.hip: src/compression.rs:29-57) against the oracle
(oracle/oracle_blosc2.cpp, tests/test_blosc2_cpu.py) and the original bytes, through the C ABI:
rdx_decompress_batch_device (batches and lone chunks) and rdx_execute / rdx_execute_device with a blosc2
request (decompress -> filters -> operation, app.rs:163-183).  Chunks come from this repo's writer
(datagen/blosc2_chunk.py): parity unpinned beyond the reference's two tests."""
import itertools
import struct

import numpy as np
import pytest

from datagen import blosc2_chunk as B
from oracle import py_oracle as oracle
from reductionist_amd import _abi

from helpers import make_request, product_convert
from test_blosc2_cpu import payload

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def device_blosc2(torch, ws, chunks, cap, skew=0):
    """Pack the chunks into one device buffer (16-byte boundary + skew), decode them in one call."""
    offs, total = [], 0
    for s in chunks:
        total = (total + 15) // 16 * 16 + skew
        offs.append(total)
        total += len(s)
    host = np.zeros(max(16, total), dtype=np.uint8)
    for o, s in zip(offs, chunks):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    d_in = torch.from_numpy(host).cuda()
    n = len(chunks)
    d_out = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_err = torch.full((n,), 0xEEEE, dtype=torch.int32, device="cuda")
    ws.decompress_batch_device("blosc2", [d_in.data_ptr() + o for o in offs], [len(s) for s in chunks],
                               d_out.data_ptr(), cap, d_len.data_ptr(), d_err.data_ptr(), None)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    lens = d_len.cpu().tolist()
    errs = d_err.cpu().tolist()
    return [(errs[i], out[i * cap:i * cap + min(lens[i], cap)].tobytes() if errs[i] == 0 else b"")
            for i in range(n)]


def expected(c, cap):
    e, d = oracle.blosc2_decompress(c, cap=cap)
    return e, d if e == 0 else b""


@pytest.mark.parametrize("kind", ["smooth", "ints", "random", "const"])
@pytest.mark.parametrize("skew", [0, 3])
def test_batch_every_layout_matches_oracle(torch, workspace, kind, skew):
    rng = np.random.default_rng(len(kind) * 7 + skew)
    chunks, datas = [], []
    for n in (1, 13, 4096, 65536 + 13, 200000):
        d = payload(rng, n, kind)
        for codec, ts, bs, split, filt, ver in itertools.product(
                [B.BLOSCLZ, B.LZ4, B.SNAPPY, B.ZLIB, B.ZSTD], [1, 4, 8], [None, 1000, 16384], [True, False],
                [(0,) * 6, (0, 0, 0, 0, 0, B.SHUFFLE), (0, 0, 0, 0, 0, B.BITSHUFFLE),
                 (0, 0, 0, 0, B.SHUFFLE, B.BITSHUFFLE)], [5, 2]):
            if ver == 2 and filt.count(0) < 5:
                continue
            chunks.append(B.build(d, ts, bs, codec, filt, split, ver))
            datas.append(d)
    cap = 200000 + 16 - 200000 % 16
    got = device_blosc2(torch, workspace, chunks, cap, skew)
    bad = []
    for i, (c, d) in enumerate(zip(chunks, datas)):
        e, out = expected(c, cap)
        if e == 0:
            assert out == d
        if got[i] != (e, out):
            bad.append((i, c[:4].hex(), len(d), got[i][0], e))
    assert not bad, bad[:8]


def test_lone_4mib_chunks_match(torch, workspace):
    """One chunk per call (a lone request): a C4-sized 4 MiB f32 chunk, blocks spread over the waves."""
    rng = np.random.default_rng(44)
    d = (np.round(np.cumsum(rng.standard_normal(1 << 20)) * 8) / 8).astype(np.float32).tobytes()
    for codec, bs, filt in ((B.BLOSCLZ, 1 << 16, (0, 0, 0, 0, 0, B.SHUFFLE)),
                            (B.LZ4, 1 << 18, (0, 0, 0, 0, 0, B.SHUFFLE)),
                            (B.LZ4, 1 << 17, (0, 0, 0, 0, 0, B.BITSHUFFLE)),
                            (B.BLOSCLZ, 1 << 15, (0,) * 6),
                            (B.SNAPPY, 1 << 16, (0, 0, 0, 0, 0, B.SHUFFLE)),
                            (B.ZSTD, 1 << 16, (0, 0, 0, 0, 0, B.SHUFFLE)),
                            (B.ZSTD, 1 << 18, (0,) * 6)):
        c = B.build(d, 4, bs, codec, filt, memcpyed=False)
        [(e, out)] = device_blosc2(torch, workspace, [c], len(d))
        assert e == 0 and out == d, (codec, bs, filt, e)


def test_far_matches_and_long_runs(torch, workspace):
    """Matches farther back than the 8 KiB LDS ring (read from the flushed output), BloscLZ far
    distances (> 8191), long literal runs and long matches."""
    rng = np.random.default_rng(5)
    motif = rng.integers(0, 256, 20000, dtype=np.uint8).tobytes()
    noise = rng.integers(0, 256, 30000, dtype=np.uint8).tobytes()
    d = motif + noise + motif + bytes(40000) + motif[:9000] + noise[:5000] + motif
    for codec in (B.BLOSCLZ, B.LZ4, B.SNAPPY):
        c = B.build(d, 1, len(d), codec, (0,) * 6, memcpyed=False)
        e, ref = oracle.blosc2_decompress(c)
        assert e == 0 and ref == d
        [(ge, out)] = device_blosc2(torch, workspace, [c], len(d) + 16 - len(d) % 16)
        assert ge == 0 and out == d, codec


def test_errors_and_overflow_match_oracle(torch, workspace):
    rng = np.random.default_rng(6)
    d = payload(rng, 70000, "smooth")
    good = B.build(d, 4, 16384, B.BLOSCLZ, memcpyed=False)
    cases = [good, b"invalid format", good[:-1], B.special(4096, 4, 2), B.special(4096, 4, 3, b"\1\2\3\4"),
             B.special(4096, 8, 1)]
    for pos, val in ((0, 6), (21, B.DELTA), (2, (good[2] & 0x1F) | (B.ZSTD << 5)), (31, 0x08), (31, 0x01)):
        b = bytearray(good)
        b[pos] = val
        cases.append(bytes(b))
    b = bytearray(good)
    struct.pack_into("<i", b, 32, 3)
    cases.append(bytes(b))
    for k in range(20):   # corrupted stream bytes: same error (or same output) as the oracle
        b = bytearray(good)
        b[int(rng.integers(32 + 4 * 5, len(b)))] ^= int(rng.integers(1, 256))
        cases.append(bytes(b))
    cap = 70000 + 16 - 70000 % 16
    got = device_blosc2(torch, workspace, cases, cap)
    for i, c in enumerate(cases):
        assert got[i] == expected(c, cap), i
    # the capacity is short of nbytes: overflow reported, with the size the header states
    assert device_blosc2(torch, workspace, [good], 4096)[0][0] == _abi.INFLATE_OUTPUT_OVERFLOW
    # Snappy streams: the hand-built element forms and malformed streams of test_blosc2_cpu, and random
    # corruption of an encoder-written chunk, give the oracle's result
    from test_blosc2_cpu import SNAPPY_BAD, snappy_chunk
    kat = bytes([20, 0x0C]) + b"abcd"
    sc = [snappy_chunk(kat + t, 20) for t in (bytes([0x11, 4, 0x11, 4]), bytes([0x3E, 4, 0]), bytes([0x3F, 4, 0, 0, 0]))]
    sc += [snappy_chunk(st, 20) for st in SNAPPY_BAD]
    sc.append(snappy_chunk(bytes([150, 1, 60 << 2, 99]) + bytes(range(100)) + bytes([0xC6, 100, 0]), 150))
    sgood = B.build(d, 4, 16384, B.SNAPPY, memcpyed=False)
    sc.append(sgood)
    for k in range(20):
        b = bytearray(sgood)
        b[int(rng.integers(32 + 4 * 5, len(b)))] ^= int(rng.integers(1, 256))
        sc.append(bytes(b))
    got = device_blosc2(torch, workspace, sc, cap)
    for i, c in enumerate(sc):
        assert got[i] == expected(c, cap), i


def test_execute_blosc2_requests_match_oracle(engine):
    """rdx_execute with blosc2 requests: decompress on the device, then the reference's shuffle filter,
    byte order, selection, missing and every op, against the oracle (app.rs:163-183)."""
    rng = np.random.default_rng(12)
    checked = 0
    for t in range(40):
        dtype = ["int32", "int64", "uint32", "uint64", "float32", "float64"][t % 6]
        op = ["count", "max", "min", "select", "sum"][t % 5]
        shape = [int(rng.integers(1, 9)), int(rng.integers(1, 17)), int(rng.integers(1, 65))]
        n = int(np.prod(shape))
        npdt = np.dtype(dtype)
        vals = rng.integers(-50 if npdt.kind != "u" else 0, 50, n).astype(npdt)
        req = {"dtype": dtype, "shape": shape, "compression": "blosc2"}
        raw = vals.tobytes()
        if t % 3 == 0:
            raw = vals.astype(npdt.newbyteorder(">")).tobytes()
            req["byte_order"] = "big"
        if t % 4 == 1:
            raw = oracle.shuffle(raw, npdt.itemsize)
            req["filters"] = [{"id": "shuffle", "element_size": npdt.itemsize}]
        if t % 4 == 2:
            req["selection"] = [[0, shape[0], 1], [shape[1] - 1, -shape[1] - 1, -1], [0, shape[2], 2]]
        if t % 5 == 3:
            req["missing"] = {"missing_value": 7}
        codec = [B.BLOSCLZ, B.LZ4][t % 2]
        filt = [(0, 0, 0, 0, 0, B.SHUFFLE), (0, 0, 0, 0, 0, B.BITSHUFFLE), (0,) * 6][t % 3]
        c = B.build(raw, npdt.itemsize, int(rng.integers(64, 4096)) * npdt.itemsize, codec, filt)
        creq = make_request(op, req, product_convert)
        ocreq = make_request(op, req, oracle.convert)
        ost, oinfo, obody, ocounts = oracle.execute(ocreq, c)
        pst, pinfo, pbody, pcounts = engine.execute_raw(creq, c)
        assert pst == ost, (t, req, pst, ost)
        if ost == 0:
            assert pbody == obody and pcounts == ocounts and pinfo.shape_list() == oinfo.shape_list(), (t, req)
            checked += 1
    assert checked >= 30
    # errors: the reference's invalid-header message; unsupported codecs
    lib = _abi.lib()
    creq = make_request("sum", {"dtype": "int32", "compression": "blosc2"}, product_convert)
    assert engine.execute_raw(creq, b"invalid format")[0] == _abi.E_DECOMPRESSION
    assert lib.rdx_inflate_last_error() == _abi.BLOSC2_INVALID
    z = bytearray(B.build(np.arange(5000, dtype=np.int32).tobytes(), 4, 4096, B.BLOSCLZ, memcpyed=False))
    z[2] = (z[2] & 0x1F) | (6 << 5)                        # a user-defined codec
    assert engine.execute_raw(creq, bytes(z))[0] == _abi.E_UNSUPPORTED
    # zstd-coded chunks through rdx_execute (decoded by k_blosc2_zstd), every op vs the oracle
    v = np.arange(20000, dtype=np.int32) % 97
    zc = B.build(v.tobytes(), 4, 8192, B.ZSTD, memcpyed=False)
    for op in ("sum", "min", "max", "count"):
        creq = make_request(op, {"dtype": "int32", "compression": "blosc2"}, product_convert)
        ocreq = make_request(op, {"dtype": "int32", "compression": "blosc2"}, oracle.convert)
        ost, oinfo, obody, ocounts = oracle.execute(ocreq, zc)
        pst, pinfo, pbody, pcounts = engine.execute_raw(creq, zc)
        assert ost == 0 and pst == 0 and pbody == obody and pcounts == ocounts, op


def test_execute_device_blosc2(torch, workspace):
    """rdx_execute_device: a device-resident blosc2 chunk (size read back from the header on overflow)."""
    rng = np.random.default_rng(13)
    vals = rng.integers(-8, 9, 1 << 20).astype(np.float32)   # small integers: every partial sum exact
    raw = vals.astype(">f4").tobytes()
    c = B.build(raw, 4, 1 << 16, B.LZ4, memcpyed=False)
    req = {"dtype": "float32", "byte_order": "big", "compression": "blosc2"}
    creq = make_request("sum", req, product_convert)
    ost, oinfo, obody, ocounts = oracle.execute(make_request("sum", req, oracle.convert), c)
    d_c = torch.from_numpy(np.frombuffer(c, np.uint8).copy()).cuda()
    body = torch.zeros(16, dtype=torch.uint8, device="cuda")
    counts = torch.zeros(4, dtype=torch.int64, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    info = workspace.execute_device(creq, d_c.data_ptr(), len(c), body.data_ptr(), counts.data_ptr(),
                                    status.data_ptr(), None)
    torch.cuda.synchronize()
    assert ost == 0 and int(status[0]) == 0
    assert body.cpu().numpy().tobytes()[:info.body_bytes] == obody
    assert counts.cpu().tolist()[:info.n_counts] == ocounts


def test_version2_bitshuffle_leftover_rule(torch, workspace):
    """c-blosc 1.x chunks (header version 2) with a block whose element count is not a multiple of 8: stored
    unshuffled, copied whole (test_blosc2_cpu.v2_bitshuffle_chunks); read as version 3 they take the newer
    rule.  Device == oracle == the original bytes."""
    from test_blosc2_cpu import v2_bitshuffle_chunks
    cases = v2_bitshuffle_chunks()
    chunks = [c for c, _ in cases] + [bytes([3]) + c[1:] for c, _ in cases]
    got = device_blosc2(torch, workspace, chunks, 16384)
    for c, (e, out) in zip(chunks, got):
        assert (e, out) == expected(c, 16384)
    for (c, d), (e, out) in zip(cases, got):
        assert e == 0 and out == d


def test_zstd_streams_match_oracle(torch, workspace):
    """zstd-coded blosc2 streams (frames by the real libzstd at levels -5..19, every block form: raw, RLE,
    Huffman literals with 1 / 4 streams and treeless repeats, predefined / RLE / FSE / repeat sequence
    tables, multi-block frames), the LZ4 / Snappy streams of the real liblz4 / libsnappy, corrupted zstd
    streams (the oracle's result), and a frame with a content checksum (not decoded on the device:
    RDX_BLOSC2_UNSUPPORTED, the host decodes it)."""
    pa = pytest.importorskip("pyarrow")
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(31)
    chunks = []
    for kind in ("smooth", "ints", "random", "const"):
        for n in (13, 4096, 65536 + 13, 300000):
            d = payload(rng, n, kind)
            for ts, bs, split, filt in ((1, None, True, (0,) * 6), (4, 16384, True, (0, 0, 0, 0, 0, B.SHUFFLE)),
                                        (8, 1000, False, (0, 0, 0, 0, 0, B.BITSHUFFLE)), (4, 1 << 18, False, (0,) * 6)):
                for codec in (B.ZSTD, B.LZ4, B.SNAPPY):
                    chunks.append(B.build(d, ts, bs, codec, filt, split, enc="lib"))
    # every zstd level over text-like data (long matches, repeat offsets)
    text = (b"the quick brown fox jumps over the lazy dog %d " * 8000)[:300000]
    for level in (-5, 1, 3, 9, 19):
        st = pa.Codec("zstd", compression_level=level).compress(text, asbytes=True)
        chunks.append(_one_stream_chunk(st, len(text), B.ZSTD))
    good = B.build(payload(rng, 70000, "ints"), 4, 16384, B.ZSTD, memcpyed=False)
    for k in range(30):
        b = bytearray(good)
        b[int(rng.integers(32 + 4 * 5, len(b)))] ^= int(rng.integers(1, 256))
        chunks.append(bytes(b))
    cap = 300000 + 16 - 300000 % 16
    got = device_blosc2(torch, workspace, chunks, cap)
    bad = [i for i, c in enumerate(chunks) if got[i] != expected(c, cap)]
    assert not bad, [(i, got[i][0], expected(chunks[i], cap)[0]) for i in bad[:8]]
    # a content checksum: the oracle decodes it, the device hands the chunk to the host
    d = payload(rng, 5000, "ints")
    f = bytearray(pa.Codec("zstd").compress(d, asbytes=True))
    f[4] |= 0x04
    st = bytes(f) + struct.pack("<I", xxhash.xxh64(d).intdigest() & 0xFFFFFFFF)
    c = _one_stream_chunk(st, len(d), B.ZSTD)
    assert oracle.blosc2_decompress(c) == (0, d)
    assert device_blosc2(torch, workspace, [c], 5008)[0][0] == _abi.BLOSC2_UNSUPPORTED


def _one_stream_chunk(stream: bytes, nbytes: int, codec: int) -> bytes:
    """One block, one stream (typesize 1, no filter) holding `stream`."""
    base = 32 + 4
    body = struct.pack("<i", len(stream)) + stream
    h = struct.pack("<BBBBiii", 5, 1, 0x05 | (codec << 5) | 0x10, 1, nbytes, nbytes, base + len(body))
    h += bytes(6) + bytes([0, 0]) + bytes(6) + bytes([0, 0])
    return h + struct.pack("<i", base) + body
