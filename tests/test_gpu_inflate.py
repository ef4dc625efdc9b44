"""MI355X parity of the device inflate (k_inflate.hip: src/compression.rs:18-82 gzip/zlib) against the
oracle (oracle/oracle_inflate.cpp, pinned in tests/test_inflate_cpu.py) and the original bytes, through
the C ABI: rdx_decompress_batch_device (the batched stage) and rdx_execute / rdx_execute_device with a
compressed request (decompress -> filters -> operation, app.rs:163-183)."""
import ctypes as C
import zlib

import numpy as np
import pytest

from oracle import py_oracle as oracle
from reductionist_amd import _abi

from helpers import make_request, product_convert
from test_inflate_cpu import STRATEGIES, gz, payload, zl

pytestmark = pytest.mark.gpu

GZIP, ZLIB = 1, 2
NAMES = {GZIP: "gzip", ZLIB: "zlib"}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def device_decompress(torch, ws, comp, streams, cap, skew=0):
    """Pack the streams into one device buffer (each at a 16-byte boundary + skew, so unaligned
    starts are exercised), inflate them in one launch, return [(err, bytes)]."""
    offs, total = [], 0
    for s in streams:
        total = (total + 15) // 16 * 16 + skew
        offs.append(total)
        total += len(s)
    host = np.zeros(max(16, total), dtype=np.uint8)
    for o, s in zip(offs, streams):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    d_in = torch.from_numpy(host).cuda()
    n = len(streams)
    d_out = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_err = torch.full((n,), 0xEEEE, dtype=torch.int32, device="cuda")
    ws.decompress_batch_device(NAMES[comp], [d_in.data_ptr() + o for o in offs], [len(s) for s in streams],
                               d_out.data_ptr(), cap, d_len.data_ptr(), d_err.data_ptr(), None)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    lens = d_len.cpu().tolist()
    errs = d_err.cpu().tolist()
    return [(errs[i], out[i * cap:i * cap + min(lens[i], cap)].tobytes()) for i in range(n)]


@pytest.mark.parametrize("comp", [GZIP, ZLIB])
@pytest.mark.parametrize("skew", [0, 3])
def test_batch_matches_original_and_oracle(torch, workspace, comp, skew):
    rng = np.random.default_rng(comp * 10 + skew)
    datas, streams = [], []
    for t in range(48):
        b = payload(rng, t % 4, int(rng.integers(0, 150000)))
        streams.append((gz if comp == GZIP else zl)(b, int(rng.integers(0, 10)), STRATEGIES[t % 5]))
        datas.append(b)
    cap = (max(len(d) for d in datas) + 16 + 15) // 16 * 16
    res = device_decompress(torch, workspace, comp, streams, cap, skew)
    for i, (e, out) in enumerate(res):
        oe, oout = oracle.decompress(comp, streams[i], cap)
        assert e == oe == 0, (i, e, oe)
        assert out == datas[i] == oout, i


@pytest.mark.parametrize("comp", [GZIP, ZLIB])
def test_large_float_chunks(torch, workspace, comp):
    """4 and 16 MiB float chunks, shuffled as netCDF/HDF5 writers do, levels 1 and 6."""
    rng = np.random.default_rng(7)
    datas = []
    for n in (1 << 20, 4 << 20):
        v = (rng.standard_normal(n) * 100).astype(np.float32)
        datas.append(oracle.shuffle(v.tobytes(), 4))
    streams = [(gz if comp == GZIP else zl)(d, lvl) for d, lvl in zip(datas, (1, 6))]
    cap = max(len(d) for d in datas)
    res = device_decompress(torch, workspace, comp, streams, cap)
    for (e, out), d in zip(res, datas):
        assert e == 0 and out == d


@pytest.mark.parametrize("comp", [GZIP, ZLIB])
def test_errors_match_oracle(torch, workspace, comp):
    b = bytes(range(256)) * 700
    f = gz if comp == GZIP else zl
    good = f(b)
    cases = [b"invalid format", b"", b"\x1f", good[:len(good) // 2], good[:-3], good[:-1]]
    flip = bytearray(good)
    flip[-1] ^= 0x40
    cases.append(bytes(flip))
    mid = bytearray(good)
    mid[len(mid) // 2] ^= 0xFF
    cases.append(bytes(mid))
    if comp == ZLIB:
        cases += [bytes([0x88, 0x1C]) + good[2:], bytes([0x78, 0x9D]) + good[2:], bytes([0x78, 0xBB]) + good[2:],
                  bytes([0x78, 0x9C, 0x07]), bytes([0x78, 0x9C, 0x01, 0x05, 0x00, 0x00, 0x00])]
    else:
        cases += [good[:2] + bytes([7]) + good[3:]]
    rng = np.random.default_rng(3)
    for _ in range(40):  # random corruption anywhere
        c = bytearray(good)
        for _ in range(int(rng.integers(1, 4))):
            c[int(rng.integers(0, len(c)))] ^= int(rng.integers(1, 256))
        cases.append(bytes(c))
    cap = len(b) + 64
    res = device_decompress(torch, workspace, comp, cases, (cap + 15) // 16 * 16)
    for i, ((e, out), c) in enumerate(zip(res, cases)):
        oe, oout = oracle.decompress(comp, c, (cap + 15) // 16 * 16)
        assert e == oe, (i, e, oe, c[:16].hex())
        if e == 0:
            assert out == oout


@pytest.mark.parametrize("comp", [GZIP, ZLIB])
def test_overflow_reports_and_never_writes_past_capacity(torch, workspace, comp):
    b = np.arange(100000, dtype=np.uint32).tobytes()
    s = (gz if comp == GZIP else zl)(b)
    res = device_decompress(torch, workspace, comp, [s, s], 4096)
    assert all(e == _abi.INFLATE_OUTPUT_OVERFLOW for e, _ in res)


def test_execute_with_compression_matches_oracle(engine):
    """rdx_execute with gzip/zlib requests: decompress on the device, then filters, byte order,
    selection, missing and every op, against the oracle (app.rs:163-183)."""
    rng = np.random.default_rng(11)
    checked = 0
    for t in range(60):
        dtype = ["int32", "int64", "uint32", "uint64", "float32", "float64"][t % 6]
        op = ["count", "max", "min", "select", "sum"][t % 5]
        shape = [int(rng.integers(1, 9)), int(rng.integers(1, 17)), int(rng.integers(1, 33))]
        n = int(np.prod(shape))
        npdt = np.dtype(dtype)
        if npdt.kind == "f":
            vals = rng.integers(-50, 50, n).astype(npdt)
        else:
            vals = rng.integers(0, 100, n).astype(npdt)
        req = {"dtype": dtype, "shape": shape}
        big = t % 3 == 0
        raw = vals.astype(npdt.newbyteorder(">")).tobytes() if big else vals.tobytes()
        if big:
            req["byte_order"] = "big"
        if t % 2:
            raw = oracle.shuffle(raw, npdt.itemsize)
            req["filters"] = [{"id": "shuffle", "element_size": npdt.itemsize}]
        if t % 4 == 1:
            req["selection"] = [[0, shape[0], 1], [shape[1] - 1, -shape[1] - 1, -1], [0, shape[2], 2]]
        if t % 5 == 2:
            req["missing"] = {"missing_value": 7}
        comp = "gzip" if t % 2 else "zlib"
        req["compression"] = comp
        stream = (gz if comp == "gzip" else zl)(raw, int(rng.integers(1, 10)))
        creq = make_request(op, req, product_convert)
        ocreq = make_request(op, req, oracle.convert)
        ost, oinfo, obody, ocounts = oracle.execute(ocreq, stream)
        pst, pinfo, pbody, pcounts = engine.execute_raw(creq, stream)
        assert pst == ost, (t, req, pst, ost)
        if ost == 0:
            assert pbody == obody and pcounts == ocounts and pinfo.shape_list() == oinfo.shape_list(), (t, req)
            checked += 1
    assert checked >= 50


def test_execute_compression_errors(engine):
    lib = _abi.lib()
    vals = np.arange(1000, dtype=np.int32)
    # decompression error first, with the reference's detail
    for comp, detail in (("gzip", _abi.INFLATE_GZIP_HEADER), ("zlib", _abi.INFLATE_ZLIB_METHOD)):
        creq = make_request("sum", {"dtype": "int32", "compression": comp}, product_convert)
        st, *_ = engine.execute_raw(creq, b"invalid format")
        assert st == _abi.E_DECOMPRESSION and lib.rdx_inflate_last_error() == detail
        assert _abi.inflate_error_string(detail).startswith(("invalid gzip header", "Unknown zlib compression method"))
    # decoded size vs shape: validate_raw_size after decompression (app.rs:169-172), both directions
    for shape in ([999], [1001]):
        creq = make_request("sum", {"dtype": "int32", "compression": "zlib", "shape": shape, "size": 5},
                            product_convert)
        st, *_ = engine.execute_raw(creq, zl(vals.tobytes()))
        assert st == _abi.E_REQUEST_VALIDATION
    creq = make_request("sum", {"dtype": "int32", "compression": "zlib", "shape": [1000]}, product_convert)
    st, info, body, counts = engine.execute_raw(creq, zl(vals.tobytes()))
    assert st == 0 and int(np.frombuffer(body, np.int32)[0]) == int(vals.sum()) and counts == [1000]
    # a stream much larger than any size hint (grows the device buffer and decodes to its end)
    big = np.zeros(3 << 20, dtype=np.int64)
    creq = make_request("count", {"dtype": "int64", "compression": "gzip"}, product_convert)
    st, info, body, counts = engine.execute_raw(creq, gz(big.tobytes(), 9))
    assert st == 0 and counts == [3 << 20]
    creq = make_request("sum", {"dtype": "int32", "compression": "blosc2"}, product_convert)
    assert engine.execute_raw(creq, b"\0" * 64)[0] == _abi.E_DECOMPRESSION
    assert lib.rdx_inflate_last_error() == _abi.BLOSC2_INVALID


def test_execute_device_with_compression(torch, workspace):
    rng = np.random.default_rng(5)
    vals = rng.standard_normal(1 << 20).astype(np.float32)
    raw = oracle.shuffle(vals.astype(">f4").tobytes(), 4)
    stream = zl(raw, 6)
    req = {"dtype": "float32", "byte_order": "big", "compression": "zlib",
           "filters": [{"id": "shuffle", "element_size": 4}]}
    for op in ("max", "min", "count"):
        creq = make_request(op, req, product_convert)
        d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        body = torch.zeros(16, dtype=torch.uint8, device="cuda")
        counts = torch.zeros(4, dtype=torch.int64, device="cuda")
        status = torch.zeros(4, dtype=torch.int32, device="cuda")
        info = workspace.execute_device(creq, d.data_ptr(), len(stream), body.data_ptr(), counts.data_ptr(),
                                        status.data_ptr(), None)
        torch.cuda.synchronize()
        ost, oinfo, obody, ocounts = oracle.execute(make_request(op, req, oracle.convert), stream)
        assert ost == 0 and int(status[0]) == 0
        assert body.cpu().numpy().tobytes()[:info.body_bytes] == obody
        assert counts.cpu().tolist()[:info.n_counts] == ocounts


def test_python_mirror_with_compression(engine):
    """The Operation mirror (reductionist_amd.operations) on a compressed request, and the error class
    a corrupt stream raises (compression.rs:165-176 -> DecompressionFlate2, HTTP 400)."""
    from reductionist_amd import RequestData, Sum
    from reductionist_amd.errors import Decompression
    vals = np.arange(1, 1001, dtype=np.uint32)
    rd = RequestData(dtype="uint32", compression="gzip", shape=[1000])
    resp = Sum.execute(rd, gz(vals.tobytes()), engine)
    assert int(np.frombuffer(resp.body, np.uint32)[0]) == int(vals.sum()) and resp.count == [1000]
    with pytest.raises(Decompression) as ei:
        Sum.execute(RequestData(dtype="uint32", compression="gzip"), b"invalid format", engine)
    assert str(ei.value) == "invalid gzip header" and ei.value.http_status == 400
