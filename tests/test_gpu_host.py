"""Host-resident entry points beyond rdx_execute's plain path:

* rdx_execute_owned — engine-allocated (pooled, page-locked) response buffers, one call for any request,
  compressed chunks included (no sizing call that inflates twice); random requests vs the oracle.
* the pipelined select / axis=[] path (chunk and response in page-locked memory: the chunk's H2D and the
  response's D2H overlap piece by piece) — C5 at full size and other >= 32 MiB layouts, bit-exact.
"""
import ctypes as C
import zlib

import numpy as np
import pytest

from helpers import encode_filters, make_request, random_case
from oracle import py_oracle as oracle
from reductionist_amd import _abi
from test_gpu_parity import same_result

pytestmark = pytest.mark.gpu


def _check(op, req, got, exp):
    st, info, body, counts = got
    ost, oinfo, obody, ocounts = exp
    assert st == ost, (op, req, st, ost)
    if ost:
        return
    assert info.shape_list() == oinfo.shape_list() and counts == ocounts, (op, req)
    assert same_result(_abi.DTYPE_NAMES[oinfo.dtype], body, obody), (op, req)


@pytest.mark.parametrize("seed", range(2))
def test_owned_random_differential(engine, seed):
    rng = np.random.default_rng(7000 + seed)
    n = 0
    while n < 250:
        op, req, raw = random_case(rng, allow_nan=True, max_dim=12)
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        if rng.random() < 0.25:
            req["compression"] = "gzip" if rng.random() < 0.5 else "zlib"
            c = zlib.compressobj(int(rng.integers(0, 10)), zlib.DEFLATED, 31 if req["compression"] == "gzip" else 15)
            data = c.compress(data) + c.flush()
        try:
            creq = make_request(op, req, oracle.convert)
        except ValueError:
            continue
        _check(op, req, engine.execute_owned(creq, data), oracle.execute(creq, data))
        n += 1


def test_owned_pool_reuse_and_large(engine):
    """Pool blocks are reused across sizes; a 128 MiB select comes back in a pooled block."""
    rng = np.random.default_rng(5)
    for n in (1, 1000, 1 << 20, 123457, 1 << 20):
        v = rng.integers(-1000, 1000, n).astype(np.int64)
        creq = make_request("select", {"dtype": "int64"}, oracle.convert)
        st, info, body, counts = engine.execute_owned(creq, v.tobytes())
        assert st == 0 and counts == [n] and body == v.tobytes()


def _pinned_run(engine, creq, data: np.ndarray):
    """rdx_execute with the chunk and the response in rdx_host_alloc buffers (the pipelined path)."""
    lib = _abi.lib()
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, data.nbytes, C.byref(info)) == 0
    src, arr = engine.host_alloc(data.nbytes)
    arr[:] = data.view(np.uint8).reshape(-1)
    bp, barr = engine.host_alloc(max(16, info.body_bytes))
    cp, carr = engine.host_alloc(max(8, 8 * info.n_counts))
    out = _abi.rdx_response_info()
    st = lib.rdx_execute(engine.ctx, creq.ref, C.c_void_p(src), data.nbytes, C.c_void_p(bp), info.body_bytes,
                         C.cast(C.c_void_p(cp), C.POINTER(C.c_int64)), info.n_counts, C.byref(out))
    body = barr[: info.body_bytes].tobytes()
    counts = [int(x) for x in carr[: 8 * info.n_counts].view(np.int64)]
    for p in (src, bp, cp):
        engine.host_free(p)
    return st, out, body, counts


def test_c5_select_pipelined_full_size(engine):
    """BASELINE configs[4] from page-locked memory: i64 [512,256,256], selection -> 128 MiB, bit-exact."""
    rng = np.random.default_rng(0x5EED0006)
    vals = rng.integers(-2 ** 63, 2 ** 63 - 1, 512 * 256 * 256, dtype=np.int64)
    req = {"dtype": "int64", "shape": [512, 256, 256], "selection": [[0, 512, 1], [64, 192, 1], [0, 256, 1]]}
    creq = make_request("select", req, oracle.convert)
    st, info, body, counts = _pinned_run(engine, creq, vals)
    assert st == 0 and counts == [16777216] and info.shape_list() == [512, 128, 256]
    assert np.array_equal(np.frombuffer(body, dtype=np.int64), vals.reshape(512, 256, 256)[:, 64:192, :].ravel())


@pytest.mark.parametrize("case", range(6))
def test_pipelined_map_layouts(engine, case):
    """>= 32 MiB maps through the pipelined path vs the oracle: reversed outer dim, F-order select,
    missing data (select's non-missing count summed over pieces), axis=[] values + 0/1 counts, Count
    with axis=[], big-endian; outer dims not divisible by the piece count."""
    rng = np.random.default_rng(300 + case)
    dtype, op, shape, sel, extra = [
        ("float64", "select", [67, 256, 256], [[66, None, -1], [3, 250, 2], [0, 256, 1]], {}),
        ("float32", "select", [256, 256, 160], [[0, 256, 1], [0, 256, 1], [10, 150, 1]], {"order": "F"}),
        ("int32", "select", [300, 200, 160], [[5, 299, 1], [0, 200, 3], [0, 160, 1]], {"missing": {"valid_min": -50}}),
        ("float32", "sum", [200, 300, 150], [[0, 200, 1], [10, 290, 1], [0, 150, 1]], {"axis": [],
                                                                                         "missing": {"valid_max": 20.0}}),
        ("int64", "count", [70, 256, 256], None, {"axis": [], "missing": {"missing_values": [1, 2, 3]}}),
        ("uint32", "select", [9, 1024, 1024], [[1, 9, 1], [0, 1024, 1], [0, 1024, 2]], {"byte_order": "big"}),
    ][case]
    n = int(np.prod(shape))
    v = rng.integers(-100, 100, n) if not dtype.startswith("u") else rng.integers(0, 1000, n)
    v = v.astype(dtype)
    req = {"dtype": dtype, "shape": shape, **extra}
    if sel:
        req["selection"] = [[a, b if b is not None else -n - 1, c] for a, b, c in sel]
    raw = v.astype(v.dtype.newbyteorder(">")) if req.get("byte_order") == "big" else v
    assert raw.nbytes >= 32 << 20
    creq = make_request(op, req, oracle.convert)
    got = _pinned_run(engine, creq, raw)
    _check(op, req, got, oracle.execute(creq, raw.tobytes()))


def test_host_read_pinned_chunks(engine):
    """Small page-locked chunks on an idle entry are read by the all-axes kernel itself over PCIe (no H2D
    copy; rdx_device_stats.host_read_requests counts them).  Every dtype / op / byte order / shuffle, chunk
    sizes from a few elements to the 4 MiB bound (and past it: the DMA path), starting at offsets inside the
    pinned block; the block is rewritten between requests and every result must follow (no stale line of a
    previous request survives in a device cache) — bit-exact against the oracle."""
    rng = np.random.default_rng(0x5EED4EAD)
    cap = (4 << 20) + (1 << 16) + 64
    ptr, view = engine.host_alloc(cap)
    try:
        before = engine.stats(0)["host_read_requests"]
        n_cases = 0
        for dtype in ("int32", "int64", "uint32", "uint64", "float32", "float64"):
            es = _abi.DTYPE_SIZE[dtype]
            for nbytes in (8 * es, 4096 + 8 * es, 1 << 20, 4 << 20, (4 << 20) + (1 << 16)):
                for off in (0, 16, 8):
                    op = ("sum", "count", "min", "max")[n_cases % 4]
                    req = {"dtype": dtype}
                    if rng.random() < 0.5:
                        req["byte_order"] = "big"
                    if rng.random() < 0.5:
                        req["filters"] = [{"id": "shuffle", "element_size": es}]
                    creq = make_request(op, req, oracle.convert)
                    for rewrite in range(2):
                        if dtype.startswith("float"):
                            vals = rng.integers(-1000, 1000, nbytes // es).astype(np.float64 if es == 8 else np.float32)
                        else:
                            vals = rng.integers(0, 1000, nbytes // es).astype(np.dtype(dtype))
                        raw = vals.astype(vals.dtype.newbyteorder(">")).tobytes() if req.get("byte_order") else vals.tobytes()
                        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
                        view[off:off + nbytes] = np.frombuffer(data, np.uint8)
                        got = engine.execute_owned(creq, (ptr + off, nbytes))
                        _check(op, req, got, oracle.execute(creq, data))
                    n_cases += 1
        used = engine.stats(0)["host_read_requests"] - before
        assert used > 0, "the host-read path never ran"
    finally:
        engine.host_free(ptr)


def test_host_read_concurrent_callers(engine):
    """Many callers with small page-locked chunks at once: besides the idle-entry direct launch, the
    dispatcher groups same-plan host chunks into one launch of a few workgroups that read them all over
    PCIe.  Each caller rewrites its own block every request; every result is exact (integer-valued data)."""
    from concurrent.futures import ThreadPoolExecutor
    n = 1 << 18
    threads, iters = 8, 40
    blocks = [engine.host_alloc(4 * n + 64) for _ in range(threads)]
    before = engine.stats(0)["host_read_requests"]
    creq = {dt: make_request("sum", {"dtype": dt}, oracle.convert) for dt in ("int32", "float32")}

    def worker(t):
        ptr, view = blocks[t]
        rng = np.random.default_rng(0x5EED7000 + t)
        bad = []
        for i in range(iters):
            dt = ("int32", "float32")[(i + t) % 2]
            v = rng.integers(-100, 100, n).astype(np.int32 if dt == "int32" else np.float32)
            view[16:16 + 4 * n] = np.frombuffer(v.tobytes(), np.uint8)
            st, info, body, counts = engine.execute_owned(creq[dt], (ptr + 16, 4 * n))
            want = int(v.astype(np.int64).sum())
            got = int(np.frombuffer(body, np.int32 if dt == "int32" else np.float32)[0])
            if st != 0 or counts != [n] or got != want:
                bad.append((t, i, dt, st, got, want))
        return bad

    try:
        with ThreadPoolExecutor(threads) as ex:
            bad = [b for r in ex.map(worker, range(threads)) for b in r]
        assert not bad, bad[:5]
        assert engine.stats(0)["host_read_requests"] - before > 0
    finally:
        for ptr, _ in blocks:
            engine.host_free(ptr)
