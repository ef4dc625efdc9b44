"""Response serialisation on the device (rdx_cbor_encode_device): the CBOR body of
serde_cbor::to_vec(&CBORResponse::new(&response)) (app.rs:33-40, models.rs:355-416) packed from
device-resident outputs, byte-identical to the oracle (oracle/cbor_oracle.py, pinned by RFC 7049 and the
reference's response tests in test_cbor_cpu.py) — every flag combination, count arrays across tile
boundaries (2048 counts per tile) and every CBOR integer length, unaligned count buffers, end to end after
device-resident requests, and at full size (axis = [] over the C5 chunk: 32 Mi counts) against the host
encoder."""
import ctypes as C

import numpy as np
import pytest

from helpers import make_request
from oracle import cbor_oracle as cb
from oracle import py_oracle as oracle
from reductionist_amd import _abi
from test_cbor_cpu import _info, host_encode, random_counts

pytestmark = pytest.mark.gpu


def device_encode(workspace, info, d_body, d_counts, flags, torch):
    lib = _abi.lib()
    bound = lib.rdx_cbor_bound(C.byref(info), flags)
    out = torch.full((bound + 64,), 0xA5, dtype=torch.uint8, device="cuda")   # canary past the bound
    meta = torch.zeros(2, dtype=torch.int64, device="cuda")
    status = torch.full((1,), 77, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    st = lib.rdx_cbor_encode_device(workspace.ws, C.byref(info), C.c_void_p(d_body), C.c_void_p(d_counts), flags,
                                    C.c_void_p(out.data_ptr()), bound, C.c_void_p(meta.data_ptr()),
                                    C.c_void_p(status.data_ptr()), C.c_void_p(stream.cuda_stream))
    assert st == 0, _abi.status_string(st)
    torch.cuda.synchronize()
    n = int(meta[0])
    assert int(status[0]) == 0
    assert n <= bound
    host = out.cpu().numpy()
    assert (host[bound:] == 0xA5).all(), "write past the bound"
    return host[:n].tobytes()


@pytest.mark.parametrize("n", [0, 1, 5, 2047, 2048, 2049, 3 * 2048 + 17, 100_003, 1 << 20])
def test_device_encoder_matches_oracle(workspace, n):
    import torch
    rng = np.random.default_rng(0xCB1 + n)
    counts = random_counts(rng, n)
    body = rng.integers(0, 256, 40 + n % 97, dtype=np.uint8).tobytes()
    dc = torch.from_numpy(counts.copy()).cuda() if n else torch.zeros(2, dtype=torch.int64, device="cuda")
    db = torch.from_numpy(np.frombuffer(body, dtype=np.uint8).copy()).cuda()
    for flags in range(4):
        shape = [n, 1] if flags & 1 else [n]
        info = _info("int64", shape, len(body), n)
        got = device_encode(workspace, info, db.data_ptr(), dc.data_ptr(), flags, torch)
        want = cb.cbor_response(body, "int64", shape, counts.tolist(), bool(flags & 1), bool(flags & 2))
        assert got == want, (n, flags)


def test_device_encoder_unaligned_counts_and_shapes(workspace):
    import torch
    rng = np.random.default_rng(0xCB2)
    for it in range(24):
        n = int(rng.integers(1, 9000))
        counts = random_counts(rng, n)
        host = np.zeros(n + 1, dtype=np.int64)
        host[1:] = counts
        dc = torch.from_numpy(host).cuda()
        d_counts = dc.data_ptr() + 8            # 8-byte aligned, not 16: scalar loads
        nd = int(rng.integers(0, 5))
        shape = [int(x) for x in rng.integers(0, 2 ** 34, nd)]
        dtype = list(_abi.DTYPES)[it % 6]
        body = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        db = torch.from_numpy(np.frombuffer(body, dtype=np.uint8).copy()).cuda() if body else dc
        flags = int(rng.integers(0, 4))
        info = _info(dtype, shape, len(body), n)
        got = device_encode(workspace, info, db.data_ptr(), d_counts, flags, torch)
        assert got == cb.cbor_response(body, dtype, shape, counts.tolist(), bool(flags & 1), bool(flags & 2))


def test_device_encoder_after_device_requests(workspace):
    """operation<T> on the device, then the response packed on the device: equal to the oracle's
    serialisation of that response (whose fields equal the oracle's own response)."""
    import torch
    rng = np.random.default_rng(0xCB3)
    lib = _abi.lib()
    cases = [
        ("count", {"dtype": "int32", "shape": [16, 64, 32], "axis": [], "missing": {"missing_value": 3}},
         rng.integers(0, 8, 16 * 64 * 32, dtype=np.int32)),
        ("sum", {"dtype": "float64", "shape": [64, 300], "axis": [1], "missing": {"valid_max": 0.5}},
         rng.random(64 * 300)),
        ("max", {"dtype": "int64", "shape": [40, 50, 60], "axis": [0, 2]},
         rng.integers(-1000, 1000, 40 * 50 * 60, dtype=np.int64)),
        ("select", {"dtype": "uint32", "shape": [33, 70], "selection": [[1, 30, 2], [3, 70, 1]]},
         rng.integers(0, 2 ** 32 - 1, 33 * 70, dtype=np.uint32)),
        ("min", {"dtype": "float32"}, rng.random(10_000, dtype=np.float32)),
    ]
    stream = torch.cuda.current_stream()
    for op, req, arr in cases:
        data = arr.tobytes()
        creq = make_request(op, req, oracle.convert)
        ost, oinfo, obody, ocounts = oracle.execute(creq, data)
        assert ost == 0
        pinfo = _abi.rdx_response_info()
        assert lib.rdx_plan(creq.ref, len(data), C.byref(pinfo)) == 0
        d = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
        body = torch.zeros(max(16, pinfo.body_bytes), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(max(2, pinfo.n_counts), dtype=torch.int64, device="cuda")
        info = workspace.execute_device(creq, d.data_ptr(), len(data), body.data_ptr(), counts.data_ptr(), None,
                                        stream.cuda_stream)
        torch.cuda.synchronize()
        ebody = body.cpu().numpy().tobytes()[: info.body_bytes]
        ecounts = [int(c) for c in counts.cpu()[: info.n_counts]]
        # the response itself is the parity suite's business (float sums within the stated bound); here:
        # the same response fields as the oracle's, and bit-exact bodies where the op is exact
        assert (info.shape_list(), info.dtype, ecounts) == (oinfo.shape_list(), oinfo.dtype, ocounts)
        if not (op == "sum" and req["dtype"].startswith("float")):
            assert ebody == obody
        for flags in range(4):
            got = device_encode(workspace, info, body.data_ptr(), counts.data_ptr(), flags, torch)
            want = cb.cbor_response(ebody, _abi.DTYPE_NAMES[info.dtype], info.shape_list(), ecounts,
                                    bool(flags & 1), bool(flags & 2))
            assert got == want, (op, req, flags)


def test_device_encoder_full_size_axis_none(workspace):
    """axis = [] count over the C5 chunk shape (i64 [512,256,256], missing_value): 32 Mi per-element
    counts (0 / 1) packed on the device; equal to the host encoder (itself equal to the oracle)."""
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(0xCB4)
    n = 512 * 256 * 256
    d = torch.randint(0, 4, (n,), dtype=torch.int64, device="cuda", generator=g)
    creq = make_request("count", {"dtype": "int64", "shape": [512, 256, 256], "axis": [],
                                  "missing": {"missing_value": 1}}, oracle.convert)
    lib = _abi.lib()
    pinfo = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, n * 8, C.byref(pinfo)) == 0
    body = torch.zeros(pinfo.body_bytes, dtype=torch.uint8, device="cuda")
    counts = torch.zeros(pinfo.n_counts, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    info = workspace.execute_device(creq, d.data_ptr(), n * 8, body.data_ptr(), counts.data_ptr(), None,
                                    stream.cuda_stream)
    hc = counts.cpu().numpy()
    assert int(hc.sum()) == int((d != 1).sum())
    hb = body.cpu().numpy().tobytes()
    for flags in (0, 2):
        got = device_encode(workspace, info, body.data_ptr(), counts.data_ptr(), flags, torch)
        assert got == host_encode(info, hb, hc, flags), flags


def test_execute_cbor_end_to_end(engine):
    """rdx_execute_cbor: host chunk in, the reference's HTTP body out (app.rs:163-183 then app.rs:33-40),
    equal to the oracle's response serialised by the oracle — exact ops bit-exact, float sums through the
    engine's own response (rdx_execute_owned) — incl. a response past the one-trip bound (two D2H trips),
    a gzip chunk and an error."""
    import gzip
    rng = np.random.default_rng(0xCB5)
    cases = [
        ("count", {"dtype": "int32", "shape": [64, 128, 64], "axis": [], "missing": {"missing_value": 3}},
         rng.integers(0, 8, 64 * 128 * 64, dtype=np.int32).tobytes()),          # 512 Ki counts: 2 trips
        ("max", {"dtype": "uint64", "shape": [30, 40], "axis": [1]},
         rng.integers(0, 2 ** 63, 1200, dtype=np.uint64).tobytes()),
        ("select", {"dtype": "float32", "shape": [50, 60], "selection": [[2, 50, 3], [0, 60, 1]]},
         rng.random(3000, dtype=np.float32).tobytes()),
        ("sum", {"dtype": "int64", "compression": "gzip"},
         gzip.compress(rng.integers(-10 ** 6, 10 ** 6, 100_000, dtype=np.int64).tobytes(), compresslevel=1)),
        ("min", {"dtype": "float64", "shape": [100, 100], "axis": [0, 1], "missing": {"valid_range": [0.1, 0.9]}},
         rng.random(10_000).tobytes()),
        ("sum", {"dtype": "float32", "shape": [200, 300], "axis": [0]}, rng.random(60_000, dtype=np.float32).tobytes()),
    ]
    for op, req, data in cases:
        creq = make_request(op, req, oracle.convert)
        for flags in range(4):
            st, info, got = engine.execute_cbor(creq, data, flags)
            ost, oinfo, obody, ocounts = oracle.execute(creq, data)
            assert st == ost == 0, (op, req, st, ost)
            if op == "sum" and req["dtype"].startswith("float"):
                est, einfo, ebody, ecounts = engine.execute_owned(creq, data)
                assert est == 0 and ecounts == ocounts
                obody = ebody
            want = cb.cbor_response(obody, _abi.DTYPE_NAMES[oinfo.dtype], oinfo.shape_list(), ocounts,
                                    bool(flags & 1), bool(flags & 2))
            assert got == want, (op, req, flags)
    bad = make_request("sum", {"dtype": "float32", "shape": [7, 7]}, oracle.convert)
    st, _, _ = engine.execute_cbor(bad, bytes(4 * 48), 0)
    assert st == oracle.execute(bad, bytes(4 * 48))[0] != 0


_UNSTAGED = r'''
import sys
sys.path[:0] = [sys.argv[1], sys.argv[2], sys.argv[3]]
import numpy as np, torch
from oracle import cbor_oracle as cb
from reductionist_amd import Engine
from test_cbor_cpu import _info, random_counts
from test_gpu_cbor import device_encode
eng = Engine([0]); ws = eng.workspace(0)
for n in (1, 2049, 3 * 2048 + 17, 100_003):
    rng = np.random.default_rng(0xCB9 + n)
    counts = random_counts(rng, n)
    body = rng.integers(0, 256, 40 + n % 97, dtype=np.uint8).tobytes()
    dc = torch.from_numpy(counts.copy()).cuda()
    db = torch.from_numpy(np.frombuffer(body, dtype=np.uint8).copy()).cuda()
    for flags in range(4):
        shape = [n, 1] if flags & 1 else [n]
        got = device_encode(ws, _info("int64", shape, len(body), n), db.data_ptr(), dc.data_ptr(), flags, torch)
        assert got == cb.cbor_response(body, "int64", shape, counts.tolist(), bool(flags & 1), bool(flags & 2)), (n, flags)
ws.close(); eng.close()
print("UNSTAGED-OK")
'''


def test_unstaged_form_matches_oracle(workspace):
    """The round-4 form (k_cbor_agg / k_cbor_scan / k_cbor), which the runtime keeps for count arrays the staged
    form cannot take (2^32 counts or more, staging memory unavailable): forced with RDX_CBOR_STAGED=0 in a
    child process (the tuning is read once per process), byte-identical to the oracle."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, RDX_CBOR_STAGED="0")
    r = subprocess.run([sys.executable, "-c", _UNSTAGED, str(root / "reductionist-rs_amd"), str(root),
                        str(root / "tests")], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "UNSTAGED-OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
