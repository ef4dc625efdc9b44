"""Heterogeneous request batches (rdx_execute_multi_device): many independent requests — different dtypes,
ops, shapes, selections, byte orders, fused shuffles, missing descriptors, plus requests that are not
all-axes reductions (they run as their own launches) and invalid ones (per-item status) — in one call;
every request's response equal to the oracle's, bit-exact (float sums of the random generator's
exactly-summable values included)."""
import ctypes as C
import struct

import numpy as np
import pytest

from helpers import NP, encode_filters, make_request, random_case
from oracle import py_oracle as oracle
from reductionist_amd import _abi
from test_gpu_parity import same_result

pytestmark = pytest.mark.gpu


def _run(workspace, cases, offsets=None):
    """cases: [(op, request dict, chunk bytes)] -> list of (oracle result, device result)."""
    import torch
    items, keep, expect = [], [], []
    for i, (op, req, data) in enumerate(cases):
        creq = make_request(op, req, oracle.convert)
        ost, oinfo, obody, ocounts = oracle.execute(creq, data)
        pinfo = _abi.rdx_response_info()      # outputs sized by the product planner (a request whose
        pst = _abi.lib().rdx_plan(creq.ref, len(data), C.byref(pinfo))   # kernel raises NaN still writes)
        off = offsets[i] if offsets else 0
        buf = torch.zeros(len(data) + off + 16, dtype=torch.uint8)
        if len(data):
            buf[off:off + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        d = buf.cuda()
        nb = pinfo.body_bytes if pst == 0 else 16
        nc = pinfo.n_counts if pst == 0 else 1
        body = torch.zeros(max(16, nb), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(max(2, nc), dtype=torch.int64, device="cuda")
        status = torch.full((1,), 77, dtype=torch.int32, device="cuda")
        keep.append((creq, d, body, counts, status))
        items.append((creq, d.data_ptr() + off, len(data), body.data_ptr(), counts.data_ptr(), status.data_ptr()))
        expect.append((ost, oinfo, obody, ocounts))
    stream = torch.cuda.current_stream()
    statuses, infos = workspace.execute_multi_device(items, stream.cuda_stream)
    torch.cuda.synchronize()
    out = []
    for i, (creq, d, body, counts, status) in enumerate(keep):
        st = statuses[i] or int(status[0])
        ost, oinfo, obody, ocounts = expect[i]
        res = None
        if st == 0:
            res = (infos[i].shape_list(), _abi.DTYPE_NAMES[infos[i].dtype],
                   body.cpu().numpy().tobytes()[: infos[i].body_bytes],
                   [int(c) for c in counts.cpu()[: infos[i].n_counts]])
        out.append(((ost, oinfo, obody, ocounts), (st, res)))
    return out


def _check(cases, results):
    for (op, req, _), ((ost, oinfo, obody, ocounts), (st, res)) in zip(cases, results):
        assert st == ost, (op, req, st, ost)
        if ost:
            continue
        shape, dtype, body, counts = res
        assert shape == oinfo.shape_list() and counts == ocounts, (op, req)
        assert same_result(dtype, body, obody), (op, req, body.hex(), obody.hex())


@pytest.mark.parametrize("seed", range(3))
def test_random_mixed_batch(workspace, seed):
    rng = np.random.default_rng(4000 + seed)
    cases = []
    while len(cases) < 250:
        op, req, raw = random_case(rng, allow_nan=True, max_dim=24, max_ndim=4)
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        try:
            make_request(op, req, oracle.convert)
        except ValueError:
            continue
        cases.append((op, req, data))
    offsets = [int(rng.choice([0, 0, 8, 16])) for _ in cases]
    _check(cases, _run(workspace, cases, offsets))


def test_mixed_sizes_and_edges(workspace):
    """Multi-workgroup requests of every dtype/op next to empty selections, zero-length chunks, fused
    big-endian shuffles, 16 / 17 missing values (inline vs listed), an invalid shape and an axis request."""
    rng = np.random.default_rng(77)
    cases = []
    for dtype in NP:
        es = np.dtype(NP[dtype]).itemsize
        for op in ("count", "max", "min", "sum"):
            v = (rng.integers(-50, 50, 300000) if not dtype.startswith("u") else rng.integers(0, 100, 300000))
            v = v.astype(NP[dtype])
            if dtype.startswith("float"):
                v[rng.integers(0, v.size, 100)] = 0.0
                v[rng.integers(0, v.size, 100)] = -0.0
            cases.append((op, {"dtype": dtype, "shape": [300, 1000], "selection": [[3, 290, 2], [10, 990, 1]],
                               "missing": {"valid_range": [-40, 40] if not dtype.startswith("u") else [3, 90]}},
                          v.tobytes()))
            cases.append((op, {"dtype": dtype, "byte_order": "big",
                               "filters": [{"id": "shuffle", "element_size": es}]},
                          oracle.shuffle(v.astype(v.dtype.newbyteorder(">")).tobytes(), es)))
            cases.append((op, {"dtype": dtype, "shape": [300, 1000], "selection": [[5, 5, 1], [0, 1000, 1]]},
                          v.tobytes()))
    lst16 = list(range(16))
    lst17 = list(range(17))
    v = rng.integers(0, 40, 5000).astype(np.int64)
    cases += [("sum", {"dtype": "int64", "missing": {"missing_values": lst16}}, v.tobytes()),
              ("sum", {"dtype": "int64", "missing": {"missing_values": lst17}}, v.tobytes()),
              ("count", {"dtype": "int64"}, b""),
              ("sum", {"dtype": "int64", "shape": [7, 7]}, v.tobytes()),                 # a shorter view
              ("sum", {"dtype": "int64", "shape": [100, 100]}, v.tobytes()),             # ShapeInvalid
              ("max", {"dtype": "int64", "shape": [50, 100], "axis": 1}, v.tobytes()),  # own launch
              ("select", {"dtype": "int64", "shape": [50, 100], "selection": [[1, 40, 3], [0, 100, 7]]},
               v.tobytes())]
    _check(cases, _run(workspace, cases))


def test_mixed_c1_c3_20(workspace):
    """The BASELINE shapes as one heterogeneous launch: 10 x C1 (f32 4 MiB sum, D-int) and 10 x C3 (f64
    [128,128,128] hyperslab min / max with missing_value -9999 at 5 %), bit-exact vs the oracle."""
    cases = []
    for i in range(10):
        v1 = np.random.default_rng(0x5EED0001 + 16 * i).integers(-8, 9, 1 << 20).astype(np.float32)
        cases.append(("sum", {"dtype": "float32"}, v1.tobytes()))
        rng = np.random.default_rng(0x5EED0005 + 16 * i)
        v3 = rng.standard_normal(128 ** 3) * 100
        v3[rng.random(v3.size) < 0.05] = -9999.0
        cases.append(("min" if i % 2 == 0 else "max",
                      {"dtype": "float64", "shape": [128, 128, 128], "selection": [[8, 120, 1], [0, 128, 2], [16, 112, 1]],
                       "missing": {"missing_value": -9999.0}}, v3.tobytes()))
    results = _run(workspace, cases)
    _check(cases, results)
    for (op, req, data), (_, (st, res)) in zip(cases, results):
        if req["dtype"] == "float32":
            assert struct.unpack("<f", res[2])[0] == float(np.frombuffer(data, np.float32).astype(np.float64).sum())


def test_no_writes_outside_planned_outputs(workspace):
    """Every device-resident request writes only its planned body / counts (rdx_plan sizes): outputs
    and input sit in a canary-filled arena with 1 MiB of canary on each side."""
    import torch
    rng = np.random.default_rng(4100)
    pad = 1 << 20
    n = 0
    while n < 150:
        op, req, raw = random_case(rng, allow_nan=True, max_dim=24, max_ndim=4)
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        try:
            creq = make_request(op, req, oracle.convert)
        except ValueError:
            continue
        info = _abi.rdx_response_info()
        if _abi.lib().rdx_plan(creq.ref, len(data), C.byref(info)):
            continue
        nb, nc = info.body_bytes, info.n_counts
        d0 = pad
        b0 = (d0 + len(data) + pad + 255) // 256 * 256
        c0 = (b0 + nb + pad + 255) // 256 * 256
        arena = torch.full((c0 + 8 * nc + pad,), 0xAB, dtype=torch.uint8, device="cuda")
        if data:
            arena[d0:d0 + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        before = arena.clone()
        st = torch.zeros(1, dtype=torch.int32, device="cuda")
        workspace.execute_device(creq, arena.data_ptr() + d0, len(data), arena.data_ptr() + b0, arena.data_ptr() + c0,
                                 st.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        diff = (arena != before).nonzero().flatten().cpu().numpy()
        ok = ((diff >= b0) & (diff < b0 + nb)) | ((diff >= c0) & (diff < c0 + 8 * nc))
        assert ok.all(), (op, req, diff[~ok][:8] - c0)
        n += 1
