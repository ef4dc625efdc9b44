"""GPU parity at BASELINE.json's own configurations and on real-valued / subnormal data.

* C1 (configs[0]): 4 MiB contiguous f32 sum, seeds 0x5EED0001 (D-int) / 0x5EED0002 (D-real).
* C4 (configs[3]): the FULL batch of 1024 x 4 MiB shuffled f32 chunks, seeds 0x5EED1000+i, summed by one
  rdx_execute_batch_device launch; every chunk checked against the oracle (oracle_execute).
* Real-valued f32 / f64 sums on the strided all-axes and the axis (rows / cols / sliced) kernels.
* Subnormal / ±inf / ±0 mixes for min, max, sum, count, select and the missing predicates (f32, f64).

Bar (SURVEY.md §8d "Parity tolerance"): bit-exact for count, select, min/max and for sums of exactly
summable (D-int) data; real-valued sums per output within
    |gpu - exact| <= max(2 ulp_T(exact), |cpu_seq - exact|)
where `exact` is math.fsum of the included values and `cpu_seq` the oracle's sequential fold in T
(the reference's own arithmetic, operations.rs:622-632).
"""
import math
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from helpers import NP, encode_filters, make_request
from oracle import py_oracle as oracle
from reductionist_amd import _abi

pytestmark = pytest.mark.gpu


def _ulp(x, dtype):
    x = abs(float(x))
    return float(np.spacing(NP[dtype](x))) if math.isfinite(x) else 0.0


def _sum_ok(dtype, gpu, cpu, exact):
    if math.isnan(exact) or math.isinf(exact):
        return (math.isnan(gpu) and math.isnan(exact)) or gpu == exact
    return abs(gpu - exact) <= max(2 * _ulp(exact, dtype), abs(cpu - exact))


# ---- C1 -------------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed,real", [(0x5EED0001, False), (0x5EED0002, True)])
def test_c1_f32_sum_4mib(engine, seed, real):
    """BASELINE configs[0]: the reference's own bench case restated for f32 (benches/operations.rs:35-69):
    1,048,576 f32 values, native order, no filter / selection / missing, op sum."""
    n = 1 << 20
    rng = np.random.default_rng(seed)
    vals = rng.random(n, dtype=np.float32) if real else rng.integers(-8, 9, n).astype(np.float32)
    creq = make_request("sum", {"dtype": "float32"}, oracle.convert)
    st, info, body, counts = engine.execute_raw(creq, vals.tobytes())
    ost, oinfo, obody, ocounts = oracle.execute(creq, vals.tobytes(), body_cap=64, counts_cap=8)
    assert st == ost == 0 and counts == ocounts == [n] and info.shape_list() == oinfo.shape_list() == []
    gpu, cpu = struct.unpack("<f", body)[0], struct.unpack("<f", obody)[0]
    exact = math.fsum(vals.astype(np.float64))
    if not real:
        assert body == obody and gpu == exact
    else:
        assert _sum_ok("float32", gpu, cpu, exact), (gpu, cpu, exact)


# ---- C4 -------------------------------------------------------------------------------------------
C4_CHUNKS, C4_ELEMS = 1024, 1 << 20


def _c4_chunk(i, real):
    rng = np.random.default_rng(0x5EED1000 + i)
    v = rng.random(C4_ELEMS, dtype=np.float32) if real else rng.integers(-8, 9, C4_ELEMS).astype(np.float32)
    return v, v.view(np.uint8).reshape(C4_ELEMS, 4).T.copy().reshape(-1)          # shuffle es=4 (native order)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("real", [False, True], ids=["D-int", "D-real"])
def test_c4_full_batch_1024x4mib(workspace, real):
    """BASELINE configs[3] at full size: 1024 independent 4 MiB shuffled f32 chunks (seeds 0x5EED1000+i),
    sum, ONE rdx_execute_batch_device launch; every chunk vs oracle_execute (D-int bit-exact, D-real
    within the §8d bound); counts and status words too."""
    import torch
    creq = make_request("sum", {"dtype": "float32", "filters": [{"id": "shuffle", "element_size": 4}]},
                        oracle.convert)
    host = np.empty((C4_CHUNKS, 4 * C4_ELEMS), dtype=np.uint8)
    exact = np.empty(C4_CHUNKS)
    cpu = [None] * C4_CHUNKS

    def prep(i):
        v, sh = _c4_chunk(i, real)
        host[i] = sh
        exact[i] = math.fsum(v.astype(np.float64))
        st, _, obody, ocounts = oracle.execute(creq, sh.tobytes(), body_cap=64, counts_cap=8)
        assert st == 0 and ocounts == [C4_ELEMS]
        cpu[i] = obody

    with ThreadPoolExecutor(16) as ex:
        list(ex.map(prep, range(C4_CHUNKS)))
    dev = torch.from_numpy(host).cuda()
    del host
    bodies = torch.full((C4_CHUNKS,), float("nan"), dtype=torch.float32, device="cuda")
    counts = torch.zeros(C4_CHUNKS, dtype=torch.int64, device="cuda")
    status = torch.full((C4_CHUNKS,), 77, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    info = workspace.execute_batch_device(creq, [dev[i].data_ptr() for i in range(C4_CHUNKS)], 4 * C4_ELEMS,
                                          bodies.data_ptr(), counts.data_ptr(), status.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    assert info.body_bytes == 4 and info.n_counts == 1 and info.shape_list() == []
    assert bool((status == 0).all()) and bool((counts == C4_ELEMS).all())
    got = bodies.cpu().numpy()
    bad = []
    for i in range(C4_CHUNKS):
        g = float(got[i])
        c = struct.unpack("<f", cpu[i])[0]
        if not real:
            if got[i:i + 1].tobytes() != cpu[i] or g != exact[i]:
                bad.append((i, g, c, exact[i]))
        elif not _sum_ok("float32", g, c, exact[i]):
            bad.append((i, g, c, exact[i]))
    assert not bad, bad[:5]


# ---- real-valued sums on the strided and axis kernels ----------------------------------------------
def _logical_view(vals, shape, order, selection):
    """The sliced view the reference builds (array.rs:58-63, 121-144): its numpy [start, end, stride]
    selections are numpy slices (models.rs:77-92)."""
    a = vals.reshape(shape, order="F" if order == "F" else "C")
    if selection:
        a = a[tuple(slice(s, e, st) for s, e, st in selection)]
    return a


def _fsum(xs):
    """Exact sum with IEEE specials (math.fsum raises on inf - inf)."""
    xs = np.asarray(xs, dtype=np.float64)
    if np.isnan(xs).any() or (np.isposinf(xs).any() and np.isneginf(xs).any()):
        return float("nan")
    if np.isinf(xs).any():
        return float(xs[np.isinf(xs)][0])
    return math.fsum(xs.tolist())


def _exact_outputs(vals, shape, order, selection, axes, included):
    """fsum of the included values per output (C order over the kept dims)."""
    a = _logical_view(vals, shape, order, selection)
    m = _logical_view(included, shape, order, selection)
    nd = a.ndim
    red = list(range(nd)) if axes is None else ([axes] if isinstance(axes, int) else list(axes))
    kept = [d for d in range(nd) if d not in red]
    a = np.transpose(a, kept + red)
    m = np.transpose(m, kept + red)
    n_out = int(np.prod([a.shape[i] for i in range(len(kept))])) if kept else 1
    a = a.reshape(n_out, -1)
    m = m.reshape(n_out, -1)
    return [_fsum(a[o][m[o]]) for o in range(n_out)]


REAL_CASES = [
    # shape, order, selection, axis
    ([96, 80, 64], "C", [[3, 90, 1], [0, 80, 2], [5, 61, 1]], None),        # strided all-axes (ND 3)
    ([96, 80, 64], "F", [[90, 3, -1], [1, 79, 3], [-1, -60, -2]], None),    # negative strides, F order
    ([96, 80, 64], "C", [[3, 90, 1], [0, 80, 2], [8, 64, 1]], None),        # 16-B vector lanes
    ([1024, 1024], "C", None, 0),                                           # cols, sliced + in-kernel fold
    ([1024, 1024], "C", None, 1),                                           # rows, a wave per output
    ([8, 131072], "C", None, 1),                                            # few long rows: row batch
    ([65536, 16], "C", None, 0),                                            # tall narrow cols, fold launch
    ([4, 60000], "C", None, 1),                                             # rows sliced
    ([64, 96, 48], "C", [[0, 64, 1], [8, 96, 2], [0, 48, 1]], [0, 2]),      # multi-axis over a hyperslab
    ([64, 96, 48], "F", None, [1]),                                         # F order, middle axis
]


@pytest.mark.parametrize("dtype", ["float32", "float64"])
@pytest.mark.parametrize("case", range(len(REAL_CASES)))
def test_real_valued_sums_strided_and_axis(engine, dtype, case):
    shape, order, sel, axis = REAL_CASES[case]
    rng = np.random.default_rng(500 + case + (dtype == "float64") * 100)
    n = int(np.prod(shape))
    vals = (rng.standard_normal(n) * 100 + 3).astype(NP[dtype])
    req = {"dtype": dtype, "shape": shape, "order": order}
    if sel:
        req["selection"] = sel
    if axis is not None:
        req["axis"] = axis
    included = np.ones(n, dtype=bool)
    if case % 3 == 1:
        req["missing"] = {"valid_range": [-150.0, 180.0]}
        included = (vals >= -150.0) & (vals <= 180.0)
    creq = make_request("sum", req, oracle.convert)
    st, info, body, counts = engine.execute_raw(creq, vals.tobytes())
    ost, oinfo, obody, ocounts = oracle.execute(creq, vals.tobytes())
    assert st == ost == 0 and counts == ocounts and info.shape_list() == oinfo.shape_list()
    gpu = np.frombuffer(body, dtype=NP[dtype])
    cpu = np.frombuffer(obody, dtype=NP[dtype])
    exact = _exact_outputs(vals, shape, order, sel, axis, included)
    assert len(exact) == len(gpu) == len(cpu)
    bad = [(o, float(gpu[o]), float(cpu[o]), exact[o]) for o in range(len(exact))
           if not _sum_ok(dtype, float(gpu[o]), float(cpu[o]), exact[o])]
    assert not bad, bad[:5]


# ---- subnormals, infinities, signed zeros ------------------------------------------------------------
def _subnormal_mix(rng, dtype, n):
    info = np.finfo(NP[dtype])
    tiny = info.smallest_subnormal
    v = rng.integers(-40, 41, n).astype(NP[dtype]) * NP[dtype](tiny)      # subnormals (and ±0)
    r = rng.random(n)
    v[r < 0.10] = (rng.integers(1, 1 << 20, int((r < 0.10).sum())) * NP[dtype](tiny)).astype(NP[dtype])
    v[(r >= 0.10) & (r < 0.13)] = -0.0
    v[(r >= 0.13) & (r < 0.16)] = info.tiny                              # smallest normal
    v[(r >= 0.16) & (r < 0.18)] = -info.tiny
    v[(r >= 0.18) & (r < 0.185)] = np.inf
    v[(r >= 0.185) & (r < 0.19)] = -np.inf
    v[(r >= 0.19) & (r < 0.20)] = rng.standard_normal(int(((r >= 0.19) & (r < 0.20)).sum())).astype(NP[dtype])
    return v


SUB_REQS = [
    {},
    {"shape": [64, 128], "axis": 0},
    {"shape": [64, 128], "axis": 1},
    {"shape": [64, 128], "selection": [[1, 63, 2], [0, 128, 1]]},
    {"shape": [64, 128], "axis": []},
    {"byte_order": "big", "filters": [{"id": "shuffle", "element_size": None}]},
]


@pytest.mark.parametrize("dtype", ["float32", "float64"])
@pytest.mark.parametrize("op", ["min", "max", "sum", "count", "select"])
@pytest.mark.parametrize("r", range(len(SUB_REQS)))
def test_subnormal_inf_mix(engine, dtype, op, r):
    """Subnormal inputs are neither flushed on load nor in a compare: the kernels run with f32/f64
    denormals enabled (the code objects' default FP mode on gfx950), so min/max/count/select are
    bit-exact with the oracle, including missing thresholds that are themselves subnormal."""
    rng = np.random.default_rng(9000 + r * 10 + (dtype == "float64"))
    n = 64 * 128
    es = np.dtype(NP[dtype]).itemsize
    tiny = float(np.finfo(NP[dtype]).smallest_subnormal)
    for mk, mv in ((None, None), ("valid_min", 3 * tiny), ("missing_value", 5 * tiny),
                   ("valid_range", [-7 * tiny, 20 * tiny]), ("valid_max", -2 * tiny)):
        vals = _subnormal_mix(rng, dtype, n)
        req = {"dtype": dtype, **{k: v for k, v in SUB_REQS[r].items()}}
        if "filters" in req:
            req["filters"] = [{"id": "shuffle", "element_size": es}]
        if mk:
            req["missing"] = {mk: mv}
        raw = vals.astype(vals.dtype.newbyteorder(">")).tobytes() if req.get("byte_order") == "big" else vals.tobytes()
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        creq = make_request(op, req, oracle.convert)
        st, info, body, counts = engine.execute_raw(creq, data)
        ost, oinfo, obody, ocounts = oracle.execute(creq, data)
        assert st == ost, (op, req, st, ost)
        if ost:
            continue
        assert counts == ocounts and info.shape_list() == oinfo.shape_list(), (op, req)
        if op != "sum":
            assert body == obody, (op, req)
        else:
            g = np.frombuffer(body, dtype=NP[dtype])
            c = np.frombuffer(obody, dtype=NP[dtype])
            inc = np.ones(n, dtype=bool)
            if mk == "valid_min":
                inc = ~(vals < mv)
            elif mk == "missing_value":
                inc = vals != mv
            elif mk == "valid_range":
                inc = ~((vals < mv[0]) | (vals > mv[1]))
            elif mk == "valid_max":
                inc = ~(vals > mv)
            shape = req.get("shape", [n])
            exact = _exact_outputs(vals, shape, None, req.get("selection"), req.get("axis"), inc) \
                if req.get("axis") != [] else None
            if exact is None:
                assert body == obody
                continue
            for o in range(len(exact)):
                assert _sum_ok(dtype, float(g[o]), float(c[o]), exact[o]), (o, g[o], c[o], exact[o], req)


# ---- f64 sums with heavy cancellation (the group sums' compensation) -------------------
@pytest.mark.parametrize("shuffled", [False, True])
@pytest.mark.parametrize("big_endian", [False, True])
def test_f64_sum_cancellation(engine, shuffled, big_endian):
    """f64 sums whose terms cancel.  (1) [1e16, 1, -1e16, 1] repeated: every group of four sums to exactly
    2, which a plain pairwise add inside the group loses entirely (the reference's sequential fold keeps
    one of the two 1s per group): the device's compensated sum (TwoSum inside each group, Neumaier across)
    gives the exact total.  (2) random ±1e15 pairs plus [0, 1) noise: within the bar."""
    n = 1 << 20
    rng = np.random.default_rng(0x5EEDCA11 + 2 * shuffled + big_endian)
    big = rng.standard_normal(n // 2) * 1e15
    noisy = np.stack([big, -big], axis=1).reshape(-1) + rng.random(n)
    for case, v in (("pattern", np.tile(np.array([1e16, 1.0, -1e16, 1.0]), n // 4)), ("noisy", noisy)):
        raw = v.astype(">f8" if big_endian else "<f8").tobytes()
        req = {"dtype": "float64", "byte_order": "big" if big_endian else "little"}
        if shuffled:
            raw = np.frombuffer(raw, np.uint8).reshape(n, 8).T.copy().tobytes()
            req["filters"] = [{"id": "shuffle", "element_size": 8}]
        creq = make_request("sum", req, oracle.convert)
        st, info, body, counts = engine.execute_raw(creq, raw)
        ost, _, obody, ocounts = oracle.execute(creq, raw, body_cap=64, counts_cap=8)
        assert st == ost == 0 and counts == ocounts == [n]
        gpu, cpu = struct.unpack("<d", body)[0], struct.unpack("<d", obody)[0]
        exact = math.fsum(v)
        assert _sum_ok("float64", gpu, cpu, exact), (case, gpu, cpu, exact)
        if case == "pattern":
            assert exact == n // 2 and gpu == exact, (gpu, cpu, exact)
