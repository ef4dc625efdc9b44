"""The context's device pool (include/rdx.h rdx_context): concurrent callers, the way the server issues
requests — every request its own synchronous operation<T>() call on a worker thread (app.rs:147-152,
app_state.rs:21-37).  Through the C ABI from Python threads (ctypes releases the GIL):

* rdx_execute_resident (chunks already in HBM) and rdx_execute (host chunks) from many threads: small
  all-axes requests coalesce into shared k_multi launches; every response bit-exact vs the oracle;
* placement over a pool listing one GPU twice (rdx_context_create([0, 0])): both entries serve, each with
  its own workspaces; least outstanding bytes;
* back-pressure: max_workspaces = 1 with many threads — all requests served by one workspace;
* a NaN min inside a coalesced launch fails only its own request."""
import threading

import numpy as np
import pytest

from helpers import encode_filters, make_request, random_case
from oracle import py_oracle as oracle
from reductionist_amd import Engine, _abi
from test_gpu_parity import same_result

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _cases(seed, n, allaxes_only=False, max_dim=24):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        op, req, raw = random_case(rng, allow_nan=True, max_dim=max_dim, max_ndim=4)
        if allaxes_only:
            req.pop("axis", None)
            req.pop("filters", None)
            if op == "select":
                op = "sum"
        data = encode_filters(raw, req.get("filters"), oracle.shuffle)
        try:
            creq = make_request(op, req, oracle.convert)
        except ValueError:
            continue
        out.append((op, req, data, creq, oracle.execute(creq, data)))
    return out


def _plannable(cases):
    """Requests that reach the pool: the Python wrappers plan first (rdx_plan, host only)."""
    import ctypes as C
    info = _abi.rdx_response_info()
    return sum(_abi.lib().rdx_plan(c[3].ref, len(c[2]), C.byref(info)) == 0 for c in cases)


def _check_one(case, st, info, body, counts):
    op, req, _, _, (ost, oinfo, obody, ocounts) = case
    assert st == ost, (op, req, st, ost)
    if ost:
        return
    assert info.shape_list() == oinfo.shape_list() and counts == ocounts, (op, req)
    assert same_result(_abi.DTYPE_NAMES[info.dtype], body, obody), (op, req, body.hex(), obody.hex())


def _threaded(n_threads, cases, fn):
    """Run fn(case) for every case from n_threads threads (case i on thread i % n_threads, started together);
    returns the results in case order."""
    results = [None] * len(cases)
    errors = []
    go = threading.Barrier(n_threads)

    def worker(t):
        try:
            go.wait()
            for i in range(t, len(cases), n_threads):
                results[i] = fn(cases[i])
        except BaseException as e:   # noqa: BLE001 - re-raised in the main thread
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    if errors:
        raise errors[0]
    return results


def _to_device(torch, cases):
    bufs = []
    for case in cases:
        data = case[2]
        buf = torch.zeros(max(16, len(data)), dtype=torch.uint8)
        if data:
            buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        bufs.append(buf.cuda())
    torch.cuda.synchronize()
    return bufs


@pytest.mark.parametrize("lanes", [1, 2])
def test_resident_threads_coalesce_bit_exact(torch, lanes):
    eng = Engine([0])
    eng.configure(coalesce_lanes=lanes)
    cases = _cases(7100 + lanes, 400)
    bufs = _to_device(torch, cases)
    idx = {id(c): i for i, c in enumerate(cases)}
    res = _threaded(8, cases, lambda c: eng.execute_resident(c[3], 0, bufs[idx[id(c)]].data_ptr(), len(c[2])))
    for case, r in zip(cases, res):
        _check_one(case, *r)
    s = eng.stats(0)
    assert s["requests"] == _plannable(cases) and s["outstanding_bytes"] == 0 and s["workspaces_busy"] == 0
    assert 0 < s["coalesced_requests"] + s["direct_requests"] < s["requests"]   # all-axes ones only
    assert s["coalesced_requests"] > 0                        # 8 callers: the queue is not always idle
    assert 0 < s["coalesced_launches"] <= s["coalesced_requests"]
    eng.close()


def test_resident_large_allaxes_and_c_shapes(torch):
    """Multi-workgroup requests per coalesced launch: C1-shaped f32 sums (D-int) and C3-shaped f64 min / max
    (missing_value -9999) from 6 threads, each bit-exact; and with coalescing off, the same answers."""
    cases = []
    for i in range(12):
        v1 = np.random.default_rng(0x5EED0001 + 16 * i).integers(-8, 9, 1 << 20).astype(np.float32)
        creq = _abi.CRequest("sum", "float32")
        cases.append(("sum", {}, v1.tobytes(), creq, oracle.execute(creq, v1.tobytes())))
        rng = np.random.default_rng(0x5EED0005 + 16 * i)
        v3 = rng.standard_normal(128 ** 3) * 100
        v3[rng.random(v3.size) < 0.05] = -9999.0
        req = {"dtype": "float64", "shape": [128, 128, 128], "selection": [[8, 120, 1], [0, 128, 2], [16, 112, 1]],
               "missing": {"missing_value": -9999.0}}
        op = "min" if i % 2 == 0 else "max"
        creq = make_request(op, req, oracle.convert)
        cases.append((op, req, v3.tobytes(), creq, oracle.execute(creq, v3.tobytes())))
    bufs = _to_device(torch, cases)
    for coalesce in (True, False):
        eng = Engine([0])
        eng.configure(coalesce=coalesce)
        res = _threaded(6, list(range(len(cases))),
                        lambda i: eng.execute_resident(cases[i][3], 0, bufs[i].data_ptr(), len(cases[i][2])))
        for case, r in zip(cases, res):
            _check_one(case, *r)
        s = eng.stats(0)
        assert s["coalesced_requests"] + s["direct_requests"] == (len(cases) if coalesce else 0)
        eng.close()


def test_host_chunks_coalesce(torch):
    """rdx_execute from threads with host chunks below coalesce_host_max_bytes: the chunk crosses PCIe on
    the caller's workspace stream, then joins a coalesced launch."""
    eng = Engine([0])
    cases = _cases(7300, 300)
    res = _threaded(8, cases, lambda c: eng.execute_raw(c[3], c[2]))
    for case, r in zip(cases, res):
        _check_one(case, *r)
    s = eng.stats(0)
    assert s["coalesced_requests"] > 0 and s["workspaces"] <= s["max_workspaces"]
    eng.close()


def test_pool_twice_one_gpu_places_and_isolates(torch):
    """rdx_context_create([0, 0]): two pool entries on one GPU.  Concurrent host requests spread over both
    (least outstanding bytes), each entry keeps its own workspaces, results bit-exact; resident requests
    name device 0 and may go to either entry."""
    eng = Engine([0, 0])
    cases = _cases(7400, 300)
    res = _threaded(8, cases, lambda c: eng.execute_raw(c[3], c[2]))
    for case, r in zip(cases, res):
        _check_one(case, *r)
    s0, s1 = eng.stats(0), eng.stats(1)
    assert s0["device"] == s1["device"] == 0
    assert s0["requests"] + s1["requests"] == _plannable(cases)
    assert s0["requests"] > 0 and s1["requests"] > 0
    assert s0["workspaces"] >= 1 and s1["workspaces"] >= 1
    assert s0["outstanding_bytes"] == s1["outstanding_bytes"] == 0
    bufs = _to_device(torch, cases)
    res = _threaded(8, list(range(len(cases))),
                    lambda i: eng.execute_resident(cases[i][3], 0, bufs[i].data_ptr(), len(cases[i][2])))
    for case, r in zip(cases, res):
        _check_one(case, *r)
    # a resident chunk on a device outside the pool is an invalid argument, not a crash
    ok = _abi.CRequest("sum", "int32")
    st, *_ = eng.execute_resident(ok, 7, bufs[0].data_ptr(), 16)
    assert st == _abi.E_INVALID_ARGUMENT
    with pytest.raises(Exception):
        eng.stats(2)
    eng.close()


def test_back_pressure_one_workspace(torch):
    """max_workspaces = 1, coalescing off, 8 threads: one workspace serves everything, the others wait."""
    eng = Engine([0])
    eng.configure(max_workspaces=1, coalesce=False)
    cases = _cases(7500, 160)
    res = _threaded(8, cases, lambda c: eng.execute_raw(c[3], c[2]))
    for case, r in zip(cases, res):
        _check_one(case, *r)
    s = eng.stats(0)
    assert s["workspaces"] == 1 and s["max_workspaces"] == 1 and s["waits"] > 0 and s["coalesced_requests"] == 0
    assert s["direct_requests"] == 0
    eng.close()


def test_nan_fails_only_its_own_request(torch):
    """min over a chunk holding a NaN panics in the reference (operations.rs:355-357 -> RDX_E_NAN_UNORDERED);
    inside a coalesced launch the neighbours still get their results."""
    eng = Engine([0])
    eng.configure(coalesce_lanes=1)
    good = np.arange(1000, dtype=np.float32)
    bad = good.copy()
    bad[500] = np.nan
    creq = _abi.CRequest("min", "float32")
    chunks = [bad if i % 3 == 0 else good for i in range(48)]
    bufs = [torch.from_numpy(c.view(np.uint8).copy()).cuda() for c in chunks]
    res = _threaded(12, list(range(48)), lambda i: eng.execute_resident(creq, 0, bufs[i].data_ptr(), 4000))
    for i, (st, info, body, counts) in enumerate(res):
        if i % 3 == 0:
            assert st == _abi.E_NAN_UNORDERED
        else:
            assert st == 0 and np.frombuffer(body, np.float32)[0] == 0.0 and counts == [1000]
    eng.close()


def test_resident_same_plan_groups(torch):
    """Concurrent requests with one plan (the same variable's chunks: shuffled big-endian f32 sums, and
    strided f64 hyperslab max with a valid_range) are served by batched launches of that plan, chunk
    pointers in the kernel arguments; D-int values, so every sum is exact.  Bit-exact vs the oracle."""
    rng = np.random.default_rng(7700)
    cases = []
    for i in range(40):
        v = rng.integers(-8, 9, 1 << 18).astype(np.float32)
        req = {"dtype": "float32", "byte_order": "big", "filters": [{"id": "shuffle", "element_size": 4}]}
        data = oracle.shuffle(v.astype(">f4").tobytes(), 4)
        creq = make_request("sum", req, oracle.convert)
        cases.append(("sum", req, data, creq, oracle.execute(creq, data)))
        w = rng.integers(-1000, 1000, 40 * 50 * 30).astype(np.float64)
        req = {"dtype": "float64", "shape": [40, 50, 30], "selection": [[1, 39, 2], [0, 50, 1], [3, 27, 1]],
               "missing": {"valid_range": [-900.0, 900.0]}}
        creq = make_request("max", req, oracle.convert)
        cases.append(("max", req, w.tobytes(), creq, oracle.execute(creq, w.tobytes())))
    bufs = _to_device(torch, cases)
    eng = Engine([0])
    res = _threaded(12, list(range(len(cases))),
                    lambda i: eng.execute_resident(cases[i][3], 0, bufs[i].data_ptr(), len(cases[i][2])))
    for case, r in zip(cases, res):
        _check_one(case, *r)
    s = eng.stats(0)
    assert s["coalesced_requests"] + s["direct_requests"] == len(cases)
    assert s["coalesced_launches"] + s["direct_requests"] < len(cases)
    eng.close()


def _config_cases():
    """Distinct chunks of the BASELINE request shapes with their oracle results: C1 (f32 4 MiB sum, D-int),
    C3 (f64 [128,128,128] hyperslab min / max, missing_value -9999 at 5 %) and C4's chunk (f32 4 MiB
    shuffled sum, D-int)."""
    cases = []
    for i in range(4):
        v1 = np.random.default_rng(0x5EED0001 + 32 * i).integers(-8, 9, 1 << 20).astype(np.float32)
        creq = _abi.CRequest("sum", "float32")
        cases.append(("sum", {}, v1.tobytes(), creq, oracle.execute(creq, v1.tobytes())))
        rng = np.random.default_rng(0x5EED0005 + 32 * i)
        v3 = rng.standard_normal(128 ** 3) * 100
        v3[rng.random(v3.size) < 0.05] = -9999.0
        req = {"dtype": "float64", "shape": [128, 128, 128], "selection": [[8, 120, 1], [0, 128, 2], [16, 112, 1]],
               "missing": {"missing_value": -9999.0}}
        op = "min" if i % 2 == 0 else "max"
        creq = make_request(op, req, oracle.convert)
        cases.append((op, req, v3.tobytes(), creq, oracle.execute(creq, v3.tobytes())))
        v4 = np.random.default_rng(0x5EED1000 + i).integers(-8, 9, 1 << 20).astype(np.float32)
        req = {"dtype": "float32", "filters": [{"id": "shuffle", "element_size": 4}]}
        data = oracle.shuffle(v4.tobytes(), 4)
        creq = make_request("sum", req, oracle.convert)
        cases.append(("sum", req, data, creq, oracle.execute(creq, data)))
    return cases


def test_direct_path_single_caller(torch):
    """One caller at a time (a lightly loaded server): every coalescible request finds the coalescer idle and
    launches on the caller's own thread (the idle-queue fast path, rdx_device_stats.direct_requests), for
    resident chunks and for host chunks up to coalesce_host_max_bytes; bit-exact vs the oracle, and no
    coalesced launch is issued."""
    eng = Engine([0])
    conf = _config_cases()
    cases = conf + _cases(7800, 120, allaxes_only=True)
    bufs = _to_device(torch, cases)
    for i, case in enumerate(cases):
        _check_one(case, *eng.execute_resident(case[3], 0, bufs[i].data_ptr(), len(case[2])))
        if i == len(conf) - 1:
            assert eng.stats(0)["direct_requests"] == len(conf)
    s = eng.stats(0)
    assert s["requests"] == _plannable(cases) and s["coalesced_requests"] == 0 and s["coalesced_launches"] == 0
    assert s["direct_requests"] > len(conf), s
    small = [c for c in cases if len(c[2]) <= 1 << 20]
    for case in small:
        _check_one(case, *eng.execute_raw(case[3], case[2]))
    s2 = eng.stats(0)
    assert s2["direct_requests"] > s["direct_requests"] and s2["coalesced_requests"] == 0
    assert s2["workspaces_busy"] == 0 and s2["outstanding_bytes"] == 0
    eng.close()


@pytest.mark.parametrize("n_threads", [15, 60])
def test_pool_eight_entries_one_gpu(torch, n_threads):
    """rdx_context_create([0] * 8): the shape an 8-GPU node runs (app_state.rs:21-37, one pool entry per
    device), here eight entries on one GPU — eight dispatcher threads, placement over eight entries, teardown.

    Mixed: 15 / 60 threads of C1 / C3 / C4 requests, resident and (every fifth) from host memory, each
    bit-exact vs the oracle, every entry used.
    Balance.  Placement keys on OUTSTANDING bytes (resource_manager.rs:54-89 bounds memory in flight), so
    what it balances is work in flight, not cumulative bytes: an entry whose requests finish more slowly
    (here: streams of eight entries share the GPU's 4 hardware queues) is given fewer.  The bound it keeps:
    a request goes to the entry with the least in flight, so with T callers no entry ever holds more than
    ceil(T / 8) requests' weight, plus one for placements racing on the relaxed loads.  Uniform (the
    server's shape: every chunk arrives in host memory, chunk_store.rs:124-150): C4 chunks from host memory
    at 15 threads, every entry's peak_outstanding_bytes <= 3 x (4 MiB + 64 KiB), and every entry serves.
    The context is destroyed with the dispatchers idle and returns."""
    eng = Engine([0] * 8)
    base = _config_cases()
    bufs = _to_device(torch, base)
    n_req = 40 * n_threads if n_threads <= 15 else 16 * n_threads
    work = [(i % len(base), i % 5 == 4) for i in range(n_req)]        # every fifth from host memory

    def one(w):
        k, host = w
        case = base[k]
        r = eng.execute_raw(case[3], case[2]) if host else \
            eng.execute_resident(case[3], 0, bufs[k].data_ptr(), len(case[2]))
        return k, r

    def placed(before=None):
        st = [eng.stats(i) for i in range(8)]
        b = [s["placed_bytes"] for s in st]
        return st, (b if before is None else [x - y for x, y in zip(b, before)])

    res = _threaded(n_threads, work, one)
    for k, r in res:
        _check_one(base[k], *r)
    stats, pb = placed()
    reqs = [s["requests"] for s in stats]
    assert sum(reqs) == n_req and sum(pb) == sum(len(base[k][2]) for k, _ in work)
    peaks = [s["peak_outstanding_bytes"] for s in stats]
    wmax = max(len(c[2]) for c in base) + (64 << 10)      # the heaviest request's placement weight
    bound = (-(-n_threads // 8) + 1) * wmax
    print("mixed: requests per entry", reqs, "placed MiB", [round(b / 2**20) for b in pb],
          "peak in flight / max weight", [round(p / wmax, 2) for p in peaks])
    # What least-outstanding placement keeps is the work IN FLIGHT per entry, not cumulative bytes: each
    # request goes to the entry holding the least, which is at most the mean of the other T - 1 callers'
    # weights, so no entry ever holds more than ceil(T / 8) heaviest requests plus the one being placed
    # (racing placements on the relaxed loads included).  Cumulative bytes are not balanced by design: with
    # eight entries on one GPU an entry whose requests finish faster is rightly given more (round 5: entry 0,
    # 2.69 x the mean).
    assert all(r > 0 for r in reqs), reqs
    assert all(p <= bound for p in peaks), (peaks, bound)
    assert all(s["device"] == 0 and s["workspaces_busy"] == 0 and s["outstanding_bytes"] == 0 for s in stats)
    assert all(s["workspaces"] <= s["max_workspaces"] for s in stats)
    assert sum(s["coalesced_requests"] + s["direct_requests"] for s in stats) > 0

    c4 = [k for k in range(len(base)) if base[k][1].get("filters")]
    uni = [(c4[i % len(c4)], True) for i in range(1500)]
    res = _threaded(15, uni, one)
    for k, r in res:
        _check_one(base[k], *r)
    eng.close()
    eng = Engine([0] * 8)
    res = _threaded(15, uni, one)
    for k, r in res:
        _check_one(base[k], *r)
    st2, pb2 = placed()
    peaks = [s["peak_outstanding_bytes"] for s in st2]
    weight = (4 << 20) + (64 << 10)
    print("uniform host C4: placed MiB", [round(b / 2**20) for b in pb2], "peak in flight (requests)",
          [round(p / weight, 2) for p in peaks])
    assert all(b > 0 for b in pb2) and all(p <= 3 * weight for p in peaks), (pb2, peaks)
    eng.close()
