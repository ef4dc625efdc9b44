#!/usr/bin/env python3
"""Per-config measurements beyond bench.py's headline (BASELINE.json configs 3 and 5, single-chunk
C2, host-inclusive rates).  Device-resident timings: HIP events on the launch stream around K
back-to-back launches over rotating buffers whose total exceeds the 256 MiB Infinity Cache.
Prints one JSON object per measurement."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

PEAK = 8000.0
eng = Engine([0])
ws = eng.workspace(0)
lib = _abi.lib()
stream = torch.cuda.current_stream()
SH = C.c_void_p(stream.cuda_stream)


def dev_time(creq, bufs, nbytes, out_bytes, k=50):
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, nbytes, C.byref(info)) == 0
    assert out_bytes >= info.body_bytes, "body buffer smaller than the planned response"
    body = torch.empty(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(max(1, info.n_counts), dtype=torch.int64, device="cuda")  # sized from rdx_plan
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    info = _abi.rdx_response_info()
    args = [(ws.ws, creq.ref, C.c_void_p(b.data_ptr()), nbytes, C.c_void_p(body.data_ptr()),
             C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), SH, C.byref(info)) for b in bufs]
    for i in range(5):
        assert lib.rdx_execute_device(*args[i % len(args)]) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    h0 = time.perf_counter()
    for i in range(k):
        lib.rdx_execute_device(*args[i % len(args)])
    HOST["us"] = round((time.perf_counter() - h0) / k * 1e6, 2)   # host cost per call (plan + launch + ctypes)
    e1.record(stream)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    return e0.elapsed_time(e1) / 1e3 / k


HOST = {}


def conc_time(creq, bufs, nbytes, n_th=4, k=4000):
    """Concurrent requests the way the server issues them (one request per worker thread,
    src/app.rs:123-153): n_th host threads, each with its own workspace, HIP stream and output
    buffers, issue k/n_th single-chunk rdx_execute_device calls over the rotating buffers (ctypes
    releases the GIL).  Returns wall seconds per request, synchronize on both sides."""
    import threading
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, nbytes, C.byref(info)) == 0
    per = []
    for t in range(n_th):
        w = eng.workspace(0)
        st = torch.cuda.Stream()
        body = torch.empty(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(max(1, info.n_counts), dtype=torch.int64, device="cuda")
        status = torch.zeros(4, dtype=torch.int32, device="cuda")
        per.append((w, st, body, counts, status))
    errs = []

    def worker(t, n):
        w, st, body, counts, status = per[t]
        inf = _abi.rdx_response_info()
        args = [(w.ws, creq.ref, C.c_void_p(b.data_ptr()), nbytes, C.c_void_p(body.data_ptr()),
                 C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), C.c_void_p(st.cuda_stream),
                 C.byref(inf)) for b in bufs]
        for i in range(n):
            r = lib.rdx_execute_device(*args[(i * n_th + t) % len(args)])
            if r:
                errs.append(r)
                return

    for t in range(n_th):   # warm-up: every thread's path once
        worker(t, 3)
    torch.cuda.synchronize()
    ths = [threading.Thread(target=worker, args=(t, k // n_th)) for t in range(n_th)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert not errs and all(int(p[4].abs().sum()) == 0 for p in per)
    for p in per:
        p[0].close()
    return el / (k // n_th * n_th)
NO_CPU = "--no-cpu" in sys.argv   # profiling runs: skip the oracle timings


def cpu_time(creq, data, seconds=3.0):
    """Oracle (sequential restatement of the reference path) on one host core."""
    if NO_CPU:
        return float("nan")
    from oracle import py_oracle as oracle
    L = oracle.lib()
    src = C.create_string_buffer(data, len(data))
    cap = len(data) + 64
    body = (C.c_uint8 * cap)()
    counts = (C.c_int64 * (len(data) // 4 + 8))()
    info = _abi.rdx_response_info()
    reps, t0 = 0, time.perf_counter()
    while True:
        assert L.oracle_execute(C.addressof(creq.c), src, len(data), body, cap, counts, len(data) // 4 + 8,
                                C.byref(info)) == 0
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return (time.perf_counter() - t0) / reps


def report(name, t, alg_bytes, chunk_bytes, **kw):
    d = {"config": name, "us_per_launch": round(t * 1e6, 2), "bytes_alg": alg_bytes,
         "GBs_alg": round(alg_bytes / t / 1e9, 1), "roofline_frac": round(alg_bytes / t / 1e9 / PEAK, 4),
         "GiBs_chunk": round(chunk_bytes / t / 2 ** 30, 1)}
    if HOST:
        d["host_us_per_call"] = HOST.pop("us")
    d.update(kw)
    print(json.dumps(d), flush=True)


# ---- C3: f64 [128,128,128], selection, missing_value -9999 @5 %, min / max / valid_range ----------------
rng = np.random.default_rng(0x5EED0005)
v = rng.standard_normal(128 ** 3) * 100
v[rng.random(v.size) < 0.05] = -9999.0
c3 = [torch.from_numpy(v.view(np.uint8).copy()).cuda() for _ in range(20)]  # 320 MiB rotating
sel = [[8, 120, 1], [0, 128, 2], [16, 112, 1]]
n_sel = 112 * 64 * 96
for op, miss in (("min", ("missing_value", -9999.0)), ("max", ("missing_value", -9999.0)),
                 ("max", ("valid_range", [-250.0, 250.0])), ("sum", ("missing_value", -9999.0))):
    vals = miss[1] if isinstance(miss[1], list) else [miss[1]]
    mv = b"".join(np.float64(x).tobytes() for x in vals)
    creq = _abi.CRequest(op, "float64", shape=[128, 128, 128], selection=sel, missing_kind=miss[0],
                         missing_values=mv, n_missing=len(vals))
    t = dev_time(creq, c3, 128 ** 3 * 8, 8)
    tc = cpu_time(creq, v.tobytes())
    report(f"c3_{op}_{miss[0]}", t, n_sel * 8 + 16, 128 ** 3 * 8, n_selected=n_sel,
           cpu_oracle_us=round(tc * 1e6, 1), gpu_over_cpu=round(tc / t, 1))
    if op == "min":
        tcc = conc_time(creq, c3, 128 ** 3 * 8)
        report(f"c3_{op}_{miss[0]}_concurrent4", tcc, n_sel * 8 + 16, 128 ** 3 * 8, n_selected=n_sel,
               note="4 host threads x (workspace, stream), wall clock per request")
# C3 as a batch: 20 independent 16 MiB chunks per launch (rdx_execute_batch_device), min
creqb = _abi.CRequest("min", "float64", shape=[128, 128, 128], selection=sel, missing_kind="missing_value",
                      missing_values=np.float64(-9999.0).tobytes(), n_missing=1)
bb = torch.zeros(len(c3), dtype=torch.float64, device="cuda")
bc = torch.zeros(len(c3), dtype=torch.int64, device="cuda")
bs = torch.zeros(len(c3), dtype=torch.int32, device="cuda")
for _ in range(3):
    ws.execute_batch_device(creqb, [b.data_ptr() for b in c3], 128 ** 3 * 8, bb.data_ptr(), bc.data_ptr(),
                            bs.data_ptr(), stream.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for _ in range(20):
    ws.execute_batch_device(creqb, [b.data_ptr() for b in c3], 128 ** 3 * 8, bb.data_ptr(), bc.data_ptr(),
                            bs.data_ptr(), stream.cuda_stream)
e1.record(stream)
torch.cuda.synchronize()
tb = e0.elapsed_time(e1) / 1e3 / 20
report("c3_min_missing_value_batch20", tb, len(c3) * (n_sel * 8 + 16), len(c3) * 128 ** 3 * 8,
       chunks_per_launch=len(c3), us_per_chunk=round(tb / len(c3) * 1e6, 2))
del c3

# ---- C1 (CPU-only config in BASELINE): f32 4 MiB contiguous sum; D-int and D-real ------------------------
for seed, real in ((0x5EED0001, False), (0x5EED0002, True)):
    r1 = np.random.default_rng(seed)
    v1 = (r1.random(1 << 20, dtype=np.float32) if real else r1.integers(-8, 9, 1 << 20).astype(np.float32))
    creq1 = _abi.CRequest("sum", "float32")
    tc = cpu_time(creq1, v1.tobytes())
    bufs = [torch.from_numpy(v1.view(np.uint8).copy()).cuda() for _ in range(80)]   # 320 MiB rotating
    t = dev_time(creq1, bufs, 4 << 20, 4)
    report("c1_sum_4MiB_" + ("real" if real else "int"), t, 4 << 20, 4 << 20, cpu_oracle_us=round(tc * 1e6, 1),
           cpu_oracle_GiBs=round((4 << 20) / tc / 2 ** 30, 3), gpu_over_cpu=round(tc / t, 1))
    if real:
        tcc = conc_time(creq1, bufs, 4 << 20)
        report("c1_sum_4MiB_real_concurrent4", tcc, 4 << 20, 4 << 20,
               note="4 host threads x (workspace, stream), wall clock per request")
    del bufs

# ---- axis reductions ---------------------------------------------------------------------------------
ra = np.random.default_rng(7)
for name, dtype, shape, axis, op in (("axis1_f32_4096x4096_sum", "float32", [4096, 4096], 1, "sum"),
                                     ("axis0_f32_4096x4096_sum", "float32", [4096, 4096], 0, "sum"),
                                     ("axes02_f64_128cube_max", "float64", [128, 128, 128], [0, 2], "max"),
                                     ("axis1_f32_64x1024x256_sum", "float32", [64, 1024, 256], 1, "sum"),
                                     ("axis2_i32_256x256x256_count_missing", "int32", [256, 256, 256], 2, "count"),
                                     ("axisnone_f32_16M_min_map", "float32", [4096, 4096], [], "min")):
    n = int(np.prod(shape))
    vals = (ra.standard_normal(n) if dtype.startswith("f") else ra.integers(-100, 100, n)).astype(dtype)
    mk, mv, nm = (None, b"", 0)
    if op == "count":
        mk, mv, nm = "valid_min", np.int32(0).tobytes(), 1
    creq = _abi.CRequest(op, dtype, shape=shape, axis=axis, missing_kind=mk, missing_values=mv, n_missing=nm)
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, vals.nbytes, C.byref(info)) == 0
    reps = max(2, (320 << 20) // vals.nbytes + 1)
    bufs = [torch.from_numpy(vals.view(np.uint8)).cuda() for _ in range(reps)]
    t = dev_time(creq, bufs, vals.nbytes, info.body_bytes, k=30)
    tc = cpu_time(creq, vals.tobytes(), seconds=2.0)
    alg = vals.nbytes + info.body_bytes + 8 * info.n_counts
    report(name, t, alg, vals.nbytes, outputs=int(info.n_counts), cpu_oracle_us=round(tc * 1e6, 1),
           gpu_over_cpu=round(tc / t, 1))
    del bufs

# ---- C5: i64 [512,256,256] select [[0,512,1],[64,192,1],[0,256,1]] -> 128 MiB out ----------------------
g = torch.Generator(device="cuda")
g.manual_seed(0x5EED0006)
c5 = [torch.randint(-2 ** 62, 2 ** 62, (512 * 256 * 256,), dtype=torch.int64, device="cuda", generator=g).view(torch.uint8)
      for _ in range(2)]
creq5 = _abi.CRequest("select", "int64", shape=[512, 256, 256], selection=[[0, 512, 1], [64, 192, 1], [0, 256, 1]])
t = dev_time(creq5, c5, 256 << 20, 128 << 20, k=20)
host5 = c5[0].cpu().numpy().tobytes()
tc = cpu_time(creq5, host5, seconds=3.0)
report("c5_select_device", t, (128 << 20) * 2, 256 << 20, note="128 MiB read + 128 MiB written",
       cpu_oracle_us=round(tc * 1e6, 1), gpu_over_cpu=round(tc / t, 1))
tcc = conc_time(creq5, c5, 256 << 20, k=400)
report("c5_select_device_concurrent4", tcc, (128 << 20) * 2, 256 << 20,
       note="4 host threads x (workspace, stream, 128 MiB body), wall clock per request")

# host-inclusive C5: host chunk in (pageable), 128 MiB body out (pageable) through rdx_execute
del c5
eng.execute_raw(creq5, host5)   # warm-up: the first call sizes the staging / device buffers
t0 = time.perf_counter()
reps = 3
for _ in range(reps):
    st, info, body, counts = eng.execute_raw(creq5, host5)
    assert st == 0
t = (time.perf_counter() - t0) / reps
print(json.dumps({"config": "c5_select_host_inclusive", "ms_per_call": round(t * 1e3, 2),
                  "GiBs_chunk": round((256 << 20) / t / 2 ** 30, 2),
                  "note": "rdx_execute: pageable H2D 256 MiB + kernel + pageable D2H 128 MiB + ctypes copies"}), flush=True)

# ---- C2 host-inclusive: 64 MiB shuffled big-endian f32 from host memory ---------------------------------
vals = np.random.default_rng(4).random(16 << 20, dtype=np.float32)
host2 = vals.astype(">f4").view(np.uint8).reshape(-1, 4).T.copy().tobytes()
creq2 = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
for _ in range(2):
    eng.execute_raw(creq2, host2)
t0 = time.perf_counter()
reps = 10
for _ in range(reps):
    st, info, body, counts = eng.execute_raw(creq2, host2)
t = (time.perf_counter() - t0) / reps
print(json.dumps({"config": "c2_host_inclusive", "ms_per_call": round(t * 1e3, 3),
                  "GiBs_chunk": round((64 << 20) / t / 2 ** 30, 2),
                  "note": "rdx_execute: pageable H2D 64 MiB + kernel + 16 B D2H"}), flush=True)
ws.close()
eng.close()
