#!/usr/bin/env python3
"""Latency probe for small single-chunk launches (C1, C3 and a C3-sized contiguous run): event time
per launch over K back-to-back launches, for the RDX_FORCE_BPC of this process (run it
once per setting).  One JSON line per config."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

eng = Engine([0])
ws = eng.workspace(0)
lib = _abi.lib()
stream = torch.cuda.current_stream()
SH = C.c_void_p(stream.cuda_stream)


def dev_time(creq, bufs, nbytes, k=200):
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, nbytes, C.byref(info)) == 0
    body = torch.empty(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(max(1, info.n_counts), dtype=torch.int64, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    args = [(ws.ws, creq.ref, C.c_void_p(b.data_ptr()), nbytes, C.c_void_p(body.data_ptr()),
             C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), SH, None) for b in bufs]
    for i in range(10):
        assert lib.rdx_execute_device(*args[i % len(args)]) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(k):
        lib.rdx_execute_device(*args[i % len(args)])
    e1.record(stream)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0
    return e0.elapsed_time(e1) / 1e3 / k


bpc = os.environ.get("RDX_FORCE_BPC", "auto")
rng = np.random.default_rng(5)
v3 = rng.standard_normal(128 ** 3) * 100
c3 = [torch.from_numpy(v3.view(np.uint8).copy()).cuda() for _ in range(20)]
sel = [[8, 120, 1], [0, 128, 2], [16, 112, 1]]
for op in ("min", "sum"):
    creq = _abi.CRequest(op, "float64", shape=[128, 128, 128], selection=sel, missing_kind="missing_value",
                         missing_values=np.float64(-9999.0).tobytes(), n_missing=1)
    print(json.dumps({"cfg": f"c3_{op}", "bpc": bpc, "us": round(dev_time(creq, c3, 128 ** 3 * 8) * 1e6, 2)}))
creq = _abi.CRequest("min", "float64", shape=[128, 128, 128], selection=sel, missing_kind="missing_value",
                     missing_values=np.float64(-9999.0).tobytes(), n_missing=1)
out = torch.zeros(20, dtype=torch.float64, device="cuda")
cnt = torch.zeros(20, dtype=torch.int64, device="cuda")
stt = torch.zeros(20, dtype=torch.int32, device="cuda")
ptrs = [b.data_ptr() for b in c3]
for i in range(5):
    ws.execute_batch_device(creq, ptrs, 128 ** 3 * 8, out.data_ptr(), cnt.data_ptr(), stt.data_ptr(), stream.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for i in range(50):
    ws.execute_batch_device(creq, ptrs, 128 ** 3 * 8, out.data_ptr(), cnt.data_ptr(), stt.data_ptr(), stream.cuda_stream)
e1.record(stream)
torch.cuda.synchronize()
assert int(stt.abs().sum()) == 0
print(json.dumps({"cfg": "c3_min_batch20", "bpc": bpc, "us": round(e0.elapsed_time(e1) / 50 * 1e3, 2)}))
creq = _abi.CRequest("min", "float64", selection=[[0, 688128, 1]], shape=[128 ** 3])
print(json.dumps({"cfg": "c3sized_contig_min", "bpc": bpc, "us": round(dev_time(creq, c3, 128 ** 3 * 8) * 1e6, 2)}))
v1 = rng.random(1 << 20, dtype=np.float32)
c1 = [torch.from_numpy(v1.view(np.uint8).copy()).cuda() for _ in range(80)]
print(json.dumps({"cfg": "c1_sum", "bpc": bpc, "us": round(dev_time(_abi.CRequest("sum", "float32"), c1, 4 << 20) * 1e6, 2)}))
ws.close()
eng.close()
