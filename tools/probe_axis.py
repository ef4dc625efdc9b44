#!/usr/bin/env python3
"""Axis-reduction probe: event time per launch for a set of axis configs under this process's
tuning environment (run it once per setting).  One JSON line per config."""
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
knobs = {k: v for k, v in os.environ.items() if k.startswith("RDX_")}

CONFIGS = (("axis1_f32_4096x4096_sum", "float32", [4096, 4096], 1, "sum"),
           ("axis0_f32_4096x4096_sum", "float32", [4096, 4096], 0, "sum"),
           ("axes02_f64_128cube_max", "float64", [128, 128, 128], [0, 2], "max"),
           ("axis1_f32_64x1024x256_sum", "float32", [64, 1024, 256], 1, "sum"),
           ("axis2_i32_256x256x256_count_missing", "int32", [256, 256, 256], 2, "count"),
           ("axis0_f64_65536x32_min", "float64", [65536, 32], 0, "min"),
           ("axis1_f32_16x1048576_sum", "float32", [16, 1 << 20], 1, "sum"))
if "--minmax" in sys.argv:   # sum vs max vs min on the same shapes (float ±0 rank bookkeeping cost)
    CONFIGS = tuple((f"{nm}_{op}", dt, sh, ax, op) + tuple(rest)
                    for nm, dt, sh, ax, *rest in (("axis1_f32_4096x4096", "float32", [4096, 4096], 1),
                                                  ("axis0_f32_4096x4096", "float32", [4096, 4096], 0),
                                                  ("all_f32_256cube_sel_stride2", "float32", [256, 256, 256], None,
                                                   [[0, 256, 1], [32, 224, 1], [0, 256, 2]]),
                                                  ("all_f64_128cube_sel", "float64", [128, 128, 128], None,
                                                   [[8, 120, 1], [0, 128, 2], [16, 112, 1]]))
                    for op in ("sum", "max", "min"))
ra = np.random.default_rng(7)
COLS_ONLY = ("axis0_f32_4096x4096_sum", "axis1_f32_64x1024x256_sum", "axis0_f64_65536x32_min")
for name, dtype, shape, axis, op, *sel in CONFIGS:
    if "--cols" in sys.argv and name not in COLS_ONLY:
        continue
    n = int(np.prod(shape))
    vals = (ra.standard_normal(n) if dtype.startswith("f") else ra.integers(-100, 100, n)).astype(dtype)
    mk, mv, nm = (None, b"", 0)
    if op == "count":
        mk, mv, nm = "valid_min", np.int32(0).tobytes(), 1
    creq = _abi.CRequest(op, dtype, shape=shape, axis=axis, missing_kind=mk, missing_values=mv, n_missing=nm,
                         selection=sel[0] if sel else None)
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, vals.nbytes, C.byref(info)) == 0
    reps = max(2, (320 << 20) // vals.nbytes + 1)
    bufs = [torch.from_numpy(vals.view(np.uint8)).cuda() for _ in range(reps)]
    body = torch.empty(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(max(1, info.n_counts), dtype=torch.int64, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    args = [(ws.ws, creq.ref, C.c_void_p(b.data_ptr()), vals.nbytes, C.c_void_p(body.data_ptr()),
             C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), SH, None) for b in bufs]
    for i in range(5):
        assert lib.rdx_execute_device(*args[i % len(args)]) == 0
    torch.cuda.synchronize()
    k = 40
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(k):
        lib.rdx_execute_device(*args[i % len(args)])
    e1.record(stream)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 or "RDX_AXIS_PROBE" in knobs
    t = e0.elapsed_time(e1) / 1e3 / k
    alg = vals.nbytes + info.body_bytes + 8 * info.n_counts
    print(json.dumps({"cfg": name, "knobs": knobs, "us": round(t * 1e6, 2),
                      "frac": round(alg / t / 8e12, 4)}), flush=True)
    del bufs
ws.close()
eng.close()
