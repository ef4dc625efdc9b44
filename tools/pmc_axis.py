#!/usr/bin/env python3
"""Round 6: the two axis kernels alone on [4096,4096] f32 (k_axis_cols: axis 0, k_axis_rows: axis 1), K launches
each over 6 rotating 64 MiB buffers, for rocprofv3 --pmc passes of occupancy / stall / VALU counters
(tools/gpu_r06_axis_pmc.sh).  usage: python tools/pmc_axis.py [K]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
eng = Engine([0])
ws = eng.workspace(0)
lib = _abi.lib()
stream = torch.cuda.current_stream()
SH = C.c_void_p(stream.cuda_stream)
g = torch.Generator(device="cuda")
g.manual_seed(3)
a = [torch.rand(4096 * 4096, device="cuda", generator=g) for _ in range(6)]
for axis in (0, 1):
    creq = _abi.CRequest("sum", "float32", shape=[4096, 4096], axis=axis)
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, 64 << 20, C.byref(info)) == 0
    body = torch.zeros(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(max(2, info.n_counts), dtype=torch.int64, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    for i in range(K + len(a)):
        assert lib.rdx_execute_device(ws.ws, creq.ref, C.c_void_p(a[i % len(a)].data_ptr()), 64 << 20,
                                      C.c_void_p(body.data_ptr()), C.c_void_p(counts.data_ptr()),
                                      C.c_void_p(status.data_ptr()), SH, C.byref(info)) == 0
    torch.cuda.synchronize()
    ref = a[(K + len(a) - 1) % len(a)].view(4096, 4096).double().sum(dim=axis)
    got = body[:4096 * 4].view(torch.float32).double()
    assert bool(((got - ref).abs() <= ref.abs() * 1e-6 + 1e-3).all())
print("pmc_axis: done", flush=True)
