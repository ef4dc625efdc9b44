#!/usr/bin/env python3
"""Kernel-level comparison of the heterogeneous launch (k_multi) against the same-request batch kernels:
run under rocprofv3 --kernel-trace; each case is K calls on one stream (marker kernels between cases)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

eng = Engine([0])
ws = eng.workspace(0)
stream = torch.cuda.current_stream().cuda_stream
v3 = bench._c3_host()
v1 = np.random.default_rng(2).random(1 << 20, dtype=np.float32)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20


def bufs(data, n):
    return [torch.from_numpy(data).cuda() for _ in range(n)]


def outs(n):
    return (torch.zeros(n, dtype=torch.float64, device="cuda"), torch.zeros(n, dtype=torch.int64, device="cuda"),
            torch.zeros(n, dtype=torch.int32, device="cuda"))


def marker(n):
    torch.full((n,), 1.0, device="cuda")   # a recognisable elementwise kernel between cases


def multi_case(specs):
    items, keep = [], []
    for creq, data, nbytes in specs:
        d = torch.from_numpy(data).cuda()
        b, c, s = outs(2)
        keep.append((d, b, c, s))
        items.append((creq, d.data_ptr(), nbytes, b.data_ptr(), c.data_ptr(), s.data_ptr()))
    for _ in range(K):
        st, _ = ws.execute_multi_device(items, stream)
        assert not any(st)
    torch.cuda.synchronize()


def batch_case(creq, data, n, nbytes):
    bb = bufs(data, n)
    b, c, s = outs(n)
    for _ in range(K):
        ws.execute_batch_device(creq, [x.data_ptr() for x in bb], nbytes, b.data_ptr(), c.data_ptr(), s.data_ptr(), stream)
    torch.cuda.synchronize()


c3 = bench._c3_req(_abi, "min")
c1 = _abi.CRequest("sum", "float32")
marker(101)
multi_case([(c3, v3, 16 << 20)] * 20)
marker(102)
batch_case(c3, v3, 20, 16 << 20)
marker(103)
multi_case([(c1, v1, 4 << 20)] * 20)
marker(104)
batch_case(c1, v1, 20, 4 << 20)
marker(105)
multi_case([(c1, v1, 4 << 20), (c3, v3, 16 << 20)] * 10)
marker(106)
