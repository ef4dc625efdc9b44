#!/usr/bin/env python3
"""Device time per launch of the two many-request kernels at small batch sizes — the coalescer's working
range (8-24 concurrent requests): k_multi (rdx_execute_multi_device, heterogeneous) against the
same-request batch kernels (rdx_execute_batch_device: k_all_contig / k_all_strided with a chunk table),
for C1 (f32 4 MiB sum) and C3 (f64 [128,128,128] hyperslab min, missing_value).  HIP events around K
back-to-back launches on one stream; chunks rotate over > 256 MiB.  One JSON line per (config, kernel, B)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

PEAK = 8000.0
eng = Engine([0])
ws = eng.workspace(0)
stream = torch.cuda.current_stream()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 60


def timed(launch, k):
    for i in range(5):
        launch(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(k):
        launch(i)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k   # us


def run(name, creq, data, nbytes, alg, nbuf):
    bufs = [torch.from_numpy(data).cuda() for _ in range(nbuf)]
    outs = (torch.zeros(64, dtype=torch.float64, device="cuda"), torch.zeros(64, dtype=torch.int64, device="cuda"),
            torch.zeros(64, dtype=torch.int32, device="cuda"))
    for B in (1, 2, 4, 8, 12, 16, 24):
        groups = [[bufs[(g * B + j) % nbuf] for j in range(B)] for g in range(max(1, nbuf // B))]
        items = [[(creq, x.data_ptr(), nbytes, outs[0].data_ptr() + 8 * j, outs[1].data_ptr() + 8 * j,
                   outs[2].data_ptr() + 4 * j) for j, x in enumerate(gr)] for gr in groups]

        def multi(i):
            st, _ = ws.execute_multi_device(items[i % len(items)], stream.cuda_stream)

        def batch(i):
            ws.execute_batch_device(creq, [x.data_ptr() for x in groups[i % len(groups)]], nbytes, outs[0].data_ptr(),
                                    outs[1].data_ptr(), outs[2].data_ptr(), stream.cuda_stream)

        for kname, fn in (("k_multi", multi), ("batch", batch)):
            t = timed(fn, K)
            print(json.dumps({"config": name, "kernel": kname, "B": B, "us": round(t, 3),
                              "us_per_request": round(t / B, 3), "frac": round(B * alg / t / 1e3 / PEAK, 4)}), flush=True)


v1 = np.random.default_rng(2).random(1 << 20, dtype=np.float32)
run("c1", _abi.CRequest("sum", "float32"), v1, 4 << 20, 4 << 20, 80)
run("c3", bench._c3_req(_abi, "min"), bench._c3_host(), 16 << 20, 112 * 64 * 96 * 8, 24)
