#!/usr/bin/env python3
"""Batched all-axes variants over 8 x 64 MiB HBM-resident chunks: f32 vs f64, sum vs min, plain vs
shuffled, native vs big-endian.  Event time per launch; isolates what the f64 legs pay for."""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

eng = Engine([0])
ws = eng.workspace(0)
stream = torch.cuda.current_stream()
NB, BYTES = 8, 64 << 20
raw = torch.randint(0, 256, (NB, BYTES), dtype=torch.uint8, device="cuda")
# keep values finite and NaN-free for min: clear the top exponent bits' byte in every element (f32 and f64)
v = raw.view(NB, -1, 8)
v[:, :, 7] &= 0x3F
v[:, :, 3] &= 0x3F
v[:, :, 0] &= 0x3F
v[:, :, 4] &= 0x3F
bodies = torch.zeros(NB, dtype=torch.float64, device="cuda")
counts = torch.zeros(NB, dtype=torch.int64, device="cuda")
status = torch.zeros(NB, dtype=torch.int32, device="cuda")
ptrs = [raw[i].data_ptr() for i in range(NB)]
for dtype, es in (("float32", 4), ("float64", 8)):
    for op in ("sum", "min", "count"):
        for shuf in (False, True):
            for bo in ("little", "big"):
                creq = _abi.CRequest(op, dtype, byte_order=bo,
                                     filters=[{"id": "shuffle", "element_size": es}] if shuf else [])
                def launch():
                    ws.execute_batch_device(creq, ptrs, BYTES, bodies.data_ptr(), counts.data_ptr(),
                                            status.data_ptr(), stream.cuda_stream)
                for _ in range(5):
                    launch()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(40):
                    launch()
                e1.record(stream)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / 40
                print(json.dumps({"dtype": dtype, "op": op, "shuffle": shuf, "byte_order": bo,
                                  "us": round(t * 1e6, 2), "frac": round(NB * BYTES / t / 8e12, 4),
                                  "status": int(status.abs().sum())}), flush=True)
