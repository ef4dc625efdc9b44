#!/usr/bin/env python3
"""Byte-shuffled all-axes sums over 8 HBM-resident chunks: does the spacing of the byte planes matter?
A 64 MiB chunk's planes start exactly 2^23 (f64) / 2^24 (f32) bytes apart; the same sums over chunks a
little longer (planes 2^23 + 8 KiB apart) tell whether the 8 (4) concurrent plane streams of a workgroup
alias onto the same memory channels.  Event time per launch (20 launches, after 5 warm-up).
Usage: python tools/probe_planes.py  (RDX_FORCE_BPC etc. from the environment)"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

eng = Engine([0])
ws = eng.workspace(0)
stream = torch.cuda.current_stream()
NB = 8
out = torch.zeros(NB, dtype=torch.float64, device="cuda")
counts = torch.zeros(NB, dtype=torch.int64, device="cuda")
status = torch.zeros(NB, dtype=torch.int32, device="cuda")
QUICK = os.environ.get("PLANES_QUICK") == "1"   # 64 MiB chunks only, PLANES_DTYPES (default float64)
SIZES = {"float64": 8, "int64": 8, "uint64": 8, "float32": 4, "int32": 4}
DTS = [(d, SIZES[d]) for d in os.environ.get("PLANES_DTYPES", "float64").split(",")]
OPS = os.environ.get("PLANES_OPS", "sum").split(",")
for dtype, es in DTS if QUICK else (("float64", 8), ("float32", 4)):
    for extra in (0,) if QUICK else (0, 8192 * es, 65536 * es):
        nbytes = (64 << 20) + extra
        raw = torch.randint(0, 256, (NB, nbytes), dtype=torch.uint8, device="cuda")
        raw.view(NB, -1)[:, (nbytes // es) * (es - 1):] &= 0x3F   # the top byte plane: finite values
        ptrs = [raw[i].data_ptr() for i in range(NB)]
        for op, shuf in [(o, sh) for o in OPS for sh in (True, False)]:
            creq = _abi.CRequest(op, dtype, byte_order="big",
                                 filters=[{"id": "shuffle", "element_size": es}] if shuf else [])

            def launch():
                ws.execute_batch_device(creq, ptrs, nbytes, out.data_ptr(), counts.data_ptr(), status.data_ptr(),
                                        stream.cuda_stream)
            for _ in range(5):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                launch()
            e1.record(stream)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 20
            print(json.dumps({"dtype": dtype, "op": op, "shuffle": shuf, "chunk_bytes": nbytes, "plane_bytes": nbytes // es,
                              "us": round(us, 2), "frac": round(NB * nbytes / us / 1e3 / 8000, 4),
                              "force_bpc": os.environ.get("RDX_FORCE_BPC", ""), "lib": Path(os.environ.get("RDX_LIB_PATH", "librdx.so")).name}), flush=True)
        del raw
ws.close()
eng.close()
