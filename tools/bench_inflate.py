#!/usr/bin/env python3
"""Device decompression throughput (k_inflate via rdx_decompress_batch_device) on batches of
compressed chunks, against the CPU: the oracle (sequential restatement, 1 core) and CPython's zlib
(the C zlib library, on a thread pool like the reference's worker threads).  One JSON line per
workload.

Workloads (4 MiB f32 chunks, byte-shuffled as HDF5/netCDF writers store them, then compressed):
  noise  : N(0,1) f32 — mantissa bytes are incompressible, exponent bytes compress well
  field  : a smooth 2-D field quantised to 16 bits of precision (scale/offset-packed climate data)
DISTINCT distinct chunks are compressed once and cycled to fill the batch."""
import argparse
import ctypes as C
import json
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from oracle import py_oracle as oracle  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--distinct", type=int, default=32)
ap.add_argument("--elems", type=int, default=1 << 20)
ap.add_argument("--level", type=int, default=1)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--formats", default="zlib,gzip")
ap.add_argument("--kinds", default="noise,field")
ap.add_argument("--cpu-threads", type=int, default=15)
args = ap.parse_args()

eng = Engine([0])
ws = eng.workspace(0)
stream = torch.cuda.current_stream()


def chunk(kind, rng, i):
    n = args.elems
    if kind == "noise":
        v = rng.standard_normal(n).astype(np.float32)
    else:
        side = int(np.sqrt(n))
        y, x = np.mgrid[0:side, 0:n // side].astype(np.float32) / side
        f = 280 + 20 * np.sin(6.3 * x + i) * np.cos(3.1 * y) + 0.05 * rng.standard_normal(x.shape).astype(np.float32)
        v = (np.round(f * 200) / 200).astype(np.float32).ravel()
    return oracle.shuffle(v.tobytes(), 4)


def compress(fmt, b):
    c = zlib.compressobj(args.level, zlib.DEFLATED, 31 if fmt == "gzip" else 15)
    return c.compress(b) + c.flush()


for kind in args.kinds.split(","):
    rng = np.random.default_rng(1)
    raws = [chunk(kind, rng, i) for i in range(args.distinct)]
    raw_len = len(raws[0])
    for fmt in args.formats.split(","):
        streams = [compress(fmt, r) for r in raws]
        offs, total = [], 0
        for s in streams:
            offs.append(total)
            total += (len(s) + 255) // 256 * 256
        host = np.zeros(total, dtype=np.uint8)
        for o, s in zip(offs, streams):
            host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
        d_in = torch.from_numpy(host).cuda()
        ptrs = [d_in.data_ptr() + offs[i % args.distinct] for i in range(args.batch)]
        lens = [len(streams[i % args.distinct]) for i in range(args.batch)]
        cap = (raw_len + 15) // 16 * 16
        d_out = torch.empty(args.batch * cap, dtype=torch.uint8, device="cuda")
        d_len = torch.zeros(args.batch, dtype=torch.int64, device="cuda")
        d_err = torch.zeros(args.batch, dtype=torch.int32, device="cuda")

        def launch():
            ws.decompress_batch_device(fmt, ptrs, lens, d_out.data_ptr(), cap, d_len.data_ptr(), d_err.data_ptr(),
                                       stream.cuda_stream)

        launch()
        torch.cuda.synchronize()
        assert int(d_err.abs().sum()) == 0 and bool((d_len == raw_len).all())
        got = d_out[:cap].cpu().numpy().tobytes()[:raw_len]
        assert got == raws[0]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            launch()
        e1.record(stream)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / args.reps
        comp_bytes = sum(lens)
        # CPU: CPython zlib (C library) on a thread pool over the whole batch, and the oracle on 1 core
        wb = 31 if fmt == "gzip" else 15

        def one(i):
            zlib.decompress(streams[i % args.distinct], wb)

        with ThreadPoolExecutor(args.cpu_threads) as ex:
            list(ex.map(one, range(args.cpu_threads)))
            c0 = time.perf_counter()
            list(ex.map(one, range(args.batch)))
            tz = time.perf_counter() - c0
        c0 = time.perf_counter()
        e, _ = oracle.decompress(1 if fmt == "gzip" else 2, streams[0], cap)
        to = time.perf_counter() - c0
        assert e == 0
        print(json.dumps({
            "workload": f"{args.batch} x {raw_len >> 20} MiB f32 chunks, shuffle es=4, {fmt} level {args.level}, {kind}",
            "ratio": round(raw_len * args.distinct / sum(len(s) for s in streams), 3),
            "device_ms": round(t * 1e3, 3),
            "device_GBs_out": round(args.batch * raw_len / t / 1e9, 2),
            "device_GBs_in": round(comp_bytes / t / 1e9, 2),
            "cpu_zlib_GBs_out": round(args.batch * raw_len / tz / 1e9, 3), "cpu_zlib_threads": args.cpu_threads,
            "cpu_oracle_GBs_out_1core": round(raw_len / to / 1e9, 4),
        }), flush=True)
        del d_in, d_out
ws.close()
eng.close()
