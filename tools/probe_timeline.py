#!/usr/bin/env python3
"""Phase timeline of one all-axes launch (probe build: make -C reductionist-rs_amd EXTRA=-DRDX_PROBES=1
BUILD=build_probe OUT=librdx_probe.so; run with RDX_LIB_PATH=reductionist-rs_amd/librdx_probe.so).

Each workgroup of k_all_contig (and k_all_strided: the C3 hyperslab case) stamps the wall clock (100 MHz) at its first instruction, when its
streaming ends, after its record is published and its arrival counted, and (last arriver) when the fold
is done (rdx_device.hpp RDX_STAMP).  For the C2 single-chunk launch (64 MiB shuffled big-endian f32, one
chunk) and the batched launch (8 chunks) this prints, relative to the first workgroup's start: the
dispatch ramp (last start), the streaming-end spread, the last arrival and the fold end, plus each
workgroup's streaming duration (median / max) — where the launch's time goes."""
import ctypes as C
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
os.environ.setdefault("RDX_LIB_PATH", str(ROOT / "reductionist-rs_amd" / "librdx_probe.so"))
import torch  # noqa: E402
import bench  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

TICK_NS = 10.0   # wall_clock64: 100 MHz


def timeline(lib, n_wg, dtype="f32"):
    buf = (C.c_uint64 * (8 * 8192))()
    assert getattr(lib, f"rdx_probe_read_{dtype}")(buf, 8 * 8192) == 0
    rows = [(buf[8 * i], buf[8 * i + 1], buf[8 * i + 2], buf[8 * i + 3], buf[8 * i + 4]) for i in range(n_wg)]
    t0 = min(r[0] for r in rows)
    us = lambda t: round((t - t0) * TICK_NS / 1e3, 3)  # noqa: E731
    folds = [r[3] for r in rows if r[3] >= r[2] and r[3] > t0]
    stream = [(r[1] - r[0]) * TICK_NS / 1e3 for r in rows]
    return {"workgroups": n_wg, "last_start_us": us(max(r[0] for r in rows)),
            "first_stream_end_us": us(min(r[1] for r in rows)), "last_stream_end_us": us(max(r[1] for r in rows)),
            "last_arrival_us": us(max(r[2] for r in rows)), "fold_end_us": us(max(folds)) if folds else None,
            "stream_us_median": round(statistics.median(stream), 3), "stream_us_max": round(max(stream), 3),
            "start_us_deciles": [us(sorted(r[0] for r in rows)[int(q * (n_wg - 1))]) for q in (0.1, 0.5, 0.9)],
            "stream_us_deciles": [round(sorted(stream)[int(q * (n_wg - 1))], 3) for q in (0.1, 0.25, 0.5, 0.75, 0.9)],
            # per block % 8 (the XCD under round-robin dispatch): median streaming time
            "stream_us_by_xcd": [round(statistics.median(stream[i::8]), 3) for i in range(8)],
            # HW_ID placement: workgroups sharing a (SE, SH, CU) slot, and the streaming time of those
            "hwid_shared_slots": sum(1 for c in _slot_counts(rows).values() if c > 1),
            "per_wg": [[i, round(stream[i], 2), (rows[i][4] >> 8) & 0xF, (rows[i][4] >> 12) & 1, (rows[i][4] >> 13) & 7]
                       for i in range(n_wg)]}


def _slot_counts(rows):
    cnt = {}
    for i, r in enumerate(rows):
        key = (i % 8, (r[4] >> 8) & 0xFF)   # (XCD under round-robin dispatch, CU_ID / SH_ID / SE_ID)
        cnt[key] = cnt.get(key, 0) + 1
    return cnt


def main():
    eng = Engine([0])
    ws = eng.workspace(0)
    lib = _abi.lib()
    stream = torch.cuda.current_stream()
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    vals = torch.rand((8, bench.C2_ELEMS), device="cuda", generator=g)
    chunks = [c.contiguous() for c in bench.shuffled_be_f32(torch, vals)]
    creq = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
    out = torch.zeros(8, dtype=torch.float64, device="cuda")
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    res = {}
    for k in range(12):   # single chunk, rotating; the last launch's timeline is read
        info = ws.execute_device(creq, chunks[k % 8].data_ptr(), bench.C2_BYTES, out.data_ptr(), cnt.data_ptr(), None,
                                 stream.cuda_stream)
    torch.cuda.synchronize()
    res["c2_single"] = timeline(lib, 256)
    for k in range(6):
        ws.execute_batch_device(creq, [c.data_ptr() for c in chunks], bench.C2_BYTES, out.data_ptr(), cnt.data_ptr(),
                                None, stream.cuda_stream)
    torch.cuda.synchronize()
    res["c2_batch8"] = timeline(lib, 256)   # 8 chunks x 32 workgroups (pick_bpc: one per CU in all)
    # C3: f64 [128,128,128] hyperslab min with missing_value (k_all_strided, VW = 2: 1024 vectors per
    # workgroup -> 336 workgroups)
    v = torch.from_numpy(bench._c3_host()).cuda()
    c3 = bench._c3_req(_abi, "min")
    o8 = torch.zeros(2, dtype=torch.float64, device="cuda")
    for k in range(12):
        ws.execute_device(c3, v.data_ptr(), v.numel() * 8, o8.data_ptr(), cnt.data_ptr(), None, stream.cuda_stream)
    torch.cuda.synchronize()
    res["c3_min"] = timeline(lib, (bench.C3_NSEL // 2 + 1023) // 1024, "f64")
    # C1: f32 4 MiB contiguous sum (k_all_contig, 128 workgroups of 2 tiles)
    v1 = torch.rand(1 << 20, device="cuda", generator=g)
    c1 = _abi.CRequest("sum", "float32")
    for k in range(12):
        ws.execute_device(c1, v1.data_ptr(), 4 << 20, o8.data_ptr(), cnt.data_ptr(), None, stream.cuda_stream)
    torch.cuda.synchronize()
    res["c1_sum"] = timeline(lib, 128)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
