#!/usr/bin/env python3
"""Where k_blosc2_zstd's time goes, per stream (probe build: RDX_LIB_PATH=reductionist-rs_amd/librdx_probe.so).
The bench's blosc2 zstd chunk (random walk quantized to 1/64, SHUFFLE, typesize 4, 64 KiB blocks x 4 streams,
libzstd level 3) decoded as a lone chunk; per-row cycles of each phase (s_memtime) from rdx_probe_zprof_read,
summarised by byte plane (row % 4), plus the lone-chunk and a 64-chunk batch event time.  JSON lines."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "reductionist-rs_amd"), str(ROOT)):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from datagen import blosc2_chunk as B  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

K = 12
NAMES = ["total", "literals_section", "seq_tables", "seq_loop", "lit_copy", "match_copy", "nseq", "far_steps",
         "lit_bytes", "match_bytes", "flushes", "blocks"]


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
    eng = Engine([0])
    ws = eng.workspace(0)
    lib = _abi.lib()
    lib.rdx_probe_zprof_read.argtypes = [C.c_void_p, C.c_uint32]
    rng = np.random.default_rng(0x5EED2100)
    elems = 1 << 20
    raw_len = 4 * elems
    raw = (np.round(np.cumsum(rng.standard_normal(elems)) * 64) / 64).astype(np.float32).tobytes()
    chunk = B.build(raw, 4, bs, B.ZSTD, (0, 0, 0, 0, 0, B.SHUFFLE), memcpyed=False, enc="lib")
    d_in = torch.from_numpy(np.frombuffer(chunk, dtype=np.uint8).copy()).cuda()
    d_out = torch.empty(nb * raw_len, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(nb, dtype=torch.int64, device="cuda")
    d_err = torch.zeros(nb, dtype=torch.int32, device="cuda")

    def run(k):
        ws.decompress_batch_device("blosc2", [d_in.data_ptr()] * k, [len(chunk)] * k, d_out.data_ptr(), raw_len,
                                   d_len.data_ptr(), d_err.data_ptr(), None)

    def timed(k, reps):
        run(k)
        torch.cuda.synchronize()
        assert int(d_err[:k].abs().sum()) == 0 and d_out[:raw_len].cpu().numpy().tobytes() == raw
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run(k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    lone_ms = timed(1, 5)
    rows = raw_len // bs * 4
    run(1)
    torch.cuda.synchronize()
    buf = (C.c_uint64 * (rows * K))()
    assert lib.rdx_probe_zprof_read(buf, rows * K) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(rows, K).astype(np.float64)
    print(json.dumps({"case": "lone", "block": bs, "chunk_bytes": len(chunk), "lone_ms": round(lone_ms, 3),
                      "rows": rows, "max_row_cycles": int(a[:, 0].max())}), flush=True)
    order = np.argsort(-a[:, 0])
    for r in list(order[:4]) + list(order[rows // 2:rows // 2 + 2]):
        print(json.dumps({"case": "row", "row": int(r), **{nm: int(a[r, k]) for k, nm in enumerate(NAMES)}}), flush=True)
    for plane in range(4):
        sel = a[np.arange(rows) % 4 == plane]
        rec = {"case": "plane", "plane": plane}
        for k, nm in enumerate(NAMES):
            rec[nm + "_mean"] = round(float(sel[:, k].mean()), 1)
        rec["max_total"] = int(sel[:, 0].max())
        rec["cyc_per_seq"] = round(float(sel[:, 3].sum() / max(1.0, sel[:, 6].sum())), 1)
        rec["cyc_per_lit_byte_section"] = round(float(sel[:, 1].sum() / max(1.0, sel[:, 8].sum())), 2)
        print(json.dumps(rec), flush=True)
    batch_ms = timed(nb, 3)
    print(json.dumps({"case": "batch", "chunks": nb, "ms": round(batch_ms, 3),
                      "GBs": round(nb * raw_len / batch_ms / 1e6, 2)}), flush=True)
    ws.close()
    eng.close()


if __name__ == "__main__":
    main()
