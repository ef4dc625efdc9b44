"""Lone-stream inflate timing (k_pinflate vs k_inflate vs one host core's zlib) on the bench's chunk kinds.
Prints one JSON line per case.  Usage: python tools/probe_pinflate.py [reps]"""
import json
import sys
import time
import zlib
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from reductionist_amd import Engine  # noqa: E402


def chunks():
    rng = np.random.default_rng(0x5EED2000)
    v = rng.standard_normal(1 << 20).astype(np.float32)
    yield "c4_shuffled_normal_f32", v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
    yield "int_valued_f32", np.random.default_rng(3).integers(-8, 9, 1 << 20).astype(np.float32).tobytes()
    yield "periodic_f32", (np.arange(1 << 20) % 1000).astype(np.float32).tobytes()


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eng = Engine([0])
    ws = eng.workspace(0)
    for name, raw in chunks():
        for level in (1, 6):
            c = zlib.compressobj(level, zlib.DEFLATED, 15)
            s = c.compress(raw) + c.flush()
            d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
            d_out = torch.empty(len(raw) + 16, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            err, n, path = ws.decompress_one_device("zlib", d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
            ok = err == 0 and n == len(raw) and d_out[:n].cpu().numpy().tobytes() == raw
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                ws.decompress_one_device("zlib", d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
                ts.append(time.perf_counter() - t0)
            # one host core, CPython's zlib (the C library)
            hs = []
            for _ in range(5):
                t0 = time.perf_counter()
                zlib.decompress(s)
                hs.append(time.perf_counter() - t0)
            print(json.dumps({"chunk": name, "level": level, "ratio": round(len(raw) / len(s), 3), "ok": ok,
                              "path": path, "device_ms_median": round(1e3 * float(np.median(ts)), 3),
                              "device_ms_min": round(1e3 * min(ts), 3), "host_zlib_1core_ms": round(1e3 * float(np.median(hs)), 3),
                              "device_GBs": round(len(raw) / float(np.median(ts)) / 1e9, 2)}), flush=True)
    ws.close()
    eng.close()


if __name__ == "__main__":
    main()
