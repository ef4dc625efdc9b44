"""Lone-stream inflate timing: the device route (k_pinflate; a stream it declines comes back to the caller,
whose host zlib then decodes it — the plugin's route, integration/app_gpu.rs) against one host core's zlib,
for the bench's chunk kinds, Z_FIXED streams (a fixed-Huffman block per 16 K symbols: declined), corrupt
streams (declined) and a GNU gzip member.  For a declined stream also the old route: the device's
sequential k_inflate (a context with inflate_fallback).  One JSON line per case.
Usage: python tools/probe_pinflate.py [reps] [filter: substrings of "<chunk>_<format><level>", comma-separated]"""
import json
import shutil
import subprocess
import sys
import time
import zlib
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from reductionist_amd import Engine, _abi  # noqa: E402


def comp(raw, fmt, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, 31 if fmt == "gzip" else 15, 9, strategy)
    return c.compress(raw) + c.flush()


def cases():
    rng = np.random.default_rng(0x5EED2000)
    v = rng.standard_normal(1 << 20).astype(np.float32)
    shuffled = v.view(np.uint8).reshape(-1, 4).T.copy().tobytes()
    ints = np.random.default_rng(3).integers(-8, 9, 1 << 20).astype(np.float32).tobytes()
    periodic = (np.arange(1 << 20) % 1000).astype(np.float32).tobytes()
    for name, raw in (("c4_shuffled_normal_f32", shuffled), ("int_valued_f32", ints), ("periodic_f32", periodic)):
        for level in (1, 6):
            yield name, "zlib", level, raw, comp(raw, "zlib", level)
    for name, raw in (("c4_shuffled_normal_f32", shuffled), ("int_valued_f32", ints)):
        yield name + "_Z_FIXED", "zlib", 6, raw, comp(raw, "zlib", 6, zlib.Z_FIXED)
    good = bytearray(comp(ints, "gzip", 1))
    good[-6] ^= 0x40                                   # the CRC: every block decodes, the check fails
    yield "int_valued_f32_bad_crc", "gzip", 1, ints, bytes(good)
    mid = bytearray(comp(ints, "zlib", 6))
    mid[len(mid) // 2] ^= 0x10                         # a flip in the middle of a Huffman body
    yield "int_valued_f32_flip_mid", "zlib", 6, ints, bytes(mid)
    if shutil.which("gzip"):
        gz = subprocess.run(["gzip", "-c", "-n", "-6"], input=ints, capture_output=True, check=True).stdout
        yield "int_valued_f32_gnu_gzip", "gzip", 6, ints, gz


def host(fmt, s):
    try:
        return zlib.decompress(s, 31 if fmt == "gzip" else 15)
    except zlib.error:
        return None


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    keep = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    eng = Engine([0])
    ws = eng.workspace(0)
    eng_serial = Engine([0])
    eng_serial.configure(inflate_fallback=True)
    ws_serial = eng_serial.workspace(0)
    for name, fmt, level, raw, s in cases():
        if keep and not any(k in f"{name}_{fmt}{level}" for k in keep):
            continue
        d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
        d_out = torch.empty(len(raw) + 16, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        err, n, path = ws.decompress_one_device(fmt, d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
        ref = host(fmt, s)
        ok = (err == 0 and n == len(raw) and d_out[:n].cpu().numpy().tobytes() == ref) if err is not None else True
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ws.decompress_one_device(fmt, d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
            ts.append(time.perf_counter() - t0)
        hs = []
        for _ in range(5):
            t0 = time.perf_counter()
            host(fmt, s)
            hs.append(time.perf_counter() - t0)
        dev, hst = float(np.median(ts)), float(np.median(hs))
        declined = path == _abi.INFLATE_PATH_DECLINED
        route = dev + hst if declined else dev
        rec = {"chunk": name, "format": fmt, "level": level, "ratio": round(len(raw) / len(s), 3), "ok": ok,
               "host_valid": ref is not None, "path": path, "declined": declined,
               "device_ms_median": round(1e3 * dev, 3), "device_ms_min": round(1e3 * min(ts), 3),
               "host_zlib_1core_ms": round(1e3 * hst, 3), "route_ms": round(1e3 * route, 3),
               "route_over_host": round(route / hst, 3)}
        if declined:   # the old route: the sequential k_inflate on the device
            t = []
            for _ in range(2):
                t0 = time.perf_counter()
                ws_serial.decompress_one_device(fmt, d_in.data_ptr(), len(s), d_out.data_ptr(), len(raw) + 16)
                t.append(time.perf_counter() - t0)
            rec["serial_k_inflate_ms"] = round(1e3 * min(t), 3)
        print(json.dumps(rec), flush=True)
    ws.close()
    ws_serial.close()
    eng.close()
    eng_serial.close()


if __name__ == "__main__":
    main()
