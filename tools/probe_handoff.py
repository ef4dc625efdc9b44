#!/usr/bin/env python3
"""A/B probe of the cross-workgroup hand-off (rdx_device.hpp handoff_release / handoff_acquire) on the
launches it sits in: device time per launch (HIP events around K back-to-back launches on one stream,
rotating buffers larger than the 256 MiB Infinity Cache) for the single-chunk C2 launch, the batched C2
launch, C1, C3 min, and the sliced axis kernels.  Library from RDX_LIB_PATH (a variant build).
Prints one JSON object per case."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

PEAK = 8000.0
eng = Engine([0])
ws = eng.workspace(0)
lib = _abi.lib()
stream = torch.cuda.current_stream()
SH = C.c_void_p(stream.cuda_stream)
TAG = os.path.basename(os.environ.get("RDX_LIB_PATH", "librdx.so"))


def timed(launch, n, k):
    for i in range(max(5, n)):
        launch(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(k):
        launch(i)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / k


def single(name, creq, bufs, nbytes, alg, k=400):
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, nbytes, C.byref(info)) == 0
    body = torch.zeros(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(max(2, info.n_counts), dtype=torch.int64, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    args = [(ws.ws, creq.ref, C.c_void_p(b.data_ptr()), nbytes, C.c_void_p(body.data_ptr()),
             C.c_void_p(counts.data_ptr()), C.c_void_p(status.data_ptr()), SH, C.byref(info)) for b in bufs]

    def launch(i):
        assert lib.rdx_execute_device(*args[i % len(args)]) == 0

    t = timed(launch, len(bufs), k)
    assert int(status.abs().sum()) == 0
    print(json.dumps({"lib": TAG, "case": name, "us": round(t * 1e6, 3), "frac": round(alg / t / 1e9 / PEAK, 4)}),
          flush=True)


def batch(name, creq, bufs, nbytes, alg, k=100):
    n = len(bufs)
    body = torch.zeros(n, dtype=torch.float64, device="cuda")
    counts = torch.zeros(n, dtype=torch.int64, device="cuda")
    status = torch.zeros(n, dtype=torch.int32, device="cuda")
    ptrs = [b.data_ptr() for b in bufs]

    def launch(i):
        ws.execute_batch_device(creq, ptrs, nbytes, body.data_ptr(), counts.data_ptr(), status.data_ptr(),
                                stream.cuda_stream)

    t = timed(launch, 1, k)
    print(json.dumps({"lib": TAG, "case": name, "us": round(t * 1e6, 3), "frac": round(n * alg / t / 1e9 / PEAK, 4)}),
          flush=True)


def main():
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    # C2: 8 x 64 MiB f32, big-endian, shuffle es=4
    c2 = [torch.randint(0, 255, (64 << 20,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(8)]
    r2 = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
    single("c2_single", r2, c2, 64 << 20, 64 << 20)
    batch("c2_batch8", r2, c2, 64 << 20, 64 << 20)
    # C1: 64 x 4 MiB f32 plain sum
    c1 = [torch.rand(1 << 20, device="cuda", generator=g) for _ in range(64)]
    single("c1", _abi.CRequest("sum", "float32"), c1, 4 << 20, 4 << 20, k=1000)
    # C3: 20 x 16 MiB f64 [128,128,128], selection, missing_value, min
    c3 = [torch.randn(128 ** 3, dtype=torch.float64, device="cuda", generator=g) * 100 for _ in range(20)]
    mv = (-9999.0).hex()
    import struct
    r3 = _abi.CRequest("min", "float64", shape=[128, 128, 128], selection=[[8, 120, 1], [0, 128, 2], [16, 112, 1]],
                       missing_kind="missing_value", missing_values=struct.pack("<d", -9999.0), n_missing=1)
    single("c3_min", r3, c3, 16 << 20, 688128 * 8, k=1000)
    del c3
    # axis reductions over 64 MiB f32 [4096,4096] (cols sliced, in-kernel fold) and [128,128,128] f64
    # axes (0,2) max (rows sliced)
    a0 = [torch.rand(4096 * 4096, device="cuda", generator=g) for _ in range(6)]
    single("axis0_4096sq_sum", _abi.CRequest("sum", "float32", shape=[4096, 4096], axis=0), a0, 64 << 20, 64 << 20,
           k=200)
    single("axis1_64x1024x256_sum", _abi.CRequest("sum", "float32", shape=[64, 1024, 256], axis=1), a0, 64 << 20,
           64 << 20, k=200)
    del a0
    a2 = [torch.randn(128 ** 3, dtype=torch.float64, device="cuda", generator=g) for _ in range(20)]
    single("axes02_128cube_max", _abi.CRequest("max", "float64", shape=[128, 128, 128], axis=[0, 2]), a2, 16 << 20,
           16 << 20, k=400)
    single("select_missing_16mib", _abi.CRequest("select", "float64", shape=[128, 128, 128],
                                                   missing_kind="missing_value",
                                                   missing_values=struct.pack("<d", 0.5), n_missing=1),
           a2, 16 << 20, 32 << 20, k=400)
    ws.close()
    eng.close()


if __name__ == "__main__":
    main()
