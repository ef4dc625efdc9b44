#!/usr/bin/env python3
"""Host-inclusive rates through rdx_execute (chunk in host memory -> H2D -> kernels -> D2H): the
path a request takes when the chunk arrives from a socket.  Pageable (a plain host buffer) vs
page-locked (rdx_host_alloc, what a downloader would write into)."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from reductionist_amd import Engine, _abi  # noqa: E402

eng = Engine([0])
lib = _abi.lib()


def host_buf(nbytes, pinned):
    if pinned:
        p = C.c_void_p()
        assert lib.rdx_host_alloc(eng.ctx, nbytes, C.byref(p)) == 0
        arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p.value))
        return p, arr
    arr = np.empty(nbytes, dtype=np.uint8)
    return C.c_void_p(arr.ctypes.data), arr


def run(name, creq, data_bytes, reps, chunk_gib):
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, len(data_bytes), C.byref(info)) == 0
    for pinned in (False, True):
        src, arr = host_buf(len(data_bytes), pinned)
        arr[:] = np.frombuffer(data_bytes, dtype=np.uint8)
        body_p, body = host_buf(max(16, info.body_bytes), pinned)
        counts = (C.c_int64 * max(1, info.n_counts))()
        out = _abi.rdx_response_info()
        for _ in range(2):
            assert lib.rdx_execute(eng.ctx, creq.ref, src, len(data_bytes), body_p, info.body_bytes, counts,
                                   info.n_counts, C.byref(out)) == 0
        t0 = time.perf_counter()
        for _ in range(reps):
            lib.rdx_execute(eng.ctx, creq.ref, src, len(data_bytes), body_p, info.body_bytes, counts, info.n_counts,
                            C.byref(out))
        t = (time.perf_counter() - t0) / reps
        print(json.dumps({"config": name, "host_memory": "pinned" if pinned else "pageable",
                          "ms_per_request": round(t * 1e3, 3), "GiBs_chunk": round(chunk_gib / t, 2),
                          "h2d_bytes": len(data_bytes), "d2h_bytes": info.body_bytes}), flush=True)
        if pinned:
            lib.rdx_host_free(eng.ctx, src)
            lib.rdx_host_free(eng.ctx, body_p)


vals = np.random.default_rng(4).random(16 << 20, dtype=np.float32)
c2 = vals.astype(">f4").view(np.uint8).reshape(-1, 4).T.copy().tobytes()
run("c2_sum_64MiB", _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}]),
    c2, 20, 64 / 1024)
c5 = np.random.default_rng(6).integers(-2 ** 62, 2 ** 62, 512 * 256 * 256, dtype=np.int64).tobytes()
run("c5_select_256MiB", _abi.CRequest("select", "int64", shape=[512, 256, 256],
                                      selection=[[0, 512, 1], [64, 192, 1], [0, 256, 1]]), c5, 5, 0.25)
v3 = np.random.default_rng(5).standard_normal(128 ** 3) * 100
run("c3_max_16MiB", _abi.CRequest("max", "float64", shape=[128, 128, 128], selection=[[8, 120, 1], [0, 128, 2], [16, 112, 1]],
                                  missing_kind="missing_value", missing_values=np.float64(-9999).tobytes(), n_missing=1),
    v3.tobytes(), 50, 16 / 1024)
eng.close()
