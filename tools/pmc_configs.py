#!/usr/bin/env python3
"""Driver for the per-kernel rocprofv3 passes (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes):
every profiled kernel on its BASELINE configuration, K launches each over rotating buffers larger than the
Infinity Cache, one kernel family per case so a dispatch's kernel name identifies its case:

  c2_batch     k_all_contig   8 x 64 MiB f32, big-endian, shuffle es=4, sum          (512 MiB read)
  c3_min       k_all_strided  f64 [128,128,128] hyperslab, missing_value, min        (5.5 MB read)
  c5_select    k_map          i64 [512,256,256] select -> 128 MiB                    (128 MiB read + written)
  axis0_cols   k_axis_cols    f32 [4096,4096] axis 0 sum                             (64 MiB read)
  axis1_rows   k_axis_rows    f32 [4096,4096] axis 1 sum                             (64 MiB read)
  mixed_multi  k_multi        10 x C1 + 10 x C3 requests in one launch               (97 MB read)
  cbor_counts  k_cbor_pack + k_cbor_place  32 Mi counts (0/1) -> CBOR integers, no body (256 MiB read, 32 MiB written)

tools/pmc_traffic.py turns the counter CSVs into profiles/r02_pmc_<case>.json."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
eng = Engine([0])
ws = eng.workspace(0)
lib = _abi.lib()
stream = torch.cuda.current_stream()
SH = C.c_void_p(stream.cuda_stream)
g = torch.Generator(device="cuda")
g.manual_seed(3)


def single(creq, bufs, nbytes, k=K):
    info = _abi.rdx_response_info()
    assert lib.rdx_plan(creq.ref, nbytes, C.byref(info)) == 0
    body = torch.zeros(max(16, info.body_bytes), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(max(2, info.n_counts), dtype=torch.int64, device="cuda")
    status = torch.zeros(4, dtype=torch.int32, device="cuda")
    for i in range(k + len(bufs)):
        assert lib.rdx_execute_device(ws.ws, creq.ref, C.c_void_p(bufs[i % len(bufs)].data_ptr()), nbytes,
                                      C.c_void_p(body.data_ptr()), C.c_void_p(counts.data_ptr()),
                                      C.c_void_p(status.data_ptr()), SH, C.byref(info)) == 0
    torch.cuda.synchronize()


# c2_batch
c2 = [torch.randint(0, 255, (64 << 20,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(8)]
r2 = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
out = torch.zeros(8, dtype=torch.float64, device="cuda")
cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
st = torch.zeros(8, dtype=torch.int32, device="cuda")
for _ in range(K + 1):
    ws.execute_batch_device(r2, [b.data_ptr() for b in c2], 64 << 20, out.data_ptr(), cnt.data_ptr(), st.data_ptr(),
                            stream.cuda_stream)
torch.cuda.synchronize()
del c2
# c3_min
v3 = bench._c3_host()
single(bench._c3_req(_abi, "min"), [torch.from_numpy(v3).cuda() for _ in range(20)], 16 << 20)
# c5_select
c5 = [torch.randint(-2 ** 62, 2 ** 62, (512 * 256 * 256,), dtype=torch.int64, device="cuda", generator=g)
      for _ in range(2)]
single(_abi.CRequest("select", "int64", shape=[512, 256, 256], selection=bench.C5_SEL), c5, 256 << 20)
del c5
# axis kernels
a = [torch.rand(4096 * 4096, device="cuda", generator=g) for _ in range(6)]
single(_abi.CRequest("sum", "float32", shape=[4096, 4096], axis=0), a, 64 << 20)
single(_abi.CRequest("sum", "float32", shape=[4096, 4096], axis=1), a, 64 << 20)
del a


# cbor_counts: the count-array kernel alone (a body-less response layout)
n = 512 * 256 * 256
cts = torch.randint(0, 2, (n,), dtype=torch.int64, device="cuda", generator=g)
info = _abi.rdx_response_info()
info.dtype, info.ndim, info.shape[0], info.body_bytes, info.n_counts = _abi.DTYPES["int64"], 1, n, 0, n
bound = lib.rdx_cbor_bound(C.byref(info), 0)
dst = torch.empty(bound, dtype=torch.uint8, device="cuda")
dlen = torch.zeros(1, dtype=torch.int64, device="cuda")
for _ in range(K + 1):
    assert lib.rdx_cbor_encode_device(ws.ws, C.byref(info), None, C.c_void_p(cts.data_ptr()), 0,
                                      C.c_void_p(dst.data_ptr()), bound, C.c_void_p(dlen.data_ptr()), None, SH) == 0
torch.cuda.synchronize()
del cts, dst


# mixed_multi (bench.leg_mixed's requests)
class _A:
    steps = 1


import torch.distributed as dist  # noqa: E402
cx = bench.Ctx(torch, dist, _A(), 1, 0, 0)
bench.leg_mixed(cx, k=K, serial=False)
torch.cuda.synchronize()
print("pmc_configs: done", flush=True)
