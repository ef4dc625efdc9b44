"""Tuning sweep for the C2 hot kernel: workgroups per CU x tiles in flight, one process."""
import ctypes as C
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
from bench import N_BUF, C2_ELEMS, C2_BYTES, shuffled_be_f32  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

eng = Engine([0])
ws = eng.workspace(0)
lib = _abi.lib()
stream = torch.cuda.current_stream()
g = torch.Generator(device="cuda")
g.manual_seed(1)
chunks = shuffled_be_f32(torch, torch.rand(N_BUF, C2_ELEMS, device="cuda", generator=g))
bodies = torch.zeros(N_BUF, dtype=torch.float32, device="cuda")
counts = torch.zeros(N_BUF, dtype=torch.int64, device="cuda")
variants = {
    "c2_f32_sum_shuffle_be": _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}]),
    "plain_f32_sum": _abi.CRequest("sum", "float32"),
    "plain_f32_max": _abi.CRequest("max", "float32"),
}
info = _abi.rdx_response_info()
configs = [(bpc, u) for bpc in (1, 2, 3, 4, 8) for u in (2, 4)]
for name, creq in variants.items():
    print(f"== {name}")
    for bpc, u in configs:
        os.environ["RDX_BLOCKS_PER_CU"] = str(bpc)
        os.environ["RDX_UNROLL"] = str(u)
        argv = [(ws.ws, creq.ref, C.c_void_p(chunks[i].data_ptr()), C2_BYTES, C.c_void_p(bodies[i:].data_ptr()),
                 C.c_void_p(counts[i:].data_ptr()), None, C.c_void_p(stream.cuda_stream), C.byref(info))
                for i in range(N_BUF)]
        for i in range(16):
            lib.rdx_execute_device(*argv[i % N_BUF])
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(64)]
        for i, (a, b) in enumerate(evs):
            a.record(stream)
            lib.rdx_execute_device(*argv[i % N_BUF])
            b.record(stream)
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in evs]
        med = statistics.median(ms) * 1e-3
        print(f"  blocks/CU={bpc} unroll={u}: median {med*1e6:7.2f} us  {C2_BYTES/med/1e9:7.1f} GB/s "
              f"({C2_BYTES/med/1e9/8000:.3f} of 8 TB/s)", flush=True)
