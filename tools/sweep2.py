"""Where does the single-chunk time go?  fixed overhead vs streaming, against torch baselines."""
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

eng = Engine([0]); ws = eng.workspace(0); lib = _abi.lib()
stream = torch.cuda.current_stream()
g = torch.Generator(device="cuda"); g.manual_seed(1)
vals = torch.rand(N_BUF, C2_ELEMS, device="cuda", generator=g)
chunks = shuffled_be_f32(torch, vals)
bodies = torch.zeros(N_BUF, dtype=torch.float32, device="cuda")
counts = torch.zeros(N_BUF, dtype=torch.int64, device="cuda")
info = _abi.rdx_response_info()


def timeit(fn, n=64):
    for i in range(8):
        fn(i)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i, (a, b) in enumerate(evs):
        a.record(stream); fn(i); b.record(stream)
    torch.cuda.synchronize()
    return statistics.median([a.elapsed_time(b) for a, b in evs]) * 1e3  # us


print("torch.sum 64 MiB f32      : %.2f us" % timeit(lambda i: vals[i % N_BUF].sum()))
dst = torch.empty_like(vals[0])
print("torch copy_ 64 MiB        : %.2f us" % timeit(lambda i: dst.copy_(vals[i % N_BUF])))
print("torch empty kernel (fill 4B): %.2f us" % timeit(lambda i: bodies[:1].fill_(1.0)))

creq = _abi.CRequest("sum", "float32", byte_order="big", filters=[{"id": "shuffle", "element_size": 4}])
plain = _abi.CRequest("sum", "float32")


def run(req, nbytes):
    def f(i):
        st = lib.rdx_execute_device(ws.ws, req.ref, C.c_void_p(chunks[i % N_BUF].data_ptr()), nbytes,
                                    C.c_void_p(bodies[i % N_BUF:].data_ptr()), C.c_void_p(counts[i % N_BUF:].data_ptr()),
                                    None, C.c_void_p(stream.cuda_stream), C.byref(info))
        assert st == 0
    return f


for bpc in (1, 8, 64, 256, 512, 1024, 2048):
    os.environ["RDX_FORCE_BPC"] = str(bpc)
    print(f"fixed overhead, 16 KiB plain sum, bpc={bpc:5d}: {timeit(run(plain, 16384)):7.2f} us")
for bpc in (128, 256, 384, 512, 768, 1024):
    os.environ["RDX_FORCE_BPC"] = str(bpc)
    t = timeit(run(creq, C2_BYTES))
    t2 = timeit(run(plain, C2_BYTES))
    print(f"C2 fused bpc={bpc:5d}: {t:7.2f} us ({C2_BYTES/t/1e3:6.0f} GB/s)   plain: {t2:7.2f} us ({C2_BYTES/t2/1e3:6.0f} GB/s)")
