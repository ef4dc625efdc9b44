#!/usr/bin/env python3
"""Is the slow XCD of the headline batch launch the same from one launch to the next?  Probe build
(RDX_LIB_PATH=librdx_probe.so): 8 x 64 MiB shuffled big-endian f32 sum, one batched launch at a time, the
phase stamps of every workgroup read after each launch; prints per launch the median streaming time of each
XCD (workgroups b % 8) and the launch's streaming spread.  usage: python tools/probe_xcd_stability.py [launches]"""
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT), str(ROOT / "tools")]
os.environ.setdefault("RDX_LIB_PATH", str(ROOT / "reductionist-rs_amd" / "librdx_probe.so"))
import torch  # noqa: E402
import bench  # noqa: E402
from probe_timeline import timeline  # noqa: E402
from reductionist_amd import Engine, _abi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
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
for k in range(3):
    ws.execute_batch_device(creq, [c.data_ptr() for c in chunks], bench.C2_BYTES, out.data_ptr(), cnt.data_ptr(), None,
                            stream.cuda_stream)
torch.cuda.synchronize()
for k in range(n):
    ws.execute_batch_device(creq, [c.data_ptr() for c in chunks], bench.C2_BYTES, out.data_ptr(), cnt.data_ptr(), None,
                            stream.cuda_stream)
    torch.cuda.synchronize()
    t = timeline(lib, 256)
    by = t["stream_us_by_xcd"]
    print(json.dumps({"launch": k, "stream_us_by_xcd": by, "slowest_xcd": by.index(max(by)), "fastest_xcd": by.index(min(by)),
                      "xcd_spread_us": round(max(by) - min(by), 2), "first_stream_end_us": t["first_stream_end_us"],
                      "last_stream_end_us": t["last_stream_end_us"], "fold_end_us": t["fold_end_us"]}), flush=True)
