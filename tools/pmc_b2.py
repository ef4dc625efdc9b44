#!/usr/bin/env python3
"""Round 6: the blosc2 LZ4 batch decode alone (bench.py leg_blosc2's lz4 chunks: 4 MiB f32 random walk quantised
to 1/64, SHUFFLE, 64 KiB blocks x 4 streams, this repo's writer), K launches of 256 chunks, for rocprofv3 --pmc
passes of issue / stall counters (tools/gpu_r06_b2_pmc.sh).  usage: python tools/pmc_b2.py [K]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from datagen import blosc2_chunk as B  # noqa: E402
from reductionist_amd import Engine  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n, distinct, elems = 256, 8, 1 << 20
eng = Engine([0])
ws = eng.workspace(0)
stream = torch.cuda.current_stream()
rng = np.random.default_rng(0x5EED2100)
raws = [(np.round(np.cumsum(rng.standard_normal(elems)) * 64) / 64).astype(np.float32).tobytes() for _ in range(distinct)]
chunks = [B.build(r, 4, 1 << 16, B.LZ4, (0, 0, 0, 0, 0, B.SHUFFLE), memcpyed=False, enc="repo") for r in raws]
offs, total = [], 0
for c in chunks:
    offs.append(total)
    total += (len(c) + 255) // 256 * 256
host = np.zeros(total, dtype=np.uint8)
for o, c in zip(offs, chunks):
    host[o:o + len(c)] = np.frombuffer(c, dtype=np.uint8)
d_in = torch.from_numpy(host).cuda()
raw_len = 4 * elems
d_out = torch.empty(n * raw_len, dtype=torch.uint8, device="cuda")
d_len = torch.zeros(n, dtype=torch.int64, device="cuda")
d_err = torch.zeros(n, dtype=torch.int32, device="cuda")
ptrs = [d_in.data_ptr() + offs[i % distinct] for i in range(n)]
lens = [len(chunks[i % distinct]) for i in range(n)]
for _ in range(K + 1):
    ws.decompress_batch_device("blosc2", ptrs, lens, d_out.data_ptr(), raw_len, d_len.data_ptr(), d_err.data_ptr(),
                               stream.cuda_stream)
torch.cuda.synchronize()
assert int(d_err.abs().sum()) == 0 and bool((d_len == raw_len).all())
assert d_out[:raw_len].cpu().numpy().tobytes() == raws[0]
print("pmc_b2: done", flush=True)
