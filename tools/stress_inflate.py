#!/usr/bin/env python3
"""Device inflate stress (GPU box): batches of random gzip / zlib streams (the payload kinds, levels
and strategies of tests/test_inflate_cpu.py, sizes up to 600 KB, unaligned starts), decoded in one
launch each and compared byte for byte with the original data.  Prints one JSON summary line; exits
1 on the first mismatch."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from reductionist_amd import Engine  # noqa: E402
from test_gpu_inflate import GZIP, ZLIB, device_decompress  # noqa: E402
from test_inflate_cpu import STRATEGIES, gz, payload, zl  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, default=6)
ap.add_argument("--streams", type=int, default=256)
ap.add_argument("--seed", type=int, default=5)
args = ap.parse_args()

eng = Engine([0])
ws = eng.workspace(0)
rng = np.random.default_rng(args.seed)
total = 0
for bi in range(args.batches):
    comp = GZIP if bi % 2 == 0 else ZLIB
    datas, streams = [], []
    for t in range(args.streams):
        b = payload(rng, int(rng.integers(0, 4)), int(rng.integers(0, 600000)))
        streams.append((gz if comp == GZIP else zl)(b, int(rng.integers(0, 10)), STRATEGIES[int(rng.integers(0, 5))]))
        datas.append(b)
    cap = (max(len(d) for d in datas) + 16 + 15) // 16 * 16
    res = device_decompress(torch, ws, comp, streams, cap, skew=int(rng.integers(0, 4)))
    for i, (e, out) in enumerate(res):
        if e != 0 or out != datas[i]:
            print(json.dumps({"status": "MISMATCH", "batch": bi, "stream": i, "err": e, "len": len(datas[i])}))
            sys.exit(1)
    total += len(res)
    print(json.dumps({"progress": total}), flush=True)
ws.close()
print(json.dumps({"status": "ok", "streams": total, "seed": args.seed}))
