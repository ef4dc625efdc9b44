#!/usr/bin/env python3
"""Randomised parity stress (GPU box): larger hyperslabs than tests/test_gpu_parity.py's random
differential (up to ~3 M elements, long rows and columns that take the sliced / row-batch / column
paths), every dtype, op, selection, order, byte order, filter and missing form, engine vs oracle.
Prints one JSON summary line; exits 1 on the first mismatch (with the failing request)."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402

from helpers import NP, encode_filters, random_case  # noqa: E402
from oracle import py_oracle as oracle  # noqa: E402
from reductionist_amd import Engine  # noqa: E402
from test_gpu_parity import assert_parity  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cases", type=int, default=2000)
ap.add_argument("--seed", type=int, default=77)
args = ap.parse_args()

eng = Engine()
rng = np.random.default_rng(args.seed)
done = skipped = 0
for i in range(args.cases):
    kind = rng.random()
    if kind < 0.4:
        op, req, raw = random_case(rng, max_dim=64, max_ndim=3, allow_nan=True)
    elif kind < 0.7:   # long rows / columns: sliced rows, row batch, cols tiles
        op, req, raw = random_case(rng, max_dim=6, max_ndim=2, allow_nan=True)
        dtype = req["dtype"]
        long = int(rng.integers(2000, 70000))
        short = int(rng.integers(1, 40))
        shape = [short, long] if rng.random() < 0.5 else [long, short]
        n = shape[0] * shape[1]
        esz = np.dtype(NP[dtype]).itemsize
        req = {k: v for k, v in req.items() if k not in ("shape", "selection", "axis", "order", "filters")}
        req["shape"] = shape
        req["axis"] = int(rng.integers(0, 2)) if rng.random() < 0.8 else [0, 1]
        if rng.random() < 0.3:
            req["order"] = "F"
        if rng.random() < 0.3:
            req["selection"] = [[int(rng.integers(0, 2)), shape[0], 1], [int(rng.integers(0, 5)), shape[1], 1]]
        # float sums stay exactly summable in f32 (every partial sum an integer below 2^24), so the
        # reference's f32 accumulation and the engine's f64 one must agree bit for bit
        v = rng.integers(-2, 3, n) if dtype.startswith("float") else rng.integers(-100, 100, n)
        raw = (np.abs(v) if dtype.startswith("u") else v).astype(NP[dtype]).tobytes()
        if rng.random() < 0.3:
            req["filters"] = [{"id": "shuffle", "element_size": esz}]
        assert len(raw) == n * esz
    else:             # mid-size 3-D with selections
        op, req, raw = random_case(rng, max_dim=40, max_ndim=3, allow_nan=True)
    if op == "sum" and req["dtype"].startswith("float") and req.get("byte_order") == "big" and len(raw) > 4096:
        # byte-swapped small integers are denormals: no longer exactly summable once the total leaves
        # the denormal range, so the reference's f32 accumulation and the engine's f64 one (which
        # rounds the exact sum once) differ; that bar is the tolerance test in test_gpu_parity.py
        skipped += 1
        continue
    data = encode_filters(raw, req.get("filters"), oracle.shuffle)
    try:
        assert_parity(eng, op, req, data)
    except ValueError:
        skipped += 1
        continue
    except AssertionError as e:
        print(json.dumps({"status": "MISMATCH", "case": i, "op": op, "request": req, "error": str(e)[:500]}))
        sys.exit(1)
    done += 1
    if (i + 1) % 500 == 0:
        print(json.dumps({"progress": i + 1}), flush=True)
print(json.dumps({"status": "ok", "cases": done, "skipped": skipped, "seed": args.seed}))
