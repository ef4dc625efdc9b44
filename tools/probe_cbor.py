#!/usr/bin/env python3
"""bench.py's cbor_response leg alone (device CBOR packing of 32 Mi counts), for RDX_CBOR_BLOCKS_PER_CU
sweeps: prints {"bpcu": ..., "r": leg}."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import bench  # noqa: E402


class _A:
    steps = 1


cx = bench.Ctx(torch, dist, _A(), 1, 0, 0)
print(json.dumps({"bpcu": os.environ.get("RDX_CBOR_BLOCKS_PER_CU", "default"), "staged": os.environ.get("RDX_CBOR_STAGED", "1"),
                  "r": bench.leg_cbor(cx, False)}), flush=True)
