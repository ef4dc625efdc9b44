#!/usr/bin/env python3
"""Probe of the heterogeneous batch (rdx_execute_multi_device) on bench.py's mixed C1/C3 leg: prints the
leg's JSON (run under rocprofv3 --kernel-trace --memory-copy-trace to split table upload vs kernel)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "reductionist-rs_amd"), str(ROOT)]
import torch  # noqa: E402
import bench  # noqa: E402


class A:
    steps = 10


def main():
    import torch.distributed as dist
    cx = bench.Ctx(torch, dist, A(), 1, 0, 0)
    print(json.dumps(bench.leg_mixed(cx, k=int(sys.argv[1]) if len(sys.argv) > 1 else 30)), flush=True)


if __name__ == "__main__":
    main()
