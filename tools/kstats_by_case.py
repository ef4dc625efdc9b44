#!/usr/bin/env python3
"""Median kernel duration per kernel name between marker kernels (tools/probe_multi_kernel.py) from a
rocprofv3 results .db."""
import sqlite3
import statistics
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, grid_x from kernels order by start").fetchall()
case, out = None, {}
for name, s, e, gx in rows:
    if "elementwise" in name or "fill" in name.lower():
        case = gx
        continue
    short = name.replace("rdx::(anonymous namespace)::", "")[:60]
    out.setdefault((case, short), []).append((e - s) / 1e3)
for (case, name), ds in sorted(out.items(), key=lambda kv: (str(kv[0][0]), kv[0][1])):
    print(f"{str(case):>8} {name:60s} n={len(ds):3d} median {statistics.median(ds):8.2f} us")
