#!/usr/bin/env python3
"""Kernel-trace summary (rocprofv3 --kernel-trace csv): per kernel name the count / mean / median duration,
and for the whole trace the device-busy fraction (union of kernel intervals over the span) and the gaps
between consecutive kernels.  Usage: trace_busy.py run_kernel_trace.csv [name-substring]"""
import csv
import json
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows if sub in r["Kernel_Name"]))
durs = [(e - s) / 1e3 for s, e, _ in ks]
iv, busy = [], 0
cs, ce = ks[0][0], ks[0][1]
gaps = []
for s, e, _ in ks[1:]:
    if s > ce:
        busy += ce - cs
        gaps.append((s - ce) / 1e3)
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
span = (ks[-1][1] - ks[0][0]) / 1e3
print(json.dumps({"kernels": len(ks), "mean_us": round(statistics.mean(durs), 3), "median_us": round(statistics.median(durs), 3),
                  "span_us": round(span, 1), "busy_frac": round(busy / 1e3 / span, 4),
                  "gap_median_us": round(statistics.median(gaps), 3) if gaps else 0,
                  "gap_mean_us": round(statistics.mean(gaps), 3) if gaps else 0}))
