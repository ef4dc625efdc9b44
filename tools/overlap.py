#!/usr/bin/env python3
"""Kernel overlap in a rocprofv3 --kernel-trace CSV: for the k_all_contig dispatches of each queue
pattern, the mean duration, the wall time they span and the fraction of that span with >= 2 of them
running at once.  Used on the concurrent-request leg of bench.py (4 streams -> 4 hardware queues).
usage: python tools/overlap.py <run_kernel_trace.csv> [kernel substring] [legs]"""
import csv
import json
import sys

path = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "k_all_contig"
rows = [r for r in csv.DictReader(open(path)) if ksub in r["Kernel_Name"]]
groups = {}
for r in rows:
    grid = int(r["Grid_Size_X"])
    groups.setdefault(grid, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"])))
nseg = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # consecutive equal-size legs (bench.py: 3)
segs = []
for grid, ev in sorted(groups.items()):
    ev.sort()
    k = len(ev) // nseg
    segs += [(grid, i, ev[i * k:(i + 1) * k]) for i in range(nseg)]
for grid, leg, ev in segs:
    queues = sorted({q for _, _, q in ev})
    # split into runs by queue set: the concurrent leg uses several queues, the serial legs one
    pts = sorted([(s, 1) for s, _, _ in ev] + [(e, -1) for _, e, _ in ev])
    active, last, multi, busy = 0, None, 0, 0
    for t, d in pts:
        if last is not None and active >= 1:
            busy += t - last
            if active >= 2:
                multi += t - last
        active += d
        last = t
    span = ev[-1][1] - ev[0][0]
    print(json.dumps({"grid_x": grid, "leg": leg, "dispatches": len(ev), "queues": queues,
                      "mean_us": round(sum(e - s for s, e, _ in ev) / len(ev) / 1e3, 3),
                      "span_us": round(span / 1e3, 1), "busy_frac": round(busy / span, 4),
                      "overlap_frac_of_busy": round(multi / max(1, busy), 4)}))
