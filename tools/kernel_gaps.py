"""Per-dispatch durations and the idle gaps between consecutive dispatches of one kernel from a rocprofv3
kernel trace (CSV): shows whether back-to-back calls are kernel-bound or pay per-call overhead between
kernels (the gated section of bench.py's mixed leg queues every call before the device starts).
usage: python tools/kernel_gaps.py <run_kernel_trace.csv> <kernel substring> [out.json]"""
import csv
import json
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
gap = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3 for i in range(len(rows) - 1)]
# gaps inside runs of queued calls (the host-side pauses between the probe's phases are > 1 ms)
queued = [g for g in gap if g < 1000.0]
out = {"kernel": sys.argv[2], "dispatches": len(rows), "us_median": round(statistics.median(dur), 3),
       "us_min": round(min(dur), 3), "gap_us_median_queued": round(statistics.median(queued), 3) if queued else None,
       "gap_us_max_queued": round(max(queued), 3) if queued else None,
       "vgpr": rows[0].get("VGPR_Count"), "sgpr": rows[0].get("SGPR_Count"), "scratch": rows[0].get("Scratch_Size"),
       "grid": rows[0].get("Grid_Size_X"), "durations_us": [round(x, 2) for x in dur], "gaps_us": [round(x, 2) for x in gap]}
s = json.dumps(out)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(s + "\n")
print(s)
