#!/usr/bin/env python3
"""Summarise tools/gpu_r06_axis_pmc.sh's passes for k_axis_cols / k_axis_rows: per-dispatch averages of every
counter, the trace's average duration, and derived figures (gfx950: SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles summed over waves; FETCH_SIZE reads half the bytes of wide streaming reads,
WRITE_SIZE exact; both KiB).  usage: python tools/pmc_axis_summary.py <dir> <out.json>"""
import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

KERNELS = ("k_axis_cols_fold", "k_axis_cols", "k_axis_rows")


def kname(n):
    for k in KERNELS:
        if k + "<" in n or n.startswith(k) or (" " + k) in n:
            return k
    return None


def counters(path):
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            out[k][c].append(v)
    return {k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in out.items()}


def durations(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: statistics.mean(v) for k, v in d.items()}


def main():
    base = Path(sys.argv[1])
    res = {"what": "k_axis_cols (f32 [4096,4096] axis 0 sum) and k_axis_rows (axis 1), tools/pmc_axis.py; one "
                   "rocprofv3 --pmc pass per counter group", "kernels": {}}
    dur = durations(base / "trace" / "run_kernel_trace.csv")
    merged = defaultdict(dict)
    for p in ("sq1", "sq2", "fetch", "write"):
        f = base / p / "run_counter_collection.csv"
        if f.exists():
            for k, cs in counters(f).items():
                merged[k].update(cs)
    for k in KERNELS:
        if k not in merged and k not in dur:
            continue
        c = merged.get(k, {})
        e = {"trace_us": round(dur.get(k, float("nan")), 3), "counters": {n: round(v, 1) for n, v in sorted(c.items())}}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM"):
                if n in c:
                    e["frac_of_wave_cycles_" + n[3:].lower()] = round(c[n] / wc, 3)
        if "GRBM_GUI_ACTIVE" in c and k in dur:
            clk_ghz = c["GRBM_GUI_ACTIVE"] / 8 / (dur[k] * 1e3)
            e["effective_clock_ghz"] = round(clk_ghz, 3)
            if wc:   # average resident waves per CU over the kernel: wave-cycles (quad) x 4 / kernel cycles / 256 CUs
                e["avg_waves_per_cu"] = round(wc * 4 / (dur[k] * 1e3 * clk_ghz) / 256, 2)
        if "SQ_WAVES" in c:
            e["waves"] = int(c["SQ_WAVES"])
        if "FETCH_SIZE" in c:
            e["hbm_read_bytes"] = int(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            e["hbm_write_bytes"] = int(c["WRITE_SIZE"] * 1024)
        res["kernels"][k] = e
    Path(sys.argv[2]).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
