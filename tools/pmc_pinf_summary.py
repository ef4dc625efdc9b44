"""Per-kernel means of the counters tools/gpu_r06_pinf_pmc.sh collected (k_pinf_* only), with per-wave ratios.
Usage: python tools/pmc_pinf_summary.py gpurun_out/r06pinfpmc"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
for f in sorted(root.glob("*/run_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_pinf_" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("k_pinf_")[1].split("(")[0]
        per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        vals[k][c].append(v)
out = {}
for k, cs in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    w = m.get("SQ_WAVES", 0) or 1
    d = {c: round(v) for c, v in sorted(m.items())}
    d["per_wave"] = {c.replace("SQ_", ""): round(m[c] / w, 1) for c in
                     ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_VMEM_RD", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if c in m}
    out[k] = d
print(json.dumps(out, indent=1))
