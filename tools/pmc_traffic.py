"""Turn a rocprofv3 --pmc FETCH_SIZE pass into profiles/<tag>_pmc.json (HBM bytes per launch).

gfx950 calibration (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is reported in KiB and counts
exactly HALF the bytes of a wide coalesced streaming read, so hbm_read_bytes = FETCH_SIZE*1024*2.
usage: python tools/pmc_traffic.py <counter_collection.csv> <kernel substring> <tag> [bytes_alg]
"""
import csv
import json
import statistics
import sys
from pathlib import Path

path, ksub, tag = sys.argv[1], sys.argv[2], sys.argv[3]
alg = int(sys.argv[4]) if len(sys.argv) > 4 else None
rows = list(csv.DictReader(open(path)))
vals = {}
for r in rows:
    if ksub in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE":
        vals.setdefault(r.get("Dispatch_Id"), 0.0)
        vals[r.get("Dispatch_Id")] += float(r["Counter_Value"])
per = sorted(vals.values())
if not per:
    raise SystemExit(f"no FETCH_SIZE rows for {ksub!r} in {path}")
med_kib = statistics.median(per)
out = {"kernel": ksub, "dispatches": len(per), "fetch_size_kib_median": med_kib,
       "hbm_bytes_per_launch": int(med_kib * 1024 * 2), "correction": "x2 (gfx950 FETCH_SIZE = 1/2 of wide streaming reads)",
       "bytes_alg_per_launch": alg}
if alg:
    out["traffic_over_alg"] = round(out["hbm_bytes_per_launch"] / alg, 4)
dst = Path(__file__).resolve().parent.parent / "profiles" / f"{tag}_pmc.json"
dst.parent.mkdir(exist_ok=True)
dst.write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
