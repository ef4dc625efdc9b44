"""Turn rocprofv3 --pmc passes (FETCH_SIZE in one run, WRITE_SIZE in another, both over tools/pmc_configs.py)
into per-kernel HBM traffic records: profiles/<round>_pmc_<case>.json, and profiles/c2_pmc.json (read by
bench.py's roofline.traffic for the headline kernel).

gfx950 calibration (MI355X_MICROARCH.md, HBM section): both counters are reported in KiB; FETCH_SIZE counts
exactly HALF the bytes of a wide coalesced streaming read (so read bytes = FETCH_SIZE*1024*2); WRITE_SIZE is
exact for 16-B-per-lane streaming stores (k_map's stores are 16 B per lane).
usage: python tools/pmc_traffic.py <round> <fetch counter_collection.csv> [<write counter_collection.csv>]
"""
import csv
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
C3_NSEL = 112 * 64 * 96
# kernel-name substring -> (case, algorithmic bytes read per launch, algorithmic bytes written per launch)
CASES = {
    "k_all_contig": ("c2_batch", 8 * (64 << 20), 0),
    "k_all_strided": ("c3_min", C3_NSEL * 8, 0),
    "k_map": ("c5_select", 128 << 20, 128 << 20),
    "k_axis_cols": ("axis0_cols", 64 << 20, 4096 * 4 + 4096 * 8),
    "k_axis_rows": ("axis1_rows", 64 << 20, 4096 * 4 + 4096 * 8),
    "k_multi": ("mixed_multi", 10 * ((4 << 20) + C3_NSEL * 8), 0),
    "k_cbor": ("cbor_counts", 8 * (512 * 256 * 256), 512 * 256 * 256),
    "k_cbor_agg": ("cbor_agg", 8 * (512 * 256 * 256), 0),   # (round 4: the tile lengths' pass re-reads the counts)
    # round 5's staged form: the counts read once by k_cbor_pack (the encoded bytes staged), k_cbor_place
    # moves the staged bytes to their offsets
    "k_cbor_pack": ("cbor_pack", 8 * (512 * 256 * 256), 512 * 256 * 256),
    "k_cbor_place": ("cbor_place", 512 * 256 * 256, 512 * 256 * 256),
}


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r.get("Kernel_Name", "")
        for ksub in CASES:
            if ksub + "<" in name or ksub + "(" in name:     # k_axis_cols, not k_axis_cols_fold
                key = (ksub, r.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (ksub, _), v in vals.items():
        out.setdefault(ksub, []).append(v)
    return out


def main():
    rnd, fetch = sys.argv[1], sys.argv[2]
    write = sys.argv[3] if len(sys.argv) > 3 else None
    f = per_dispatch(fetch, "FETCH_SIZE")
    w = per_dispatch(write, "WRITE_SIZE") if write else {}
    for ksub, (case, alg_r, alg_w) in CASES.items():
        if ksub not in f:
            print(f"no FETCH_SIZE rows for {ksub}", file=sys.stderr)
            continue
        # the first dispatches of each case run over cold / freshly written buffers: median over all
        rd = int(statistics.median(f[ksub]) * 1024 * 2)
        rec = {"kernel": ksub, "case": case, "dispatches": len(f[ksub]),
               "fetch_size_kib_median": statistics.median(f[ksub]), "hbm_read_bytes_per_launch": rd,
               "bytes_alg_read_per_launch": alg_r, "read_over_alg": round(rd / alg_r, 4),
               "correction": "read = FETCH_SIZE KiB x 1024 x 2 (gfx950: FETCH_SIZE = 1/2 of wide streaming reads); "
                             "write = WRITE_SIZE KiB x 1024 (exact for 16-B stores)"}
        if ksub in w:
            wr = int(statistics.median(w[ksub]) * 1024)
            rec.update({"write_size_kib_median": statistics.median(w[ksub]), "hbm_write_bytes_per_launch": wr,
                        "bytes_alg_write_per_launch": alg_w})
            if alg_w >= (1 << 20):
                rec["write_over_alg"] = round(wr / alg_w, 4)
        rec["hbm_bytes_per_launch"] = rd + rec.get("hbm_write_bytes_per_launch", 0)
        (ROOT / "profiles" / f"{rnd}_pmc_{case}.json").write_text(json.dumps(rec, indent=1) + "\n")
        if case == "c2_batch":
            (ROOT / "profiles" / "c2_pmc.json").write_text(json.dumps(rec, indent=1) + "\n")
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
