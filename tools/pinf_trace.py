"""Per-call kernel breakdown of the single-stream inflate from a rocprofv3 kernel trace (CSV).
Usage: python tools/pinf_trace.py run_kernel_trace.csv [every]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    seq = []
    for r in rows:
        n = r["Kernel_Name"]
        if "pinf" not in n:
            continue
        seq.append((re.sub(r"rdx::\(anonymous namespace\)::|\(.*", "", n),
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    calls, cur = [], []
    for s in seq:
        if s[0] == "k_pinf_find" and cur:
            calls.append(cur)
            cur = []
        cur.append(s)
    calls.append(cur)
    for i, c in enumerate(calls):
        if i % every:
            continue
        agg = {}
        for n, d in c:
            agg[n] = agg.get(n, 0) + d
        print(i, round(sum(agg.values()), 1), {k.replace("k_pinf_", ""): round(v, 1) for k, v in agg.items()})


if __name__ == "__main__":
    main()
