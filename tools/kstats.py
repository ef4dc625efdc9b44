"""Print the rdx kernels of a rocprofv3 kernel_stats.csv: calls, average and min duration (us)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    if "rdx" in r["Name"]:
        n = r["Name"].replace("void rdx::(anonymous namespace)::", "").split("(rdx::")[0]
        print(f"{n:60s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.2f} {float(r['MinNs']) / 1e3:9.2f}")
