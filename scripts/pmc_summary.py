"""Average rocprofv3 PMC counters of one kernel over its dispatches: python scripts/pmc_summary.py <dir> [kernel-substr]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "pgd_tv2d"
acc = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
for f in glob.glob(f"{root}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Name"]:
            print("stats:", r["Name"][:60], "calls", r["Calls"], "avg_ns", r["AverageNs"])
