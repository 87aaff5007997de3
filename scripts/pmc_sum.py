"""Per-kernel mean of every PMC counter in rocprofv3 --pmc output directories (counter_collection.csv):
usage: python scripts/pmc_sum.py <kernel-name regex> <dir> [<dir> ...]; prints one line per directory and
counter (mean over the dispatches of the matching kernel)."""
import collections
import csv
import glob
import os
import re
import sys


def summarize(pattern, d):
    vals = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if re.search(pattern, r["Kernel_Name"]):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in sorted(vals.items())}


def main():
    pattern = sys.argv[1]
    for d in sys.argv[2:]:
        for k, (m, n) in summarize(pattern, d).items():
            print(f"{os.path.basename(d.rstrip('/')):12s} {k:26s} {m:16.1f}  (n={n})")


if __name__ == "__main__":
    main()
