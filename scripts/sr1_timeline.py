"""Device timeline of the stop_rate = 1 PGD run (rocprofv3 --kernel-trace of scripts/sr1_phases.py): kernel
durations and the idle gaps between consecutive kernels over the last 1000 steps.

usage: python scripts/sr1_timeline.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import re
import sys

rows = []
for fn in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(fn)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:40]))
rows.sort()
steps = [i for i, r in enumerate(rows) if r[2] == "pgd_tv2d_kernel"]
win = rows[steps[-1000]:steps[-1]]
busy, cnt, gaps = collections.Counter(), collections.Counter(), collections.Counter()
pe, pn = win[0][0], None
for s, e, n in win:
    busy[n] += e - s
    cnt[n] += 1
    if pn is not None and s > pe:
        gaps[f"{pn} -> {n}"] += s - pe
    pe, pn = max(pe, e), n
span = win[-1][0] - win[0][0]
print(f"{span / 1e3 / 999:.2f} us per step over 999 steps")
for n, t in busy.most_common():
    print(f"  {n:32s} {t / 1e3 / cnt[n]:8.2f} us per launch  ({cnt[n]} launches)")
for n, t in gaps.most_common(6):
    print(f"  gap {n:50s} {t / 1e3 / 999:8.2f} us per step")
