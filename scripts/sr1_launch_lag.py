"""Development probe: for the stop_rate = 1 PGD run traced with rocprofv3 --kernel-trace --hip-runtime-trace, the
lag between each kernel's launch call (host, hipLaunchKernel / hipModuleLaunchKernel returning) and the kernel's
start on the device, and the device idle before each PGD kernel: whether the device waits for the host.

usage: python scripts/sr1_launch_lag.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
kern, api = {}, {}
for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(fn)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        kern[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else "?")
for fn in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
    for r in csv.DictReader(open(fn)):
        if "Launch" in r["Function"]:
            api[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
ks = sorted((v[0], v[1], v[2], c) for c, v in kern.items())
pgd = [i for i, k in enumerate(ks) if k[2] == "pgd_tv2d_kernel"]
lo = pgd[-1000]
stats = collections.defaultdict(list)
for i in range(lo + 1, pgd[-1]):
    s, e, n, c = ks[i]
    prev_end = max(k[1] for k in ks[max(lo, i - 3):i])
    if c in api:
        stats[f"{n}: launch call end -> kernel start"].append(s - api[c][1])
        stats[f"{n}: launch call end -> previous kernel end"].append(prev_end - api[c][1])
    stats[f"{n}: idle before it"].append(max(0, s - prev_end))
for k, v in sorted(stats.items()):
    v = sorted(v)
    print(f"{k:58s} median {v[len(v) // 2] / 1e3:8.2f} us   p10 {v[len(v) // 10] / 1e3:8.2f}   p90 {v[9 * len(v) // 10] / 1e3:8.2f}")
