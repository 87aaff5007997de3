"""Per-pass durations of the FFT kernels in a rocprofv3 kernel trace directory (scripts/fft_probe.py runs):
usage: python scripts/fft_passes.py <dir> [<dir> ...]  (the last 8 launches)
       python scripts/fft_passes.py --chunks K <dir>  (scripts/fft_modes_probe.py runs: launches split into
       consecutive chunks of K, one per mode; median duration of each pass position in the chunk)"""
import csv
import glob
import os
import re
import statistics
import sys


def launches(d):
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if "fft" in r["Kernel_Name"]:
                m = re.search(r"(fft_\w+_kernel)", r["Kernel_Name"])
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), m.group(1)))
    rows.sort()
    return rows


args = sys.argv[1:]
if args and args[0] == "--chunks":
    k, d = int(args[1]), args[2]
    rows = [r for r in launches(d) if "twiddle" not in r[2]]
    per = int(args[3]) if len(args) > 3 else 2  # launches per apply
    for c in range(len(rows) // k):
        ch = rows[c * k:(c + 1) * k]
        meds = [statistics.median(dur for _, dur, _ in ch[j::per]) / 1e3 for j in range(per)]
        print(f"chunk {c}: " + " ".join(f"{v:.1f}" for v in meds) + f" us  ({ch[0][2]})")
else:
    for d in args:
        rows = launches(d)
        print(d, " ".join(f"{dur / 1e3:.1f}" for _, dur, _ in rows[-8:]), rows[-1][2] if rows else "")
