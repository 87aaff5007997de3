"""Median duration per (kernel, LDS size) in launch order from a rocprofv3 kernel trace directory."""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
d = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    key = (r["Kernel_Name"][:70], r.get("LDS_Block_Size", r.get("Lds_Size", "")), r.get("Grid_Size", ""))
    d.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in d.items():
    v = sorted(v)
    print(f"{v[len(v) // 2]:>8} ns  x{len(v):<4} {k}")
