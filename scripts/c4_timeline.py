"""Device timeline of the C4 ADMM run (bench.py --only c4 under rocprofv3 --kernel-trace): per-kernel time
per CG iteration and the idle gaps between consecutive kernels, over the timed outer iterations.

usage: python scripts/c4_timeline.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    rows = []
    for fn in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:40]))
    rows.sort()
    # the timed window: from the 2nd-to-last run of normal_rows_kernel launches of the warm-up onwards; take
    # the last 4 outer iterations' worth: the last 60% of normal_rows launches
    idx = [i for i, r in enumerate(rows) if r[2] in ("normal_rows_kernel", "normal_group_kernel")]
    if not idx:
        raise SystemExit("no normal_rows_kernel / normal_group_kernel")
    lo = idx[int(len(idx) * 0.4)]
    win = rows[lo:]
    n_cg = sum(1 for r in win if r[2] in ("normal_rows_kernel", "normal_group_kernel"))
    busy = collections.Counter()
    cnt = collections.Counter()
    gaps = collections.Counter()
    prev_end, prev_name = win[0][1], win[0][2]
    busy[win[0][2]] += win[0][1] - win[0][0]
    cnt[win[0][2]] += 1
    for s, e, n in win[1:]:
        busy[n] += e - s
        cnt[n] += 1
        if s > prev_end:
            gaps[f"{prev_name} -> {n}"] += s - prev_end
        prev_end, prev_name = max(prev_end, e), n
    span = win[-1][1] - win[0][0]
    print(f"window: {span / 1e3:.1f} us, {n_cg} normal operator passes ({span / 1e3 / n_cg:.1f} us each)")
    for n, t in busy.most_common():
        print(f"  {n:32s} {t / 1e3 / n_cg:8.2f} us per pass  ({cnt[n]} launches)")
    print("  idle gaps per pass:")
    for n, t in gaps.most_common(10):
        print(f"    {n:60s} {t / 1e3 / n_cg:8.2f} us")


if __name__ == "__main__":
    main()
