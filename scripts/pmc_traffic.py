"""Per-launch HBM traffic of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substr> <key> <out.json> [tag]

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of a wide coalesced
stream, WRITE_SIZE is exact, both in KiB -> hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
The two counters cannot share a pass (TCC slots), hence two directories.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(root, counter, pat):
    vals = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and r["Counter_Name"] == counter:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, pat, key, out = sys.argv[1:6]
    tag = sys.argv[6] if len(sys.argv) > 6 else ""
    fs = per_dispatch(fdir, "FETCH_SIZE", pat)
    ws = per_dispatch(wdir, "WRITE_SIZE", pat)
    if not fs or not ws:
        raise SystemExit(f"no {pat} dispatches with FETCH_SIZE/WRITE_SIZE under {fdir} / {wdir}")
    f = sum(fs) / len(fs)
    w = sum(ws) / len(ws)
    tab = {}
    if os.path.exists(out):
        tab = json.load(open(out))
    tab[key] = {"fetch_size_kib": f, "write_size_kib": w, "dispatches": [len(fs), len(ws)], "tag": tag,
                "kernel_match": pat,
                "hbm_bytes_per_launch": int((2 * f + w) * 1024),
                "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"}
    json.dump(tab, open(out, "w"), indent=1)
    print(key, tab[key])


if __name__ == "__main__":
    main()
