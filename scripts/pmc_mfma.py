"""MFMA-busy fraction of the dense LinOp's MFMA kernel from a rocprofv3 PMC pass over
`bench.py --only dense_mfma` (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE in one pass).

usage: python scripts/pmc_mfma.py <pmc dir> <out.json> [tag]

  mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
    (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES counts 64 cycles per
    v_mfma_f32_32x32x2_f32, which the count of MFMAs in the GEMM, 2 M N B / 4096, confirms);
  clock_ghz = GRBM_GUI_ACTIVE / 8 / kernel duration (the clock the chip held under this load).
The dispatches of the record are taken in bench.py's order: for each B, `apply` then `adjoint` (warm-up
launches included: the counters are per dispatch and identical from launch to launch).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    keys = sys.argv[4].split(",") if len(sys.argv) > 4 else ["apply_b64", "adjoint_b64", "apply_b128", "adjoint_b128"]
    cnt = collections.defaultdict(dict)
    name = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            cnt[k][r["Counter_Name"]] = cnt[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            name[k] = r["Kernel_Name"]
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = [k for k in sorted(cnt) if "mfma" in name[k] and "SQ_VALU_MFMA_BUSY_CYCLES" in cnt[k]]
    groups = []  # consecutive dispatches of one (kernel, MFMA count, VALU count): one bench key
    for k in ids:
        sig = (name[k], cnt[k]["SQ_VALU_MFMA_BUSY_CYCLES"], cnt[k].get("SQ_INSTS_VALU"))
        if groups and groups[-1][0] == sig:
            groups[-1][1].append(k)
        else:
            groups.append((sig, [k]))
    tab = json.load(open(out)) if os.path.exists(out) else {}
    for key, (sig, ks) in zip(keys, groups):
        busy = sum(cnt[k]["SQ_VALU_MFMA_BUSY_CYCLES"] for k in ks) / len(ks)
        gui = sum(cnt[k]["GRBM_GUI_ACTIVE"] for k in ks) / len(ks) / 8.0
        t = sum(dur.get(k, 0.0) for k in ks) / len(ks)
        m = re.search(r"(\w+_kernel<[^>]*>)", sig[0])
        tab[key] = {"kernel": m.group(1) if m else sig[0][:80], "dispatches": len(ks), "SQ_VALU_MFMA_BUSY_CYCLES": busy,
                    "GRBM_GUI_ACTIVE_per_xcd": gui, "mfma_busy_frac": round(busy / (1024.0 * gui), 4),
                    "clock_ghz": round(gui / t / 1e9, 3) if t > 0 else None, "profiled_ms": round(1e3 * t, 4), "tag": tag,
                    "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)"}
        print(key, tab[key])
    json.dump(tab, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
