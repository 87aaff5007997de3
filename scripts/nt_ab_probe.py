"""A/B of the non-temporal stream policy in the PDS dual-update kernels (PXA_TUNE_PDS_MARCH bit 1):
k4 (kernel C alone, 1024^3) and the C3 look-ahead step (kernels B + D), each with the policy on (default)
and off, interleaved.  Prints one JSON line per (variant, record).

usage: python scripts/nt_ab_probe.py [n] [reps]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from pyxu_amd import _dev

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    torch.cuda.set_device(0)
    args = argparse.Namespace(c3_n=n, c3_steps=10, c3_three_launch=False, k4_which="3d")
    ctx = bench.Ctx(1, 0, None)
    for rep in range(reps):
        for knob in (0, 2):
            prev = _dev.tuning(_dev.TUNE_PDS_MARCH, knob)
            try:
                k4 = bench.bench_k4(ctx, args)["3d_1024"]
                c3 = bench.bench_c3(ctx, args)
            finally:
                _dev.tuning(_dev.TUNE_PDS_MARCH, prev)
            rec = {"rep": rep, "nt": knob == 0, "k4_ms": k4["kernel_ms"], "k4_frac": k4["roofline"]["frac"]}
            for algo in ("pd3o", "cv"):
                r = c3[algo]
                rec[f"{algo}_ms_per_step"] = r["ms_per_step"]
                rec[f"{algo}_kernels_ms"] = [k["kernel_ms"] for k in r.get("kernels", [])]
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
