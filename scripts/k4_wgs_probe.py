"""A/B of kernel C's axis-0 segmentation (PXA_TUNE_DUAL_WGS: target workgroup count) on the k4 record at
1024^3, interleaved, 3 reps.  usage: python scripts/k4_wgs_probe.py [targets]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from pyxu_amd import _dev

    targets = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,2048,8192").split(",")]
    torch.cuda.set_device(0)
    args = argparse.Namespace(c3_n=1024, k4_which="3d")
    for rep in range(3):
        for t in targets:
            prev = _dev.tuning(_dev.TUNE_DUAL_WGS, t)
            try:
                r = bench.bench_k4(bench.Ctx(1, 0, None), args)["3d_1024"]
            finally:
                _dev.tuning(_dev.TUNE_DUAL_WGS, prev)
            print(json.dumps({"rep": rep, "target_wgs": t or 4096, "kernel_ms": r["kernel_ms"],
                              "frac": r["roofline"]["frac"]}), flush=True)


if __name__ == "__main__":
    main()
