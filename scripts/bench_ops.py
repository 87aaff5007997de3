"""Operator microbenchmarks (HIP events, back-to-back launches, inputs resident in HBM): FFT (complex
fp32, all axes) and the Gradient / Gradient-adjoint / L21-prox operators at C2/C3 sizes.  One JSON
line per case with ms and the effective bandwidth of the compulsory bytes (read + write once)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import pyxu_amd.operator as pxo
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    out = []
    with pxrt.Precision(pxrt.Width.SINGLE):
        for sh in [(2048, 2048), (4096, 4096), (256, 256, 256)]:
            N = int(np.prod(sh))
            op = pxo.FFT(arg_shape=sh)
            x = torch.randn(2 * N, device="cuda", dtype=torch.float32, generator=g)
            ms = timed(lambda: op.apply(x))
            passes = len(sh)
            out.append({"op": "FFT.apply", "shape": sh, "ms": round(ms, 4),
                        "gbs_per_pass": round(passes * 2 * 8 * N / (ms * 1e-3) / 1e9, 1),
                        "flops_5nlogn_tf": round(5 * N * np.log2(N) / (ms * 1e-3) / 1e12, 2)})
        for sh in [(2048, 2048), (1024, 1024, 1024)]:
            N = int(np.prod(sh))
            D = len(sh)
            G = pxo.Gradient(arg_shape=sh)
            x = torch.randn(N, device="cuda", dtype=torch.float32, generator=g)
            ms = timed(lambda: G.apply(x), reps=5 if N > 1e8 else 20)
            out.append({"op": "Gradient.apply", "shape": sh, "ms": round(ms, 4),
                        "gbs": round((4 + 4 * D) * N / (ms * 1e-3) / 1e9, 1)})
            z = G.apply(x)
            ms = timed(lambda: G.adjoint(z), reps=5 if N > 1e8 else 20)
            out.append({"op": "Gradient.adjoint", "shape": sh, "ms": round(ms, 4),
                        "gbs": round((4 * D + 4) * N / (ms * 1e-3) / 1e9, 1)})
            h = pxo.L21Norm(arg_shape=(D, *sh))
            ms = timed(lambda: h.prox(z, 0.1), reps=5 if N > 1e8 else 20)
            out.append({"op": "L21Norm.prox", "shape": sh, "ms": round(ms, 4),
                        "gbs": round(8 * D * N / (ms * 1e-3) / 1e9, 1)})
            del z, x
            torch.cuda.empty_cache()
    with pxrt.Precision(pxrt.Width.SINGLE):  # large non-separable zero-boundary stencil: FFT path vs direct taps
        for sh, K in [((2048, 2048), (31, 31)), ((2048, 2048), (15, 15)), ((256, 256, 256), (9, 9, 9))]:
            N = int(np.prod(sh))
            k = np.random.default_rng(0).standard_normal(K)
            x = torch.randn(N, device="cuda", dtype=torch.float32, generator=g)
            for path in ("fft", "direct"):
                op = pxo.Stencil(arg_shape=sh, kernel=k, center=tuple(s // 2 for s in K))
                op.FFT_MIN_TAPS = 1 << 60 if path == "direct" else 1  # force the path (default: by ndim and taps)
                ms = timed(lambda: op.apply(x), reps=5 if path == "direct" and N * k.size > 1e10 else 20)
                out.append({"op": f"Stencil.apply[{path}]", "shape": sh, "kernel": list(K), "ms": round(ms, 4),
                            "gbs": round(8 * N / (ms * 1e-3) / 1e9, 1)})
    with pxrt.Precision(pxrt.Width.SINGLE):  # separable Gaussian (13 taps per axis), constant and reflect modes
        for sh in [(2048, 2048), (512, 512, 512)]:
            N = int(np.prod(sh))
            x = torch.randn(N, device="cuda", dtype=torch.float32, generator=g)
            for mode in ("constant", "reflect"):
                op = pxo.Gaussian(arg_shape=sh, sigma=2.0, truncate=3.0, mode=mode) if hasattr(pxo, "Gaussian") else None
                if op is None:
                    continue
                for knob in (0, 4):  # PXA_TUNE_STENCIL_ND bit 2 set: no LDS-tiled off-last-axis passes
                    old = _dev.tuning(_dev.TUNE_STENCIL_ND, knob)
                    ms = timed(lambda: op.apply(x), reps=5 if N > 1e8 else 20)
                    _dev.tuning(_dev.TUNE_STENCIL_ND, old)
                    out.append({"op": f"Gaussian.apply[{mode}]", "knob": knob, "shape": sh, "ms": round(ms, 4),
                                "gbs_per_axis_pass": round(len(sh) * 8 * N / (ms * 1e-3) / 1e9, 1)})
    for line in out:
        line["shape"] = list(line["shape"])
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
