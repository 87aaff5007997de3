"""C3 benchmark (BASELINE.json configs[2]): PD3O / Condat-Vu on an n^3 volume, S = Gaussian(sigma=2)
(13 taps/axis, zero boundary), K = Gradient (3 directions), h = lam L1 (anisotropic TV), g = None,
fp32, synthetic piecewise-constant phantom + 1% noise.

Prints one JSON line per (algo, path) with the m_step time (HIP events over K back-to-back
iterations, inputs resident in HBM), iterations/s and the effective bandwidth at the compulsory
bytes of the fused dataflow (PD3O 76 B/voxel, CV 68 B/voxel) and at SURVEY §8(d)'s figure
(PD3O 80 B, CV 68 B).  Env: PXA_N (edge, default 1024), PXA_STEPS, PXA_GENERIC_N (edge of the generic
rule-by-rule comparison run, default 256; 0 skips it), PXA_NSEG (axis-0 segments, default 0 = auto)."""
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import pyxu_amd.abc as pxa
import pyxu_amd.operator as pxo
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

BYTES = {"pd3o": (76, 80), "cv": (68, 68)}


def problem(n, lam=0.01, sigma=2.0, seed=0):
    sh = (n, n, n)
    N = n**3
    g = torch.Generator(device="cuda").manual_seed(seed)
    x_gt = torch.zeros(sh, device="cuda", dtype=torch.float32)
    rng = np.random.default_rng(seed)
    for _ in range(12):
        lo = [int(rng.integers(0, n // 2)) for _ in sh]
        hi = [l + int(rng.integers(n // 8 + 1, n // 2 + 1)) for l in lo]
        x_gt[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = float(rng.uniform(0.2, 1.0))
    with pxrt.Precision(pxrt.Width.SINGLE):
        S = pxo.Gaussian(arg_shape=sh, sigma=sigma, truncate=3.0)
        y = S.apply(x_gt.reshape(-1))
        noise = 0.01 * torch.randn(N, device="cuda", dtype=torch.float32, generator=g)
        y = _dev.axpby(1.0, y, 1.0, noise)
        del x_gt, noise
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * S
        f.diff_lipschitz = 1.0  # ||S||^2 <= 1 for the normalised Gaussian (set analytically, §8(d))
        K = pxo.Gradient(arg_shape=sh)
        h = lam * pxo.L1Norm(dim=3 * N)
    return f, K, h, N


def run(algo, n, steps, fused, nseg):
    f, K, h, N = problem(n)
    klass = pxs.PD3O if algo == "pd3o" else pxs.CondatVu
    with pxrt.Precision(pxrt.Width.SINGLE):
        s = klass(f=f, g=None, h=h, K=K, show_progress=False)
        # MANUAL mode: m_init only (no end-of-fit writeback of the multi-GB iterates to disk)
        s.fit(x0=torch.zeros(N, device="cuda", dtype=torch.float32), stop_crit=pxst.MaxIter(1), fused=fused,
              mode=pxa.Mode.MANUAL)
        if s._astate.get("exception") is not None:
            raise RuntimeError("solver init failed") from s._astate["exception"]
        if fused:
            s._plan["nseg"] = nseg
        for _ in range(2):
            s.m_step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            s.m_step()
        e1.record()
        e1.synchronize()
        wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / steps
    b_fused, b_survey = BYTES[algo]
    line = {"algo": algo, "path": "fused" if fused else "generic", "n": n, "steps": steps, "ms_per_iter": round(ms, 3),
            "iters_per_s": round(1e3 / ms, 2), "host_ms_per_iter": round(1e3 * wall / steps, 3)}
    if fused:
        line["gbs_fused_bytes"] = round(b_fused * N / (ms * 1e-3) / 1e9, 1)
        line["gbs_survey_bytes"] = round(b_survey * N / (ms * 1e-3) / 1e9, 1)
        line["frac_survey_8tbs"] = round(b_survey * N / (ms * 1e-3) / 8e12, 3)
        line["nseg"] = nseg
    print(json.dumps(line), flush=True)
    shutil.rmtree(s.workdir, ignore_errors=True)
    del s, f, K, h
    torch.cuda.empty_cache()


def main():
    n = int(os.environ.get("PXA_N", "1024"))
    steps = int(os.environ.get("PXA_STEPS", "10"))
    gn = int(os.environ.get("PXA_GENERIC_N", "256"))
    nsegs = [int(v) for v in os.environ.get("PXA_NSEG", "0").split(",")]
    for algo in ("pd3o", "cv"):
        for nseg in nsegs:
            run(algo, n, steps, True, nseg)
        if gn:
            run(algo, gn, max(2, steps // 2), False, 0)
            run(algo, gn, steps, True, 0)


if __name__ == "__main__":
    main()
