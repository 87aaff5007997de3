"""C5 benchmark (BASELINE.json configs[4]): batched PGD TV-deblur, batch-as-axis (B, 512, 512) with
Gaussian(sigma=(0, 2, 2)), Gradient(directions=(1, 2)), lam env_mu(L21) TV, PositiveOrthant; the
per-GPU share of the 512-image job at 8 GPUs is B = 64.  Solver API, MANUAL mode, stop_rate 50,
MaxIter | RelError.  One JSON line: image-iterations/s, ms per solver step, kernel ms (HIP events
on the launch stream) and the SURVEY §8(d) roofline figure (48 B/pixel/iteration).
Env: PXA_B (default 64), PXA_N (default 512), PXA_STEPS (default 200)."""
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


def main():
    B = int(os.environ.get("PXA_B", "64"))
    n = int(os.environ.get("PXA_N", "512"))
    steps = int(os.environ.get("PXA_STEPS", "200"))
    lam = mu = 0.01
    sh = (B, n, n)
    N = B * n * n
    g = torch.Generator(device="cuda").manual_seed(0)
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=(0, 2.0, 2.0), truncate=3.0)
        x_gt = (torch.rand(N, device="cuda", generator=g) > 0.7).float()
        y = _dev.axpby(1.0, H.apply(x_gt), 0.01, torch.randn(N, device="cuda", generator=g))
        G = pxo.Gradient(arg_shape=sh, directions=(1, 2))
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * G
        f.diff_lipschitz = 1.0 + 8 * lam / mu
        s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=N), show_progress=False, stop_rate=50)
        rel = pxst.RelError(eps=1e-30)
        s.fit(x0=torch.zeros(N, device="cuda"), stop_crit=pxst.MaxIter(10**9) | rel, mode=pxa.Mode.MANUAL)
        assert s._plan is not None
        rel.stop({"x": s._mstate["x"]})
        rel.stop({"x": s._mstate["x"]})
        rel.clear()
        gen = s.steps()
        for _ in range(20):
            next(gen)
        torch.cuda.synchronize()
        timer = _dev.LaunchTimer(window=10)
        _dev.set_launch_timer(timer)
        t0 = time.perf_counter()
        for _ in range(steps):
            next(gen)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        _dev.set_launch_timer(None)
        shutil.rmtree(s.workdir, ignore_errors=True)
    kms = timer.mean_ms()
    print(json.dumps({"config": "C5 per-GPU share", "images": B, "image": [n, n],
                      "image_iters_per_s": round(B * steps / dt, 1), "ms_per_step": round(1e3 * dt / steps, 4),
                      "kernel_ms": round(kms, 4), "survey_gbs": round(48 * N / (kms * 1e-3) / 1e9, 1),
                      "survey_frac_8tbs": round(48 * N / (kms * 1e-3) / 8e12, 3),
                      "compulsory_frac_8tbs": round(16 * N / (kms * 1e-3) / 8e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
