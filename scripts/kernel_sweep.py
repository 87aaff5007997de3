"""Time the fused PGD step kernel (HIP events, back-to-back launches) over a sweep of image sizes,
blur radii and TV on/off, to locate where the kernel's time goes (one process, interleaved rounds)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import pyxu_amd.operator as pxo
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.util import to_device


def plan(n0, n1, sigma, lam, mu=0.01):
    sh = (n0, n1)
    N = n0 * n1
    with pxrt.Precision(pxrt.Width.SINGLE):
        y = to_device(np.random.default_rng(0).standard_normal(N).astype(np.float32))
        H = pxo.Gaussian(arg_shape=sh, sigma=sigma)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H
        if lam > 0:
            f = f + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * pxo.Gradient(arg_shape=sh)
        f.diff_lipschitz = 1 + 8 * lam / mu
        s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=N), show_progress=False)
        s.fit(x0=_dev.zeros((N,), y), stop_crit=pxst.MaxIter(2))
        return s


def time_it(s, reps=100):
    p = s._plan
    x, xp = s._mstate["x"], s._mstate["x_prev"]
    out = _dev.empty_like(x)

    def step():
        _dev.pgd_tv2d_step(x, xp, p["hty"], out, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"], p["h0"],
                           p["h1"], p["lam"], p["mu"], 0.5, s._mstate["tau"], p["prox"], 0.0)

    for _ in range(5):
        step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        step()
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


def main():
    cases = [(2048, 2048, 2.0, 0.01), (2048, 2048, 2.0, 0.0), (2048, 2048, 1.0, 0.01), (2048, 2048, 0.3, 0.01),
             (1024, 1024, 2.0, 0.01), (4096, 4096, 2.0, 0.01), (2048, 4096, 2.0, 0.01)]
    solvers = [(c, plan(*c)) for c in cases]
    res = {c: [] for c in cases}
    for _ in range(3):
        for c, s in solvers:
            res[c].append(time_it(s))
    for c in cases:
        n0, n1, sig, lam = c
        t = min(res[c])
        print(f"n={n0}x{n1} sigma={sig} lam={lam}: {t:8.2f} us  ({t * 1e3 / (n0 * n1):.3f} ns/pixel)", flush=True)


if __name__ == "__main__":
    main()
