"""Profiling driver: the fused PGD-TV step alone at 2048^2 (fp32), `reps` launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

n = int(os.environ.get("PXA_N", "2048"))
reps = int(os.environ.get("PXA_REPS", "20"))
f, g, y = bench.build_problem(n, n, seed=1)
with pxrt.Precision(pxrt.Width.SINGLE):
    s = pxs.PGD(f=f, g=g, show_progress=False)
    s.fit(x0=_dev.zeros((n * n,), y), stop_crit=pxst.MaxIter(3))
    p = s._plan
    x, xp = s._mstate["x"], s._mstate["x_prev"]
    out = _dev.empty_like(x)
    for _ in range(reps):
        _dev.pgd_tv2d_step(x, xp, p["hty"], out, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"],
                           p["h0"], p["h1"], p["lam"], p["mu"], 0.9, s._mstate["tau"], p["prox"], 0.0)
    torch.cuda.synchronize()
print("done")
