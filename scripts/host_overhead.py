"""Host-side cost of one fused PGD solver step (tiny image => GPU time negligible): cProfile top list."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import pyxu_amd.abc as pxa
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

n = int(os.environ.get("PXA_N", "64"))
steps = int(os.environ.get("PXA_STEPS", "3000"))
f, g, y = bench.build_problem(n, n, seed=1)
with pxrt.Precision(pxrt.Width.SINGLE):
    s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=50)
    s.fit(x0=_dev.zeros((n * n,), y), stop_crit=pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30), mode=pxa.Mode.MANUAL)
    gen = s.steps()
    for _ in range(200):
        next(gen)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        next(gen)
    torch.cuda.synchronize()
    print(f"plain: {1e6 * (time.perf_counter() - t0) / steps:.2f} us/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        next(gen)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
