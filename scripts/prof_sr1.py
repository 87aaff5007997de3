"""Development probe: host-side profile (cProfile) of the PGD headline at the reference default stop_rate = 1,
to find where the host spends its time per step (the device runs ~29 us of work per step)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

f, g, _ = bench.build_problem(2048, 2048, seed=1)
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30), mode=pxa.Mode.MANUAL)
    gen = s.steps()
    for _ in range(200):
        next(gen)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500):
        next(gen)
    torch.cuda.synchronize()
    print(f"plain: {1e6 * (time.perf_counter() - t0) / 500:.1f} us/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(500):
        next(gen)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
