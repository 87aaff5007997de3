"""Development probe: wall time per PGD step at stop_rate=1 with and without the host profiler, and the
GPU-only time of the same launches (HIP events), to split host-bound from device-bound cost."""
import os
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

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
f, g, _ = bench.build_problem(N, N, seed=1)
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    for sr, crit in ((1, "rel"), (1, "maxiter"), (50, "rel")):
        s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=sr)
        sc = pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30) if crit == "rel" else pxst.MaxIter(10**9)
        s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=sc, mode=pxa.Mode.MANUAL)
        gen = s.steps()
        for _ in range(100):
            next(gen)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(500):
            next(gen)
        e1.record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"stop_rate={sr} crit={crit}: {1e6 * dt / 500:7.1f} us/step wall, {1e3 * e0.elapsed_time(e1) / 500:7.1f} us/step device span")
