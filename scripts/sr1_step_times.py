"""Development probe: per-step wall times of the PGD loop at stop_rate=1 (RelError | MaxIter) at n x n, after
warm-up: median / p90 / max and the mean, to separate steady host cost from periodic bursts."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

for n in [int(v) for v in sys.argv[1:]] or [2048]:
    f, g, _ = bench.build_problem(n, n, seed=1)
    with pxrt.Precision(pxrt.Width.SINGLE):
        like = torch.empty((1,), dtype=torch.float32, device="cuda")
        for sr in (1, 50):
            s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=sr)
            s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30), mode=pxa.Mode.MANUAL)
            gen = s.steps()
            for _ in range(100):
                next(gen)
            torch.cuda.synchronize()
            ts = np.empty(1001)
            ts[0] = time.perf_counter()
            for i in range(1000):
                next(gen)
                ts[i + 1] = time.perf_counter()
            torch.cuda.synchronize()
            tot = time.perf_counter() - ts[0]
            d = np.diff(ts) * 1e6
            print(f"n={n} stop_rate={sr}: mean {1e6 * tot / 1000:6.1f} us/step (host-side diffs: median {np.median(d):6.1f} "
                  f"p90 {np.percentile(d, 90):6.1f} max {d.max():7.1f}; top-5 {np.sort(d)[-5:].round(0)})", flush=True)
