"""Development probe: host-side profile (cProfile) of the C4 ADMM outer iterations (bench.py --only c4 workload):
where the Python time of an outer iteration (QuadraticFunc.prox -> CG setup + 13 CG steps, L1 prox, updates) goes."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.util import to_device  # noqa: E402

M, N = 8192, 65536
gen = torch.Generator(device="cuda").manual_seed(1000)
Kr = torch.randn((M, N), generator=gen, device="cuda", dtype=torch.float32).mul_(1.0 / np.sqrt(M))
rng = np.random.default_rng(5)
xs = np.zeros(N, np.float32)
xs[rng.choice(N, 64, replace=False)] = rng.standard_normal(64).astype(np.float32)
with pxrt.Precision(pxrt.Width.SINGLE):
    K = pxa.LinOp.from_array(Kr)
    y = K.apply(to_device(xs))
    f = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(y) * K
    h = 0.01 * pxo.L1Norm(dim=N)
    s = pxs.ADMM(f=f, h=h, show_progress=False)
    s.fit(x0=torch.zeros((N,), device="cuda", dtype=torch.float32), tau=1.0, stop_crit=pxst.MaxIter(10**9), mode=pxa.Mode.MANUAL)
    it = s.steps()
    for _ in range(2):
        next(it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        next(it)
    torch.cuda.synchronize()
    print(f"plain: {1e3 * (time.perf_counter() - t0) / 4:.3f} ms per outer", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(4):
        next(it)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
    pstats.Stats(pr).sort_stats("tottime").print_stats(40)
