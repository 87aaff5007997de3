"""Development probe: host wall time of the pieces of a C4 ADMM outer iteration (no device syncs added): the time
spent in each wrapped function excluding the CG device waits, averaged over 4 outer iterations."""
import collections
import functools
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.abc.solver as pxsolver  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.solver.cg as pcg  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.util import to_device  # noqa: E402

T = collections.defaultdict(float)
C = collections.Counter()


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[label] += time.perf_counter() - t0
            C[label] += 1

    setattr(obj, name, g)


M, N = 8192, 65536
gen = torch.Generator(device="cuda").manual_seed(1000)
Kr = torch.randn((M, N), generator=gen, device="cuda", dtype=torch.float32).mul_(1.0 / np.sqrt(M))
xs = np.zeros(N, np.float32)
xs[np.random.default_rng(5).choice(N, 64, replace=False)] = 1.0
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
    wrap(pxa.QuadraticFunc, "prox", "QuadraticFunc.prox (whole CG solve)")
    wrap(pxsolver.Solver, "_solve_inline", "CG _solve_inline")
    wrap(pcg.CG, "m_init", "CG.m_init")
    wrap(pcg.CG, "solution", "CG.solution")
    wrap(pcg.CG, "m_step", "CG.m_step")
    wrap(pcg.CG, "__init__", "CG.__init__")
    wrap(_dev, "wait_event", "wait_event (device waits)")
    wrap(pxs.ADMM, "m_step", "ADMM.m_step")
    wrap(pxsolver.Solver, "_step", "Solver._step (all solvers)")
    t0 = time.perf_counter()
    for _ in range(4):
        next(it)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
print(f"outer: {1e3 * tot / 4:.3f} ms")
for k, v in sorted(T.items(), key=lambda kv: -kv[1]):
    print(f"  {k:40s} {1e3 * v / 4:8.3f} ms per outer  ({C[k] / 4:.1f} calls)")
