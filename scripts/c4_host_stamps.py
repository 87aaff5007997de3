"""Development probe: host timeline of one ADMM outer-iteration boundary in the C4 workload (bench.py --only c4):
every pyxu_amd._dev call and the solver entry points are wrapped with time.perf_counter_ns stamps, and the
stamps from the last CG step of one outer iteration to the first operator pass of the next are printed
(offsets in us, call duration in us) -- where the ~0.3 ms of device idle time at each boundary goes."""
import functools
import os
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
from pyxu_amd.opt.solver.cg import CG  # noqa: E402
from pyxu_amd.util import to_device  # noqa: E402

LOG = []
DEPTH = [0]


def wrap(owner, name, label):
    fn = getattr(owner, name)

    @functools.wraps(fn)
    def w(*a, **k):
        t = time.perf_counter_ns()
        DEPTH[0] += 1
        try:
            return fn(*a, **k)
        finally:
            DEPTH[0] -= 1
            LOG.append((t, time.perf_counter_ns(), label, DEPTH[0]))

    setattr(owner, name, w)


for n in dir(_dev):
    f = getattr(_dev, n)
    if callable(f) and not n.startswith("_") and getattr(f, "__module__", "") == "pyxu_amd._dev" and not isinstance(f, type):
        wrap(_dev, n, "_dev." + n)
for cls, names in ((pxs.ADMM, ("m_step", "_x_update")), (CG, ("m_init", "m_step", "solution", "_solve_inline", "fit")),
                   (pxa.Solver, ("_step", "_solve_inline", "stats")), (pxa.QuadraticFunc, ("prox",))):
    for n in names:
        if n in cls.__dict__:
            wrap(cls, n, f"{cls.__name__}.{n}")

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
    for _ in range(3):
        next(it)
    torch.cuda.synchronize()
    LOG.clear()
    for _ in range(2):
        next(it)
    torch.cuda.synchronize()
LOG.sort()
# the boundary: from the last CG.m_step before the 2nd ADMM.m_step's first dense_normal
starts = [i for i, e in enumerate(LOG) if e[2] == "ADMM.m_step"]
a = max(i for i, e in enumerate(LOG) if e[2] == "CG.m_step" and e[0] < LOG[starts[1]][0])
b = min(i for i, e in enumerate(LOG) if e[2] == "_dev.dense_normal" and e[0] > LOG[starts[1]][0])
t0 = LOG[a][0]
for t, e, lab, d in LOG[a:b + 1]:
    print(f"{(t - t0) / 1e3:9.1f} {(e - t) / 1e3:8.1f}  {'  ' * d}{lab}")
