"""Development probe: host cost per PGD step at stop_rate=1 (RelError | MaxIter) on a small image (device time
per step far below the host's), with parts of the per-step host work stubbed out (timing only) to price them."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.abc.solver as pxsolver  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
f, g, _ = bench.build_problem(n, n, seed=1)


def run(label, steps=2000, crit="rel"):
    with pxrt.Precision(pxrt.Width.SINGLE):
        like = torch.empty((1,), dtype=torch.float32, device="cuda")
        s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
        sc = pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30) if crit == "rel" else pxst.MaxIter(10**9)
        s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=sc, mode=pxa.Mode.MANUAL)
        gen = s.steps()
        for _ in range(200):
            next(gen)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            next(gen)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"n={n} {label:40s} {1e6 * dt / steps:7.1f} us/step", flush=True)


run("baseline (RelError | MaxIter)")
run("MaxIter only", crit="maxiter")
orig_record = pxsolver.Solver._record
pxsolver.Solver._record = lambda self, *a, **k: None
run("history records + log lines stubbed")
pxsolver.Solver._record = orig_record
orig_info = pxa.Solver._step_speculative if hasattr(pxa, "Solver") else None
import logging  # noqa: E402

orig_info_fn = logging.Logger.info
logging.Logger.info = lambda self, *a, **k: None
run("log lines stubbed")
logging.Logger.info = orig_info_fn
