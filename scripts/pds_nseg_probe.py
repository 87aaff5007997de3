"""Axis-0 segment count (the plan's nseg; 0 = auto) of the look-ahead PDS step's kernel D on the C3
workload: per-kernel times (HIP events inside pxa_pds_step_la) of interleaved runs of 3 steps per
setting, 4 rounds; prints the median per kernel and setting.
usage: python scripts/pds_nseg_probe.py NSEG1 NSEG2 ... [--n 1024]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

args = sys.argv[1:]
n = 1024
if "--n" in args:
    i = args.index("--n")
    n = int(args[i + 1])
    args = args[:i] + args[i + 2:]
vals = [int(v) for v in args]
sh = (n, n, n)
N = n ** 3
gen = torch.Generator(device="cuda").manual_seed(7)
with pxrt.Precision(pxrt.Width.SINGLE):
    S = pxo.Gaussian(arg_shape=sh, sigma=2.0, truncate=3.0)
    y = torch.rand(N, device="cuda", generator=gen)
    f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * S
    f.diff_lipschitz = 1.0
    Kop = pxo.Gradient(arg_shape=sh)
    h = 0.01 * pxo.L1Norm(dim=3 * N)
    for algo, klass in (("pd3o", pxs.PD3O), ("cv", pxs.CondatVu)):
        s = klass(f=f, g=None, h=h, K=Kop, show_progress=False, stop_rate=10**6)
        s.fit(x0=torch.zeros(N, device="cuda"), stop_crit=pxst.MaxIter(10**9), mode=pxa.Mode.MANUAL)
        it = s.steps()
        for _ in range(2):
            next(it)
        res = {v: [] for v in vals}
        prev_ev = _dev.tuning(_dev.TUNE_PDS_EVENTS, 1)
        for _ in range(4):
            for v in vals:
                s._plan["nseg"] = v
                next(it)  # one untimed step at the new segmentation
                torch.cuda.synchronize()
                _dev.pds_kernel_ms(reset=True)
                for _ in range(3):
                    next(it)
                torch.cuda.synchronize()
                nrec, ms = _dev.pds_kernel_ms(reset=True)
                res[v].append([m / max(nrec, 1) for m in ms])
        _dev.tuning(_dev.TUNE_PDS_EVENTS, prev_ev)
        for v in vals:
            med = np.median(np.array(res[v]), axis=0)
            print(f"{algo} nseg {v}: A {med[0]:.3f} B {med[1]:.3f} C/D {med[2]:.3f} ms, sum {med.sum():.3f}", flush=True)
        del s, it
        torch.cuda.empty_cache()
