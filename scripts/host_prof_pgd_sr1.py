# host-side profile of the PGD stop_rate=1 loop (cProfile), GPU box
import cProfile, pstats, sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import bench
import pyxu_amd.runtime as pxrt
import pyxu_amd.abc as pxa
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
from pyxu_amd import _dev
f, g, _ = bench.build_problem(int(sys.argv[1]) if len(sys.argv) > 1 else 2048, int(sys.argv[1]) if len(sys.argv) > 1 else 2048, seed=1)
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30), mode=pxa.Mode.MANUAL)
    gen = s.steps()
    for _ in range(50): next(gen)
    torch.cuda.synchronize()
    pr = cProfile.Profile(); t0 = time.perf_counter(); pr.enable()
    NS = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    for _ in range(NS): next(gen)
    torch.cuda.synchronize(); pr.disable(); dt = time.perf_counter() - t0
    print("us/step", 1e6 * dt / NS)
    pstats.Stats(pr).sort_stats("tottime").print_stats(45)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
