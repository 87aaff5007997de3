"""Development probe: latency from the launch of a fused PGD step to the host seeing its RelError statistics,
(a) folded by the tile kernel's last workgroup into a HostFlagBuffer (pxa_pgd_tv2d_plan_step with a sink),
(b) by the separate fold kernel (pxa_tile_partials_fold into the same kind of buffer)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

f, g, _ = bench.build_problem(2048, 2048, seed=1)
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    s = pxs.PGD(f=f, g=g, show_progress=False)
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(3))
    p, m = s._plan, s._mstate
    x, xp, hty = m["x"], m["x_prev"], p["hty"]
    parts = _dev.empty_f64((2 * int(_dev.lib.pxa_pgd_tv2d_partials_count(1, 2048, 2048)),), x)
    sink = _dev.HostFlagBuffer(1)
    out = _dev.empty_like(x)
    for mode in ("kernel", "fold", "kernel", "fold"):
        lat = []
        for rep in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "kernel":
                seq = sink.next_seq()
                p["plan"].step(x, xp, hty, out, 0.3, m["tau"], 0.0, partials=parts, sink=sink, seq=seq)
            else:
                p["plan"].step(x, xp, hty, out, 0.3, m["tau"], 0.0, partials=parts)
                seq = sink.fold(parts, 8192)
            t1 = time.perf_counter()
            while not (sink.flags == seq).all():
                pass
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            lat.append((t1 - t0, t2 - t0, t3 - t0))
        a = np.array(lat[5:]) * 1e6
        print(f"{mode:7s} launch {a[:, 0].mean():7.1f} us  flag seen {a[:, 1].mean():7.1f} us (min {a[:, 1].min():.1f})  "
              f"stream done {a[:, 2].mean():7.1f} us  values {sink.values.tolist()}")
