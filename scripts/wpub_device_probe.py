"""Development probe: device time per PGD step at 2048^2 for the plain launch, the window-statistics launch with
publication (pxa_pgd_tv2d_plan_step_wpub) and the epilogue-partials launch, 400 launches each queued back to back
(no host waits), HIP events around each run."""
import os
import sys

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
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(3), mode=pxa.Mode.BLOCK)
    p, m = s._plan, s._mstate
    plan, hty, tau = p["plan"], p["hty"], float(m["tau"])
    bufs = [m["x"].clone(), m["x_prev"].clone(), torch.empty_like(m["x"])]
    parts = [p["parts"], torch.empty_like(p["parts"])]
    fb = _dev.HostFlagBuffer(p["rows"])
    N = 400

    def run(kind):
        prev = None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for rep in range(2):
            torch.cuda.synchronize()
            e0.record()
            for i in range(N):
                x, xp, out = bufs[i % 3], bufs[(i + 2) % 3], bufs[(i + 1) % 3]
                if kind == "plain":
                    plan.step(x, xp, hty, out, 0.5, tau, tau * p["prox_scale"])
                elif kind == "epilogue":
                    plan.step(x, xp, hty, out, 0.5, tau, tau * p["prox_scale"], partials=parts[0])
                else:
                    cur = parts[i & 1]
                    plan.step_wpub(x, xp, hty, out, 0.5, tau, tau * p["prox_scale"], cur, prev)
                    prev = (cur, fb, fb.next_seq()) if kind == "wpub" else None  # "wpart": statistics, no publication
            e1.record()
            torch.cuda.synchronize()
        return 1e3 * e0.elapsed_time(e1) / N

    for kind in ("plain", "wpub", "wpart", "epilogue", "plain", "wpub", "wpart"):
        print(f"{kind:9s} {run(kind):7.2f} us per launch (device, {N} queued)")
