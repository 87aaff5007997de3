"""Development probe: device time per (PGD step with RelError partials + fold) pair, queued back to back without
host waits, with the fold writing its values and completion flags (a) into coherent host memory (the stop
check's HostFlagBuffer), (b) into device memory, (c) no fold at all.  A gap that only (a) shows is the cost of
the kernel boundary after a kernel that wrote host memory."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

f, g, _ = bench.build_problem(2048, 2048, seed=1)
N = 200
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    s = pxs.PGD(f=f, g=g, show_progress=False)
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(3))
    p, m = s._plan, s._mstate
    x, xp, hty = m["x"], m["x_prev"], p["hty"]
    parts = p["parts"]
    tpr = p["tiles_per_row"]
    fb = _dev.HostFlagBuffer(1)
    dev_out = torch.zeros(2, dtype=torch.float64, device="cuda")
    dev_flags = torch.zeros(2, dtype=torch.int32, device="cuda")
    outs = [_dev.empty_like(x), _dev.empty_like(x)]

    def run(mode):
        for i in range(N):
            p["plan"].step(x, xp, hty, outs[i & 1], 0.5, float(m["tau"]), 0.0, partials=parts)
            if mode == "host":
                fb.fold(parts, tpr)
            elif mode == "device":
                _dev.check(_dev.lib.pxa_tile_partials_fold(1, tpr, parts.data_ptr(), dev_out.data_ptr(),
                                                           dev_flags.data_ptr(), i + 1, _dev.stream()), "fold")

    for mode in ("none", "host", "device", "none", "host", "device"):
        run(mode)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(mode)
        e1.record()
        e1.synchronize()
        print(f"{mode:7s} {1e3 * e0.elapsed_time(e1) / N:7.2f} us per step")
