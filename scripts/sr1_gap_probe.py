"""Development probe: 600 PGD steps at 2048^2, stop_rate 1, MaxIter only (or RelError with argv[1] == 'rel'), for a
rocprofv3 kernel trace: the gaps between consecutive step launches show where the device waits."""
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
rel = len(sys.argv) > 1 and sys.argv[1] == "rel"
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
    sc = pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30) if rel else pxst.MaxIter(10**9)
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=sc, mode=pxa.Mode.MANUAL)
    gen = s.steps()
    for _ in range(600):
        next(gen)
    torch.cuda.synchronize()
print("done")
