"""Development probe: 10 fused PGD steps of the bench problem at 2048^2 (and at 1000 x 1500: edge tiles), x saved
to a .npy file, so that two builds of the library (PXA_LIB_PATH) can be compared bit for bit.
usage: python scripts/pgd_bits_dump.py <out.npz>"""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

out = {}
for n0, n1 in ((2048, 2048), (1000, 1500)):
    f, g, _ = bench.build_problem(n0, n1, seed=3)
    with pxrt.Precision(pxrt.Width.SINGLE):
        like = torch.empty((1,), dtype=torch.float32, device="cuda")
        s = pxs.PGD(f=f, g=g, show_progress=False)
        s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10))
        assert s._plan is not None
        out[f"x_{n0}x{n1}"] = s.solution().cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", list(out))
