"""Debug: where do two PGD kernel variants differ? (development helper)"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402

n0, n1 = int(sys.argv[1]), int(sys.argv[2])
ka, kb = int(sys.argv[3]), int(sys.argv[4])
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand((n0, n1), device="cuda", generator=g)
xp = torch.rand((n0, n1), device="cuda", generator=g)
b = torch.rand((n0, n1), device="cuda", generator=g)
t = ([-1, 0, 1], [0.25, 0.5, 0.25])
outs = []
for k in (ka, kb):
    out = torch.full_like(x, -7.0)
    prev = _dev.tuning(_dev.TUNE_PGD_KERNEL, k)
    _dev.pgd_tv2d_step(x, xp, b, out, 1, 1, n0, n1, t, t, 1.0, 1.0, 0.02, 0.01, 0.3, 0.5, 0, 0.0)
    _dev.tuning(_dev.TUNE_PGD_KERNEL, prev)
    torch.cuda.synchronize()
    outs.append(out.cpu().numpy())
d = outs[0] != outs[1]
print("mismatches", d.sum(), "of", d.size)
if d.any():
    r, c = np.nonzero(d)
    print("rows", np.unique(r)[:40])
    print("cols", np.unique(c)[:80])
    print("sample", [(int(i), int(j), float(outs[0][i, j]), float(outs[1][i, j])) for i, j in list(zip(r, c))[:10]])
