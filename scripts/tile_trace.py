"""Development probe: phase durations of the tile kernel (pgd_tv2d_kernel) from its s_memtime trace
(PXA_TUNE_PGD_DIAG bit 5): workgroups 0, 1, grid/2, grid-1.  usage: python scripts/tile_trace.py [n] [sigma]"""
import ctypes as ct
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd._lib import lib  # noqa: E402
from scripts.pgd_probe import taps  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
sigma = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
g = torch.Generator(device="cuda").manual_seed(0)
x, xp, b = (torch.rand((n, n), device="cuda", generator=g) for _ in range(3))
out = torch.empty_like(x)
t = taps(sigma)
prev = [(_dev.TUNE_PGD_DIAG, _dev.tuning(_dev.TUNE_PGD_DIAG, 32))]
for _ in range(10):
    _dev.pgd_tv2d_step(x, xp, b, out, 1, 1, n, n, t, t, 1.0, 1.0, 0.02, 0.01, 0.3, 0.5, 1, 0.0)
torch.cuda.synchronize()
buf = np.zeros(128, dtype=np.uint64)
assert lib.pxa_pgd_tile_trace(buf.ctypes.data_as(ct.c_void_p), 128) == 0
for k, v in prev:
    _dev.tuning(k, v)
names = ["load", "B1", "passA", "B2(+ghost)", "passB", "stage O+B", "epilogue"]
tr = buf.astype(np.int64).reshape(4, 4, 8)
t0 = tr[:, :, 0].min()
for slot, lab in enumerate(["wg0", "wg1", "wg n/2", "wg n-1"]):
    for w in range(4):
        d = np.diff(tr[slot, w])
        print(f"{lab:7s} w{w} start {tr[slot, w, 0] - t0:7d}  " + "  ".join(f"{names[i]} {d[i]:6d}" for i in range(7)),
              f"| total {tr[slot, w, 7] - tr[slot, w, 0]:6d}")
