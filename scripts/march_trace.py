"""Development probe: per-band phase durations of the march kernel from its s_memtime trace
(PXA_TUNE_PGD_DIAG bit 5).  usage: python scripts/march_trace.py [bands_per_wg] [n]"""
import ctypes as ct
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd._lib import lib  # noqa: E402
from scripts.pgd_probe import taps  # noqa: E402

sb = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
g = torch.Generator(device="cuda").manual_seed(0)
x, xp, b = (torch.rand((n, n), device="cuda", generator=g) for _ in range(3))
out = torch.empty_like(x)
t = taps(2.0)
prev = [(k, _dev.tuning(k, v)) for k, v in ((_dev.TUNE_PGD_KERNEL, 5), (_dev.TUNE_MARCH_BANDS, sb), (3, 32))]
for _ in range(5):
    _dev.pgd_tv2d_step(x, xp, b, out, 1, 1, n, n, t, t, 1.0, 1.0, 0.02, 0.01, 0.3, 0.5, 1, 0.0)
torch.cuda.synchronize()
buf = np.zeros(1024, dtype=np.uint64)
assert lib.pxa_pgd_march_trace(buf.ctypes.data_as(ct.c_void_p), 1024) == 0
for k, v in prev:
    _dev.tuning(k, v)
names = ["wait+B1", "shift/conv+B2", "DMA issue+passA", "B3", "passB", "B4+vmwait", "epilogue", "->next top"]
tr = buf.astype(np.int64).reshape(2, 4, 16, 8)
for wg in range(2):
    for w in range(4):
        d = np.diff(tr[wg, w], axis=1)  # (16, 7) phase durations
        nxt = tr[wg, w, 1:, 0] - tr[wg, w, :-1, 7]
        med = np.median(d[1:min(sb, 16) - 1], axis=0) if sb > 3 else d[0]
        print(f"wg{wg} wave{w}: " + "  ".join(f"{names[i]} {med[i]:6.0f}" for i in range(7)),
              f" | gap {np.median(nxt[:max(1, min(sb, 16) - 1)]):6.0f}  band total {np.median(np.diff(tr[wg, w, :min(sb, 16), 0])):7.0f}")
