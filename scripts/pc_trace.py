"""Development probe: per-iteration phases of the pipelined PGD kernel (PXA_TUNE_PGD_KERNEL = 2) from its
s_memtime trace (PXA_TUNE_PGD_DIAG bit 5): workgroups 0, 1, grid/2, grid-1; consumer wave 0 and producer
wave 4; iterations 0-3.  usage: python scripts/pc_trace.py [n[:stack]]"""
import ctypes as ct
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd._lib import lib  # noqa: E402
from scripts.pgd_modes_probe import T, launch, setup  # noqa: E402

spec = sys.argv[1] if len(sys.argv) > 1 else "2048"
diag = 32 | (int(sys.argv[2]) if len(sys.argv) > 2 else 0)  # + 64: producers idle, + 128: consumers idle
n, stack = (int(v) for v in (spec.split(":") + ["1"])[:2])
a, pre = setup(n, stack)
prev = [(k, _dev.tuning(k, v)) for k, v in ((_dev.TUNE_PGD_KERNEL, 2), (_dev.TUNE_PGD_DIAG, diag))]
for _ in range(10):
    launch(a, pre)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    launch(a, pre)
e1.record()
e1.synchronize()
print(f"n={n} stack={stack} diag={diag}: {e0.elapsed_time(e1) * 50:.2f} us per launch")
buf = np.zeros(128, dtype=np.uint64)
assert lib.pxa_pgd_tile_trace(buf.ctypes.data_as(ct.c_void_p), 128) == 0
for k, v in prev:
    _dev.tuning(k, v)
tr = buf.astype(np.int64).reshape(4, 2, 4, 4)
t0 = tr[tr > 0].min()
for slot, lab in enumerate(["wg0", "wg1", "wg n/2", "wg n-1"]):
    for role, rn in enumerate(["consumer", "producer"]):
        row = []
        for i in range(4):
            p = tr[slot, role, i]
            if p[0] == 0:
                continue
            nxt = tr[slot, role, i + 1, 0] if i < 3 and tr[slot, role, i + 1, 0] > 0 else None
            row.append(f"it{i}@{p[0] - t0:6d}: X {p[1] - p[0]:5d} B1 {p[2] - p[1]:5d} Y {p[3] - p[2]:5d}"
                       + (f" B2 {nxt - p[3]:5d}" if nxt is not None else ""))
        print(f"{lab:7s} {rn:8s} " + " | ".join(row))
