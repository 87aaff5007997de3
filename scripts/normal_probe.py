"""Timing probes of pxa_dense_normal at C4's 8192 x 65536 (HIP events): the kernel as shipped and the
PXA_TUNE_NORMAL_DIAG variants with one part of the work removed (their results are wrong; only the time
is read).  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pyxu_amd import _dev

M, N = int(os.environ.get("PXA_M", "8192")), int(os.environ.get("PXA_N", "65536"))
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, N, device="cuda", generator=g)
x = torch.randn(N, device="cuda", generator=g)
out = {"M": M, "N": N}
for diag in (0, 1, 2, 3, 0):
    _dev.tuning(_dev.TUNE_NORMAL_DIAG, diag)
    for _ in range(3):
        _dev.dense_normal(A, x, 1.0, 1.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        _dev.dense_normal(A, x, 1.0, 1.0)
    e1.record()
    e1.synchronize()
    out[f"diag{diag}_ms"] = round(e0.elapsed_time(e1) / 20, 4)
_dev.tuning(_dev.TUNE_NORMAL_DIAG, 0)
print(json.dumps(out))
