"""Probe build only (PXA_LIB_PATH=build/libpyxu_amd_probe.so): per-workgroup timing stats of the row-split
normal kernel (normal_group_kernel) at C4's 8192 x 65536, read back from the workspace tail -- kernel span,
the poller's gather time and poll rounds, one wave's row-arrival wait and barrier wait, degraded flags, and
the XCC id against blockIdx % 8.  Argument: the PXA_TUNE_NORMAL_KERNEL value (+16: plain exchange stores instead of write-through)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pyxu_amd import _dev  # noqa: E402

M, N = 8192, 65536
tune = int(sys.argv[1]) if len(sys.argv) > 1 else 0
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, N, device="cuda", generator=g).mul_(M ** -0.5)
x = torch.randn(N, device="cuda", generator=g)
wsz = int(_dev.lib.pxa_dense_normal_workspace_bytes(_dev.dtcode(x), M, N, 1))
work = torch.zeros((wsz,), dtype=torch.uint8, device="cuda")
_dev.tuning(_dev.TUNE_NORMAL_KERNEL, tune)
for _ in range(3):
    _dev.dense_normal(A, x, 1.0, 1.0, work=work)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    _dev.dense_normal(A, x, 1.0, 1.0, work=work)
e1.record()
e1.synchronize()
G = 256
st = work[wsz - G * 64:].view(torch.int64).cpu().numpy().reshape(G, 8).astype(np.float64)
span = (st[:, 1] - st[:, 0]) * 10e-3  # 100 MHz ticks -> us
rows = 129
xcc = st[:, 5].astype(int)
out = {"tune": tune, "ms": round(e0.elapsed_time(e1) / 10, 4),
       "span_us": [round(float(np.min(span)), 1), round(float(np.median(span)), 1), round(float(np.max(span)), 1)],
       "start_spread_us": round(float((st[:, 0].max() - st[:, 0].min()) * 10e-3), 2),
       "gather_us_per_row": round(float(np.median(st[:, 2]) * 10e-3 / rows), 3),
       "polls_per_row": round(float(np.median(st[:, 3]) / rows), 2),
       "dot_wait_us_per_row": round(float(np.median(st[:, 6]) * 10e-3 / rows), 3),
       "barrier_us_per_row": round(float(np.median(st[:, 7]) * 10e-3 / rows), 3),
       "degraded": int(st[:, 4].sum()),
       "xcc_matches_g_mod_8": bool(np.all((xcc - np.arange(G)) % 8 == (xcc[0] - 0) % 8)),
       "xcc_first16": xcc[:16].tolist()}
print(json.dumps(out), flush=True)
