"""Probe build only (PXA_LIB_PATH=build/libpyxu_amd_probe.so): FFT.apply 2048x2048 with parts of the in-LDS
kernel skipped (PXA_TUNE_FFT_KERNEL bits 16 stages, 32 global loads, 64 global stores, 128 twiddle loads:
WRONG results, timing only), HIP events over 20 launches after 3 warm-ups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

for spec in sys.argv[1:] or ["2048x2048"]:
    sh = tuple(int(v) for v in spec.split("x"))
    N = 1
    for v in sh:
        N *= v
    with pxrt.Precision(pxrt.Width.SINGLE):
        op = pxo.FFT(arg_shape=sh)
        x = torch.randn(2 * N, device="cuda", dtype=torch.float32)
        for mode in (0, 16, 32, 64, 48, 80, 96, 112, 128, 224, 256, 512, 1):
            _dev.tuning(_dev.TUNE_FFT_KERNEL, mode)
            for _ in range(3):
                op.apply(x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                op.apply(x)
            e1.record()
            e1.synchronize()
            print(f"{spec} mode {mode:3d}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per FFT.apply", flush=True)
        _dev.tuning(_dev.TUNE_FFT_KERNEL, 0)
