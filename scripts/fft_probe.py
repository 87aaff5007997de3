"""FFT.apply at one shape, `reps` back-to-back launches (for rocprofv3 kernel-trace / PMC passes).
usage: python scripts/fft_probe.py <n0>x<n1>[x<n2>] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402

sh = tuple(int(v) for v in sys.argv[1].split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
N = int(np.prod(sh))
with pxrt.Precision(pxrt.Width.SINGLE):
    op = pxo.FFT(arg_shape=sh)
    x = torch.randn(2 * N, device="cuda", dtype=torch.float32, generator=torch.Generator(device="cuda").manual_seed(0))
    for _ in range(reps):
        y = op.apply(x)
    torch.cuda.synchronize()
