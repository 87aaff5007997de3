"""Gradient.apply / .adjoint and L21Norm.prox at one shape, `reps` calls each (for rocprofv3 kernel-trace / PMC
passes).  usage: python scripts/grad_probe.py <n0>x<n1>[x<n2>] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402

sh = tuple(int(v) for v in sys.argv[1].split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N = 1
for v in sh:
    N *= v
with pxrt.Precision(pxrt.Width.SINGLE):
    G = pxo.Gradient(arg_shape=sh)
    h = pxo.L21Norm(arg_shape=(len(sh), *sh))
    x = torch.randn(N, device="cuda", dtype=torch.float32, generator=torch.Generator(device="cuda").manual_seed(0))
    for _ in range(reps):
        z = G.apply(x)
    for _ in range(reps):
        y = G.adjoint(z)
    for _ in range(reps):
        p = h.prox(z, 0.1)
    torch.cuda.synchronize()
