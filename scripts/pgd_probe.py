"""Time pxa_pgd_tv2d_step on a synthetic 2048^2 fp32 problem under tuning knobs (development probe).
usage: python scripts/pgd_probe.py [key=value ...] -- each arg 'K:k=v' sets tuning key k to v for a line"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.operator.linop.filter import gaussian_kernel1d  # noqa: E402


def taps(sigma):
    k = gaussian_kernel1d(sigma, 0, int(3 * sigma + 0.5)) if sigma else np.array([1.0])
    R = (len(k) - 1) // 2
    return (list(range(-R, R + 1)), [float(v) for v in k])


def run(n=2048, sigma=2.0, lam=0.02, knobs=(), iters=200):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand((n, n), device="cuda", generator=g)
    xp = torch.rand((n, n), device="cuda", generator=g)
    b = torch.rand((n, n), device="cuda", generator=g)
    out = torch.empty_like(x)
    t = taps(sigma)
    prev = [(k, _dev.tuning(k, v)) for k, v in knobs]
    pre = _dev.pgd_tv2d_args(1, 1, n, n, t, t, 1.0, 1.0, lam, 0.01, 1, 0.0)
    try:
        for _ in range(20):
            _dev.pgd_tv2d_step(x, xp, b, out, 1, 1, n, n, t, t, 1.0, 1.0, lam, 0.01, 0.3, 0.5, 1, 0.0, pre=pre)
        torch.cuda.synchronize()
        # per-launch event pairs: the kernel's own duration, independent of the host issue rate
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for e0, e1 in evs:
            e0.record()
            _dev.pgd_tv2d_step(x, xp, b, out, 1, 1, n, n, t, t, 1.0, 1.0, lam, 0.01, 0.3, 0.5, 1, 0.0, pre=pre)
            e1.record()
        torch.cuda.synchronize()
        return float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])) * 1000.0
    finally:
        for k, v in prev:
            _dev.tuning(k, v)


if __name__ == "__main__":
    for spec in sys.argv[1:] or ["base"]:
        knobs, kw = [], {}
        for part in spec.split(","):
            if part == "base":
                continue
            k, v = part.split("=")
            if k in ("n", "sigma", "lam"):
                kw[k] = float(v) if k != "n" else int(v)
            else:
                knobs.append((int(k), int(v)))
        print(f"{spec:40s} {run(knobs=knobs, **kw):8.2f} us", flush=True)
