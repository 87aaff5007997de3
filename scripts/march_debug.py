"""Development probe: pxa_pgd_tv2d_step through the march kernel (PXA_TUNE_PGD_KERNEL = 5) against the
tile kernel on random inputs; prints where x_new differs (band row mod 16, strip column mod 64) and by
how much.  usage: python scripts/march_debug.py n0 n1 [sigma] [lam]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from scripts.pgd_probe import taps  # noqa: E402


def main():
    n0, n1 = int(sys.argv[1]), int(sys.argv[2])
    sigma = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    lam = float(sys.argv[4]) if len(sys.argv) > 4 else 0.02
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand((n0, n1), device="cuda", generator=g)
    xp = torch.rand((n0, n1), device="cuda", generator=g)
    b = torch.rand((n0, n1), device="cuda", generator=g)
    t = taps(sigma)
    outs = {}
    for k in (0, 5):
        prev = _dev.tuning(_dev.TUNE_PGD_KERNEL, k)
        out = torch.full_like(x, float("nan"))
        _dev.pgd_tv2d_step(x, xp, b, out, 1, 1, n0, n1, t, t, 1.0, 1.0, lam, 0.01, 0.3, 0.5, 1, 0.0)
        torch.cuda.synchronize()
        _dev.tuning(_dev.TUNE_PGD_KERNEL, prev)
        outs[k] = out.cpu().numpy()
    a, m = outs[0], outs[5]
    bad = ~((a == m) | (np.isnan(a) & np.isnan(m)))
    print(f"{n0}x{n1} sigma={sigma} lam={lam}: {bad.sum()} of {a.size} differ; nan(march)={np.isnan(m).sum()}")
    if bad.any():
        d = np.abs(a - m)[bad]
        print(f"  max |diff| {np.nanmax(d):.3e}  median {np.nanmedian(d):.3e}  rel {np.nanmax(d / np.maximum(np.abs(a[bad]), 1e-30)):.3e}")
        rr, cc = np.nonzero(bad)
        print("  rows mod 16:", np.bincount(rr % 16, minlength=16).tolist())
        print("  cols mod 64:", np.bincount(cc % 64, minlength=64).tolist())
        print("  first rows:", sorted(set(rr.tolist()))[:20], " first cols:", sorted(set(cc.tolist()))[:20])


if __name__ == "__main__":
    main()
