"""A/B probe of the fused PGD launch (pxa_pgd_tv2d_step) under PXA_TUNE_PGD_STAGGER start-delay settings, at 2048^2 / 4096^2 fp32 (Gaussian sigma=2, TV, PositiveOrthant).
Each configuration is timed as windows of 50 back-to-back launches between two HIP events (the bench's
LaunchTimer convention), the configurations interleaved over 5 rounds; prints the median per launch.
usage: python scripts/pgd_modes_probe.py [n ...]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.operator.linop.filter import gaussian_kernel1d  # noqa: E402

k = gaussian_kernel1d(2.0, 0, 6)
T = (list(range(-6, 7)), [float(v) for v in k])


def setup(n):
    g = torch.Generator(device="cuda").manual_seed(0)
    a = {name: torch.rand((n, n), device="cuda", generator=g) for name in ("x", "xp", "y", "b")}
    a.update(out=torch.empty_like(a["x"]), yn=torch.empty_like(a["x"]))
    return a, _dev.pgd_tv2d_args(1, 1, n, n, T, T, 1.0, 1.0, 0.01, 0.01, 1, 0.0)


def launch(a, pre, mode):
    _dev.lib.pxa_pgd_tv2d_step(0, *pre, 0.3, 0.5, 1, 0.0, a["x"].data_ptr(), a["xp"].data_ptr(), a["b"].data_ptr(),
                               a["out"].data_ptr(), None, _dev.stream())


def window(a, pre, mode, stagger, n_launch=50):
    _dev.tuning(_dev.TUNE_PGD_STAGGER, stagger)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n_launch):
        launch(a, pre, mode)
    e1.record()
    e1.synchronize()
    _dev.tuning(_dev.TUNE_PGD_STAGGER, 0)
    return e0.elapsed_time(e1) * 1000.0 / n_launch


def main():
    sizes = [int(v) for v in sys.argv[1:]] or [2048, 4096]
    confs = [("classic", 0)] + [("classic", (sel << 8) | nn) for sel in (4,) for nn in (4,)]
    for n in sizes:
        a, pre = setup(n)
        for m, s in confs:
            for _ in range(3):
                window(a, pre, m, s)
        res = {c: [] for c in confs}
        for _ in range(5):
            for m, s in confs:
                res[(m, s)].append(window(a, pre, m, s))
        for (m, s), v in res.items():
            print(f"n={n} mode={m:8s} stagger=0x{s:04x}  {np.median(v):8.2f} us  (min {min(v):.2f})", flush=True)
        del a


if __name__ == "__main__":
    main()
