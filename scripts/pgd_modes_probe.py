"""Timing probe of the fused PGD launch (pxa_pgd_tv2d_step), fp32, Gaussian sigma=2 (R = 6), TV, PositiveOrthant,
at n x n images (`stack` images of n x n with per-image data when given as n:stack): the tile kernel as it is and
with parts of its work skipped (PXA_TUNE_PGD_DIAG bits 6-10: WRONG results, timing only), which prices the
window loads, the passes and the rest.  Each configuration is timed as windows of back-to-back launches between
two HIP events (the bench's LaunchTimer convention), interleaved over 5 rounds; prints the median per launch.
usage: python scripts/pgd_modes_probe.py diag [n[:stack] ...] | stagger | one <diag>   (probe build:
PXA_LIB_PATH=build/libpyxu_amd_probe.so)"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.operator.linop.filter import gaussian_kernel1d  # noqa: E402

k = gaussian_kernel1d(2.0, 0, 6)
T = (list(range(-6, 7)), [float(v) for v in k])


def setup(n, stack):
    g = torch.Generator(device="cuda").manual_seed(0)
    a = {name: torch.rand((stack, n, n), device="cuda", generator=g) for name in ("x", "xp", "b")}
    a["out"] = torch.empty_like(a["x"])
    return a, _dev.pgd_tv2d_args(stack, stack, n, n, T, T, 1.0, 1.0, 0.01, 0.01, 1, 0.0)


def launch(a, pre):
    _dev.lib.pxa_pgd_tv2d_step(0, *pre, 0.3, 0.5, 1, 0.0, a["x"].data_ptr(), a["xp"].data_ptr(), a["b"].data_ptr(),
                               a["out"].data_ptr(), None, None, _dev.stream())


def window(a, pre, kern, n_launch, diag=0):
    pd = _dev.tuning(_dev.TUNE_PGD_DIAG, diag)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n_launch):
        launch(a, pre)
    e1.record()
    e1.synchronize()
    _dev.tuning(_dev.TUNE_PGD_DIAG, pd)
    return e0.elapsed_time(e1) * 1000.0 / n_launch


def diag_probe(sizes):
    """tile kernel with its passes skipped (64) / its window loads skipped (128): WRONG results, timing only"""
    for spec in sizes:
        n, stack = (int(v) for v in (spec.split(":") + ["1"])[:2])
        a, pre = setup(n, stack)
        nl = max(5, int(2e6 / (n * n * stack) * 50) if n * n * stack < 2e7 else 10)
        res = {d: [] for d in (0, 64, 128, 192, 256, 320, 512, 1024, 1536)}
        for d in res:
            window(a, pre, 1, 3, d)
        for _ in range(5):
            for d in res:
                res[d].append(window(a, pre, 1, nl, d))
        for d, v in res.items():
            lab = {0: "full", 64: "no passes", 128: "no window loads", 192: "neither", 256: "x window only",
                   320: "x window, no passes", 512: "no H^T y loads", 1024: "no x_new stores",
                   1536: "no H^T y, no x_new"}[d]
            print(f"n={n} stack={stack} tile kernel {lab:16s} {np.median(v):9.2f} us", flush=True)
        del a





def stagger_probe(n=2048):
    """first-round workgroups picked by `sel` start n x 1024 cycles late (PXA_TUNE_PGD_STAGGER, probe build):
    same results, only the phase of the four workgroups of a CU changes"""
    a, pre = setup(n, 1)
    cfg = [0] + [(sel << 8) | d for sel in (1, 2, 3, 4) for d in (4, 8, 12, 20)]
    res = {c: [] for c in cfg}
    for _ in range(5):
        for c in cfg:
            old = _dev.tuning(_dev.TUNE_PGD_STAGGER, c)
            window(a, pre, 1, 3)
            res[c].append(window(a, pre, 1, 40))
            _dev.tuning(_dev.TUNE_PGD_STAGGER, old)
    for c, v in res.items():
        print(f"n={n} stagger sel={c >> 8} delay={c & 255}x1024 cyc {np.median(v):9.2f} us", flush=True)


def one(diag, n=2048, launches=30):
    """`launches` launches with PXA_TUNE_PGD_DIAG = diag (for rocprofv3 --pmc passes, one variant per run)"""
    a, pre = setup(n, 1)
    _dev.tuning(_dev.TUNE_PGD_DIAG, diag)
    for _ in range(launches):
        launch(a, pre)
    torch.cuda.synchronize()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "stagger":
        return stagger_probe()
    if len(sys.argv) > 2 and sys.argv[1] == "one":
        return one(int(sys.argv[2]))
    return diag_probe([v for v in sys.argv[1:] if v != "diag"] or ["2048", "4096", "512:512"])


if __name__ == "__main__":
    main()
