"""
PGD kernel variants against the tile kernel (pgd_tv2d_kernel with the staged row-major epilogue,
PXA_TUNE_PGD_KERNEL = 1): 4 (item-order epilogue) and 5 (march kernel: fp32, R <= 6, n1 % 4 == 0,
no partials; 64-column strips marched in 16-row bands).  All run the same per-pixel fp32 operations in
the same order (csrc/pgd_tv2d.hip), so x_new must agree BIT FOR BIT on every shape class: interior
and edge tiles / bands, ragged strips and band counts, runs of any length, fewer work units than
resident workgroups, stacks with shared and per-image data, every blur radius 1..8, every prox kind.
The default kernel itself is pinned to the oracle by test_gpu_parity.py and test_gpu_bench_shapes.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd._lib import lib  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402


def _plan(sh, stack, y_images, sigma, g_kind, lam=0.02, mu=0.01, seed=0, fused=True):
    rng = np.random.default_rng(seed)
    N = int(np.prod(sh))
    y = rng.standard_normal(y_images * N).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        if y_images == 1:
            H = pxo.Gaussian(arg_shape=sh, sigma=sigma)
            G = pxo.Gradient(arg_shape=sh)
            dim = N
            l21 = pxo.L21Norm(arg_shape=(2, *sh))
        else:
            H = pxo.Gaussian(arg_shape=(y_images, *sh), sigma=(0, sigma, sigma))
            G = pxo.Gradient(arg_shape=(y_images, *sh), directions=(1, 2))
            dim = y_images * N
            l21 = pxo.L21Norm(arg_shape=(2, y_images, *sh))
        f = 0.5 * pxo.SquaredL2Norm(dim=dim).asloss(to_device(y)) * H + lam * l21.moreau_envelope(mu) * G
        f.diff_lipschitz = 1 + 8 * lam / mu
        g = {"none": None, "pos": pxo.PositiveOrthant(dim=dim), "l1": 0.01 * pxo.L1Norm(dim=dim)}[g_kind]
        s = pxs.PGD(f=f, g=g, show_progress=False)
        rows = stack // y_images
        x0 = rng.uniform(0, 1, (rows, dim) if rows > 1 else dim).astype(np.float32)
        s.fit(x0=to_device(x0), stop_crit=pxst.MaxIter(2))
        assert (s._plan is not None) == fused
        return s


def _step(s, kernel, bands=0):
    p, m = s._plan, s._mstate
    x, xp = m["x"], m["x_prev"]
    out = _dev.empty_like(x)
    nparts = int(lib.pxa_pgd_tv2d_partials_count(p["stack"], p["n0"], p["n1"]))
    parts = torch.full((2 * nparts,), -1.0, dtype=torch.float64, device=x.device)
    prev = _dev.tuning(_dev.TUNE_PGD_KERNEL, kernel)
    prev_b = _dev.tuning(_dev.TUNE_MARCH_BANDS, bands)
    try:
        _dev.pgd_tv2d_step(x, xp, p["hty"], out, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"], p["h0"],
                           p["h1"], p["lam"], p["mu"], 0.37, m["tau"], p["prox"], m["tau"] * p["prox_scale"])
        ran = int(lib.pxa_pgd_tv2d_last_kernel())
        out2 = _dev.empty_like(x)
        _dev.pgd_tv2d_step(x, xp, p["hty"], out2, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"], p["h0"],
                           p["h1"], p["lam"], p["mu"], 0.37, m["tau"], p["prox"], m["tau"] * p["prox_scale"], partials=parts)
        torch.cuda.synchronize()
    finally:
        _dev.tuning(_dev.TUNE_PGD_KERNEL, prev)
        _dev.tuning(_dev.TUNE_MARCH_BANDS, prev_b)
    return to_NUMPY(out), to_NUMPY(out2), to_NUMPY(parts), ran


CASES = [
    # (shape, stack, y_images, sigma, g)
    ((2048, 2048), 1, 1, 2.0, "pos"),   # the bench workload: interior + edge tiles, 4 tiles / workgroup
    ((96, 128), 1, 1, 2.0, "l1"),       # fewer tiles than workgroups (idle XCD groups)
    ((1000, 1004), 1, 1, 2.5, "pos"),   # ragged tile grid, R = 8
    ((300, 260), 1, 1, 0.3, "none"),    # R = 1
    ((257, 516), 1, 1, 1.0, "l1"),      # R = 3, odd row count
    ((128, 192), 3, 1, 2.0, "pos"),     # stacked initial points, one y
    ((64, 320), 4, 4, 1.5, "pos"),      # batch-as-axis: per-image data
    ((517, 1004), 1, 1, 2.0, "l1"),     # R = 6, ragged strips (1004 = 15 x 64 + 44) and bands (517 = 32 x 16 + 5)
    ((40, 36), 2, 2, 1.0, "none"),      # one band-and-a-half, one narrow strip
]


def _march_applies(case):
    sh, stack, y_images, sigma, g_kind = case
    return sigma <= 2.0 and sh[1] % 4 == 0  # R = int(3 sigma + 0.5) <= 6


@pytest.mark.parametrize("kernel", [0, 4, 5])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0][0]}x{c[0][1]}-s{c[1]}-y{c[2]}-sig{c[3]}-{c[4]}")
def test_kernel_variants_bit_exact_vs_tile_kernel(case, kernel):
    """0 the default, 4 the item-order epilogue, 5 the march kernel, against the tile kernel: x_new bit
    for bit; the RelError partials (tile kernel in every variant) are the same double sums in another
    association order (<= 1e-12 relative).  The march kernel runs wherever it applies."""
    sh, stack, y_images, sigma, g_kind = case
    s = _plan(sh, stack, y_images, sigma, g_kind)
    a, a_p, pa, ran = _step(s, kernel)
    b, b_p, pb, ran_tile = _step(s, 1)
    assert ran_tile == 1
    if kernel == 5:
        assert ran == (2 if _march_applies(case) else 1)
    assert np.array_equal(a, b)
    assert np.array_equal(a_p, b_p) and np.array_equal(a, a_p)
    assert np.allclose(pa, pb, rtol=1e-12, atol=0) and np.all(pa >= 0)


@pytest.mark.parametrize("bands", [1, 3, 7, 200])
def test_march_run_lengths_bit_exact(bands):
    """March runs of 1, 3, 7 bands and whole strips (runs ending mid-image, at the last partial band,
    runs with a single band: no DMA prefetch at all) give the tile kernel's bits."""
    s = _plan((517, 1004), 1, 1, 2.0, "pos")
    a, _, _, ran = _step(s, 5, bands)
    b, _, _, _ = _step(s, 1)
    assert ran == 2
    assert np.array_equal(a, b)


def test_kernel_knob_round_trips():
    """The kernel-selection knob round-trips (default 0 = auto)."""
    assert _dev.tuning(_dev.TUNE_PGD_KERNEL) == 0
    prev = _dev.tuning(_dev.TUNE_PGD_KERNEL, 5)
    assert prev == 0 and _dev.tuning(_dev.TUNE_PGD_KERNEL) == 5
    _dev.tuning(_dev.TUNE_PGD_KERNEL, 0)


def test_wide_blur_warns_and_runs_generic_path():
    """A sigma = 3 blur (radius 9 > MAX_R) keeps the generic path, loudly (FusedPathWarning)."""
    from pyxu_amd.opt.solver._fused import FusedPathWarning

    with pytest.warns(FusedPathWarning):
        _plan((64, 96), 1, 1, 3.0, "pos", fused=False)
