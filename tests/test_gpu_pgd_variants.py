"""
Fused PGD step modes (csrc/pgd_tv2d.hip) against each other, bit for bit.

The classic launch (pxa_pgd_tv2d_step) forms the momentum point yk = (x - x_prev) * a + x inside its
window load.  The y-state launches (pxa_pgd_tv2d_step_y) carry yk as solver state: the seed launch
forms it like the classic one and also writes y_next = (x_new - x) * a_next + x_new, the steady-state
launch reads y instead of (x, x_prev).  Every per-pixel fp32 operation is the same, so x_new must agree
BIT FOR BIT on every shape class: interior and edge tiles, ragged tile grids, fewer tiles than
resident workgroups, stacks with shared and per-image data, every blur radius 1..8, every prox kind.
The classic kernel itself is pinned to the oracle by test_gpu_parity.py and test_gpu_bench_shapes.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd._lib import lib  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402


def _problem(sh, y_images, sigma, g_kind, lam=0.02, mu=0.01, seed=0):
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
    return f, g, dim, rng


def _plan(sh, stack, y_images, sigma, g_kind, fused=True, **kw):
    f, g, dim, rng = _problem(sh, y_images, sigma, g_kind, **kw)
    with pxrt.Precision(pxrt.Width.SINGLE):
        s = pxs.PGD(f=f, g=g, show_progress=False)
        rows = stack // y_images
        x0 = rng.uniform(0, 1, (rows, dim) if rows > 1 else dim).astype(np.float32)
        s.fit(x0=to_device(x0), stop_crit=pxst.MaxIter(2))
        assert (s._plan is not None) == fused
        return s


def _classic(s, x, xp, a, parts=None):
    p, m = s._plan, s._mstate
    out = _dev.empty_like(x)
    _dev.pgd_tv2d_step(x, xp, p["hty"], out, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"], p["h0"],
                       p["h1"], p["lam"], p["mu"], a, m["tau"], p["prox"], m["tau"] * p["prox_scale"], partials=parts,
                       pre=p["pre"])
    assert int(lib.pxa_pgd_tv2d_last_kernel()) == 1
    return out


def _ystep(s, x, xp, y, a, a_next, parts=None):
    p, m = s._plan, s._mstate
    out, yn = _dev.empty_like(x), _dev.empty_like(x)
    _dev.pgd_tv2d_step_y(x, xp, y, p["hty"], out, yn, a, a_next, m["tau"], p["prox"], m["tau"] * p["prox_scale"],
                         p["pre"], partials=parts)
    assert int(lib.pxa_pgd_tv2d_last_kernel()) == (3 if y is not None else 2)
    return out, yn


def _parts(s):
    p = s._plan
    n = int(lib.pxa_pgd_tv2d_partials_count(p["stack"], p["n0"], p["n1"]))
    return torch.full((2 * n,), -1.0, dtype=torch.float64, device="cuda")


CASES = [
    # (shape, stack, y_images, sigma, g)
    ((2048, 2048), 1, 1, 2.0, "pos"),   # the bench workload: interior + edge tiles
    ((96, 128), 1, 1, 2.0, "l1"),       # fewer tiles than workgroups (idle XCD groups)
    ((1000, 1004), 1, 1, 2.5, "pos"),   # ragged tile grid, R = 8
    ((300, 260), 1, 1, 0.3, "none"),    # R = 1
    ((257, 516), 1, 1, 1.0, "l1"),      # R = 3, odd row count
    ((128, 192), 3, 1, 2.0, "pos"),     # stacked initial points, one y
    ((64, 320), 4, 4, 1.5, "pos"),      # batch-as-axis: per-image data
    ((517, 1003), 1, 1, 2.0, "l1"),     # R = 6, odd row length (no 16-B vector path)
    ((40, 36), 2, 2, 1.0, "none"),      # tiles larger than the image
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0][0]}x{c[0][1]}-s{c[1]}-y{c[2]}-sig{c[3]}-{c[4]}")
def test_y_state_modes_bit_exact_vs_classic(case):
    """Two iterations k, k+1 with momenta a = 0.37, a' = 0.61: the seed launch and then the y-state launch
    reproduce the classic launch's x_new bit for bit, and the RelError partials of every mode are the same
    bits (same per-tile order)."""
    sh, stack, y_images, sigma, g_kind = case
    s = _plan(sh, stack, y_images, sigma, g_kind)
    m = s._mstate
    x, xp = m["x"], m["x_prev"]
    a, a2 = 0.37, 0.61
    pc, ps, py = _parts(s), _parts(s), _parts(s)
    c1 = _classic(s, x, xp, a, pc)
    s1, y1 = _ystep(s, x, xp, None, a, a2, ps)
    assert np.array_equal(to_NUMPY(c1), to_NUMPY(s1))
    assert np.array_equal(to_NUMPY(pc), to_NUMPY(ps)) and np.all(to_NUMPY(pc) >= 0)
    # y_next is the classic window's yk of the next iteration: (x1 - x) * a2 + x1 in one fma
    x1, x0 = to_NUMPY(s1).astype(np.float64), to_NUMPY(x).astype(np.float64)
    d = (to_NUMPY(s1) - to_NUMPY(x)).astype(np.float64)
    ref = (d * np.float64(np.float32(a2)) + x1).astype(np.float32)
    assert np.max(np.abs(to_NUMPY(y1) - ref) / np.maximum(np.abs(ref), 1e-30)) <= 1.2e-7
    c2 = _classic(s, c1, x, a2, pc)
    s2, _ = _ystep(s, s1, None, y1, a2, 0.7, py)
    assert np.array_equal(to_NUMPY(c2), to_NUMPY(s2))
    assert np.array_equal(to_NUMPY(pc), to_NUMPY(py))
    torch.cuda.synchronize()


def test_solver_y_state_trajectory_equals_classic_loop():
    """30 iterations of the fused solver (seed launch, then y-state launches with the look-ahead momentum
    a_{k+1} = (k+1)/(k+2+d)) against a loop of classic launches fed the reference's a_k: identical x."""
    s = _plan((256, 320), 1, 1, 2.0, "pos")
    f, g = s._f, s._g
    rng = np.random.default_rng(3)
    x0 = to_device(rng.uniform(0, 1, 256 * 320).astype(np.float32))
    with pxrt.Precision(pxrt.Width.SINGLE):
        sol = pxs.PGD(f=f, g=g, show_progress=False)
        sol.fit(x0=x0, stop_crit=pxst.MaxIter(30))
        got = to_NUMPY(sol.solution())
        x, xp = x0, x0
        for k in range(30):
            a = float(np.float32(k / (k + 1 + 75)))
            x, xp = _classic(s, x, xp, a), x
    assert np.array_equal(got, to_NUMPY(x))


@pytest.mark.parametrize("stack,rows", [(1, 1), (6, 3)])
def test_fused_relerr_matches_separate_pass(stack, rows):
    """stop_rate 1 RelError from the kernel's per-tile partials (pxa_tile_partials_fold) against the
    separate relerr_stats pass: the same stop iteration, values within 1e-6 relative, and the fused
    path launches no relerr pass (no x copy)."""
    y_images = stack // rows
    outs = {}
    for fused_rel in (True, False):
        f, g, dim, rng = _problem((128, 192), y_images, 2.0, "pos")
        x0 = to_device(np.zeros((rows, dim) if rows > 1 else dim, np.float32))
        with pxrt.Precision(pxrt.Width.SINGLE):
            s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
            s._fused_relerr = fused_rel
            s.fit(x0=x0, stop_crit=pxst.RelError(eps=2e-3) | pxst.MaxIter(500), mode=pxa.Mode.MANUAL)
            calls = {"relerr": 0}
            orig = _dev.relerr_stats

            def spy(*a, **k):
                calls["relerr"] += 1
                return orig(*a, **k)

            _dev.relerr_stats = spy
            try:
                hist = [h for h in s.steps()]
            finally:
                _dev.relerr_stats = orig
            _, h = s.stats()
        outs[fused_rel] = (len(hist), h, to_NUMPY(s.solution()), calls["relerr"])
    (n1, h1, x1, c1), (n2, h2, x2, c2) = outs[True], outs[False]
    assert n1 == n2 and 1 < n1 < 500
    assert np.array_equal(x1, x2)
    key = [k for k in h1.dtype.names if k.startswith("RelError")]
    for k in key:
        v1, v2 = h1[k].astype(np.float64), h2[k].astype(np.float64)
        assert np.allclose(v1, v2, rtol=1e-6, atol=0), k
    assert c1 <= 1 and c2 >= n2 - 2  # fused: at most the first comparison falls back to the separate pass


def test_wide_blur_warns_and_runs_generic_path():
    """A sigma = 3 blur (radius 9 > MAX_R) keeps the generic path, loudly (FusedPathWarning)."""
    from pyxu_amd.opt.solver._fused import FusedPathWarning

    with pytest.warns(FusedPathWarning):
        _plan((64, 96), 1, 1, 3.0, "pos", fused=False)
