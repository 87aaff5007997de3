"""
The fused PGD tile kernel (csrc/pgd_tv2d.hip) against itself on its different code paths, bit for bit:

* the 16-B vector path of the edge tiles (a vector that lies inside the image is moved as one access)
  against the all-scalar path the kernel takes when the arrays are not 16-B aligned;
* launches with and without the RelError partials;
* the partials themselves against the separate RelError pass (pxa_relerr_stats) and the solver's
  stop_rate = 1 path that consumes them (pxa_tile_partials_fold);
* the strip kernel (a workgroup walks a column strip of tiles, keeping the 4R shared window rows in LDS and
  prefetching the next tile's new rows) against the tile kernel, at every strip length.

Every per-pixel fp32 operation is the same on every path, so x_new must agree BIT FOR BIT on every shape
class: interior and edge tiles, ragged tile grids, fewer tiles than resident workgroups, stacks with shared
and per-image data, every blur radius 1..8, every prox kind.  The kernel itself is pinned to the oracle by
test_gpu_parity.py and test_gpu_bench_shapes.py.
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


def _launch(s, x, xp, hty, a, parts=None):
    p, m = s._plan, s._mstate
    out = _dev.empty_like(x)
    _dev.pgd_tv2d_step(x, xp, hty, out, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"], p["h0"],
                       p["h1"], p["lam"], p["mu"], a, m["tau"], p["prox"], m["tau"] * p["prox_scale"], partials=parts)
    assert int(lib.pxa_pgd_tv2d_last_kernel()) in (1, 2, 3)  # tile, strip or pipelined kernel (PXA_TUNE_PGD_KERNEL)
    return out


def _misaligned(t):
    """A copy of t whose data pointer is 4 B past a 16-B boundary (the kernel's scalar path)."""
    buf = torch.empty(t.numel() + 4, dtype=t.dtype, device=t.device)
    v = buf[1: 1 + t.numel()].view(t.shape)
    v.copy_(t)
    assert v.data_ptr() % 16 != 0
    return v


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
    ((40, 36), 2, 2, 1.0, "none"),      # tiles larger than the image
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0][0]}x{c[0][1]}-s{c[1]}-y{c[2]}-sig{c[3]}-{c[4]}")
def test_vector_and_scalar_paths_bit_exact(case):
    """Aligned arrays (16-B vector loads / stores, also on the edge tiles' inside vectors) against
    misaligned copies (every access scalar): x_new and the RelError partials bit for bit; a launch
    without partials gives the same x_new."""
    sh, stack, y_images, sigma, g_kind = case
    s = _plan(sh, stack, y_images, sigma, g_kind)
    m, p = s._mstate, s._plan
    x, xp, hty = m["x"], m["x_prev"], p["hty"]
    pa, pb = _parts(s), _parts(s)
    a = _launch(s, x, xp, hty, 0.37, pa)
    b = _launch(s, _misaligned(x), _misaligned(xp), _misaligned(hty), 0.37, pb)
    c = _launch(s, x, xp, hty, 0.37)
    torch.cuda.synchronize()
    assert np.array_equal(to_NUMPY(a), to_NUMPY(b))
    assert np.array_equal(to_NUMPY(a), to_NUMPY(c))
    assert np.array_equal(to_NUMPY(pa), to_NUMPY(pb)) and np.all(to_NUMPY(pa) >= 0)


@pytest.mark.parametrize("stop_rate", [1, 4])
@pytest.mark.parametrize("stack,rows", [(1, 1), (6, 3)])
def test_fused_relerr_matches_separate_pass(stack, rows, stop_rate):
    """RelError from the kernel's per-tile partials (pxa_tile_partials_fold; at stop_rate > 1 taken against
    the iterate of the previous check, the x_ref operand) against the separate relerr_stats pass: the same
    stop iteration, the same iterates, RelError values within 1e-6 relative; the fused path launches the
    separate pass at most once (the first comparison)."""
    y_images = stack // rows
    outs = {}
    for fused_rel in (True, False):
        f, g, dim, rng = _problem((128, 192), y_images, 2.0, "pos")
        x0 = to_device(np.zeros((rows, dim) if rows > 1 else dim, np.float32))
        with pxrt.Precision(pxrt.Width.SINGLE):
            s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=stop_rate)
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
    assert n1 == n2 and 1 < n1 < 500 * stop_rate
    assert np.array_equal(x1, x2)
    assert np.array_equal(h1["iteration"], h2["iteration"])
    for k in [k for k in h1.dtype.names if k.startswith("RelError")]:
        v1, v2 = h1[k].astype(np.float64), h2[k].astype(np.float64)
        assert np.allclose(v1, v2, rtol=1e-6, atol=0), k
    assert c1 <= 1 and c2 >= len(h2) - 2


@pytest.mark.parametrize("case", [((2048, 2048), 1, 1), ((128, 192), 6, 2), ((40, 36), 2, 2)],
                         ids=lambda c: f"{c[0][0]}x{c[0][1]}-s{c[1]}-y{c[2]}")
@pytest.mark.parametrize("fold_launch", [False, True], ids=["in_kernel", "step_fold"])
def test_in_kernel_fold_matches_fold_kernel(case, fold_launch):
    """pxa_pgd_tv2d_plan_step with a RelError sink: the workgroup that finishes last folds the partials into the
    host buffer with its completion flags -- the same bits as pxa_tile_partials_fold on the same partials, the
    same x_new as a launch without the fold, and the device counter is reset for the next launch (two launches
    in a row both publish).  pxa_pgd_tv2d_plan_step_fold (the fold launched behind the step by the same C
    call): the same."""
    sh, stack, y_images = case
    s = _plan(sh, stack, y_images, 2.0, "pos")
    m, p = s._mstate, s._plan
    x, xp, hty = m["x"], m["x_prev"], p["hty"]
    rows = stack // y_images
    per_row = int(lib.pxa_pgd_tv2d_partials_count(p["stack"], p["n0"], p["n1"])) // rows
    sink = _dev.HostFlagBuffer(rows)
    for rep in range(2):
        parts = _parts(s)
        seq = sink.next_seq()
        out = _dev.empty_like(x)
        p["plan"].step(x, xp, hty, out, 0.37, m["tau"], m["tau"] * p["prox_scale"], partials=parts, sink=sink, seq=seq,
                       fold_launch=fold_launch)
        sink.wait(seq)
        got = sink.values.copy()
        ref = _dev.empty_f64((2, rows), x)
        _dev.tile_partials_fold(parts, rows, per_row, ref)
        plain = _launch(s, x, xp, hty, 0.37)
        torch.cuda.synchronize()
        assert np.array_equal(got, to_NUMPY(ref).reshape(-1)), rep
        assert np.array_equal(to_NUMPY(out), to_NUMPY(plain)), rep


def test_wide_blur_warns_and_runs_generic_path():
    """A sigma = 3 blur (radius 9 > MAX_R) keeps the generic path, loudly (FusedPathWarning)."""
    from pyxu_amd.opt.solver._fused import FusedPathWarning

    with pytest.warns(FusedPathWarning):
        _plan((64, 96), 1, 1, 3.0, "pos", fused=False)


def _with_kernel(v, fn):
    old = _dev.tuning(0, v)  # PXA_TUNE_PGD_KERNEL: 1 tile kernel, v >= 2 strip kernel of v tiles, 0 auto
    try:
        return fn()
    finally:
        _dev.tuning(0, old)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0][0]}x{c[0][1]}-s{c[1]}-y{c[2]}-sig{c[3]}-{c[4]}")
def test_strip_kernel_matches_tile_kernel(case):
    """The strip kernel (PXA_TUNE_PGD_KERNEL = strip length; opt-in, measured slower) against the tile kernel:
    x_new and the RelError partials bit for bit, for strips of 2 and 3 tiles and whole-column strips (the top,
    interior and bottom tiles of one strip, ragged last strips); radii 1..8; 0 (the default) is the tile kernel."""
    sh, stack, y_images, sigma, g_kind = case
    s = _plan(sh, stack, y_images, sigma, g_kind)
    m, p = s._mstate, s._plan
    x, xp, hty = m["x"], m["x_prev"], p["hty"]

    def run(v):
        parts = _parts(s)
        out = _with_kernel(v, lambda: _launch(s, x, xp, hty, 0.37, parts))
        kern = int(lib.pxa_pgd_tv2d_last_kernel())
        torch.cuda.synchronize()
        return to_NUMPY(out), to_NUMPY(parts), kern

    ref, ref_parts, k1 = run(1)
    assert k1 == 1
    tiles0 = -(-sh[0] // 32)
    for v in sorted({2, 3, max(2, tiles0), 0}):
        got, got_parts, k = run(v)
        assert k == (2 if v >= 2 and tiles0 >= 2 else 1), (v, k)  # a strip of one tile is the tile kernel
        assert np.array_equal(got, ref), v
        assert np.array_equal(got_parts, ref_parts), v


@pytest.mark.parametrize("v", [2, 3])
def test_strip_kernel_solver_trajectory_and_misaligned_fallback(v):
    """30 PGD iterations through the solver (stop checks at stop_rate 1: the partials path) with the strip kernel
    give the tile kernel's iterates bit for bit; misaligned arrays fall back to the tile kernel (the strip kernel's
    prefetch moves whole 16-B vectors)."""
    pxa.Solver._LAG, lag0 = 0, pxa.Solver._LAG  # the speculative engine (the lagged one uses the window-partials launch,
    # which the strip kernel does not implement: it falls back to the tile kernel)

    def traj(kv):
        def go():
            f, g, dim, rng = _problem((200, 260), 1, 2.0, "pos")
            with pxrt.Precision(pxrt.Width.SINGLE):
                sv = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
                sv.fit(x0=to_device(rng.uniform(0, 1, dim).astype(np.float32)),
                       stop_crit=pxst.MaxIter(30) | pxst.RelError(eps=1e-9), mode=pxa.Mode.MANUAL)
                for _ in sv.steps():  # this thread launches the steps (pxa_pgd_tv2d_last_kernel is per thread)
                    pass
                return to_NUMPY(sv.solution()), int(lib.pxa_pgd_tv2d_last_kernel())
        return _with_kernel(kv, go)

    try:
        (xt, kt), (xs_, ks) = traj(1), traj(v)
    finally:
        pxa.Solver._LAG = lag0
    assert kt == 1 and ks == 2
    assert np.array_equal(xt, xs_)
    s = _plan((200, 260), 1, 1, 2.0, "pos")
    m, p = s._mstate, s._plan
    out = _with_kernel(2, lambda: _launch(s, _misaligned(m["x"]), _misaligned(m["x_prev"]), _misaligned(p["hty"]), 0.37))
    assert int(lib.pxa_pgd_tv2d_last_kernel()) == 1
    ref = _with_kernel(1, lambda: _launch(s, m["x"], m["x_prev"], p["hty"], 0.37))
    torch.cuda.synchronize()
    assert np.array_equal(to_NUMPY(out), to_NUMPY(ref))


def _with_pipe(on, fn):
    old = _dev.tuning(_dev.TUNE_PGD_PIPE, 1 if on else 0)
    try:
        return fn()
    finally:
        _dev.tuning(_dev.TUNE_PGD_PIPE, old)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0][0]}x{c[0][1]}-s{c[1]}-y{c[2]}-sig{c[3]}-{c[4]}")
def test_pipe_kernel_matches_tile_kernel(case):
    """The pipelined kernel (PXA_TUNE_PGD_PIPE = 1; opt-in, measured slower: resident workgroups, the next tile's window
    fetched by LDS-DMA during the current tile) against the tile kernel: x_new and the RelError partials bit for bit,
    with and without partials, on every shape class (edge tiles fetched clamped and zeroed, fewer tiles than
    workgroups, stacks); misaligned arrays and R = 8 (its LDS would not fit twice per CU) keep the tile kernel."""
    sh, stack, y_images, sigma, g_kind = case
    s = _plan(sh, stack, y_images, sigma, g_kind)
    m, p = s._mstate, s._plan
    x, xp, hty = m["x"], m["x_prev"], p["hty"]

    def run(on, with_parts=True):
        parts = _parts(s) if with_parts else None
        out = _with_pipe(on, lambda: _launch(s, x, xp, hty, 0.37, parts))
        kern = int(lib.pxa_pgd_tv2d_last_kernel())
        torch.cuda.synchronize()
        return to_NUMPY(out), (to_NUMPY(parts) if with_parts else None), kern

    ref, ref_parts, k1 = run(False)
    got, got_parts, k = run(True)
    assert (k1, k) == (1, 1 if sigma == 2.5 else 3)  # (sigma 2.5: R = 8)
    assert np.array_equal(got, ref)
    assert np.array_equal(got_parts, ref_parts)
    got2, _, _ = run(True, with_parts=False)
    assert np.array_equal(got2, ref)
    if sh == (300, 260):
        out = _with_pipe(True, lambda: _launch(s, _misaligned(x), _misaligned(xp), _misaligned(hty), 0.37))
        assert int(lib.pxa_pgd_tv2d_last_kernel()) == 1
        torch.cuda.synchronize()
        assert np.array_equal(to_NUMPY(out), ref)


@pytest.mark.parametrize("lag", [0, 8])
def test_pipe_kernel_solver_trajectory(lag):
    """PGD iterations through the solver at stop_rate 1 with the pipelined kernel give the tile kernel's iterates,
    stop iteration and RelError history bit for bit: through the speculative engine (lag 0: epilogue partials + fold
    launch) and the lagged one (lag 8: window partials, publication by the extra workgroup).  eps is set from a
    first run so that RelError stops the solve mid-run."""
    pxa.Solver._LAG, lag0 = lag, pxa.Solver._LAG

    def traj(on, eps):
        def go():
            f, g, dim, rng = _problem((260, 300), 1, 2.0, "pos")
            with pxrt.Precision(pxrt.Width.SINGLE):
                sv = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
                sv.fit(x0=to_device(rng.uniform(0, 1, dim).astype(np.float32)),
                       stop_crit=pxst.MaxIter(60) | pxst.RelError(eps=eps), mode=pxa.Mode.MANUAL)
                for _ in sv.steps():
                    pass
                hist = sv.stats()[1]
                return (to_NUMPY(sv.solution()), int(lib.pxa_pgd_tv2d_last_kernel()), int(sv._astate["idx"]),
                        {k: np.asarray(hist[k]) for k in hist.dtype.names})
        return _with_pipe(on, go)

    try:
        _, _, _, h0 = traj(False, 1e-30)
        key = next(k for k in h0 if k.startswith("RelError"))
        eps = float(h0[key][25]) * (1 + 1e-9)
        (xt, kt, it_t, ht), (xp_, kp, it_p, hp) = traj(False, eps), traj(True, eps)
    finally:
        pxa.Solver._LAG = lag0
    assert kt == 1 and kp == 3
    assert it_t == it_p and 1 < it_t < 59
    assert np.array_equal(xt, xp_)
    assert ht.keys() == hp.keys()
    for k in ht:
        assert np.array_equal(ht[k], hp[k]), k
