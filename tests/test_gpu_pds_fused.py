"""
GPU parity of the fused primal-dual splitting step (pxa_pds_step: PD3O and Condat-Vu, three launches
per iteration) against the CPU oracle's restatement of the reference's m_step (pds.py:429-442,
747-761) on the same seeded inputs, and against the generic rule-by-rule path.

Tolerance (north_star): trajectories after 8 iterations <= 1e-5 norm-wise relative in fp32,
<= 1e-10 in fp64.  Cases cover 2-D images, 3-D volumes, batch-as-axis volumes (directions (1, 2)),
sizes smaller than the blur radius, ragged multi-tile planes, blur radii 2..8, anisotropic (L1) and
isotropic (L21) TV, and g in {None, PositiveOrthant, lam L1}.
"""
import numpy as np
import pytest

import oracle as orc
from conftest import rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402

TOL = {np.float32: 1e-5, np.float64: 1e-10}
ALGOS = {"pd3o": pxs.PD3O, "cv": pxs.CondatVu}


def W(dt):
    return pxrt.Width.SINGLE if np.dtype(dt) == np.float32 else pxrt.Width.DOUBLE


def D(a):
    return to_device(np.ascontiguousarray(a))


def _problem(sh, sigma, h_kind, g_kind, dt, batch_axis=False, lam=0.05, seed=0):
    """(f, g, h, K, host pieces for the oracle) of 1/2||S.-y||^2 + g + lam TV."""
    rng = np.random.default_rng(seed)
    N = int(np.prod(sh))
    y = rng.standard_normal(N).astype(dt)
    taps, c = orc.gaussian_taps(sigma, 3.0, dt)
    if batch_axis:
        kern = [np.array([1.0], dtype=dt), taps, taps]
        cen = [0, c, c]
        dirs = (1, 2)
    else:
        kern = [taps] * len(sh)
        cen = [c] * len(sh)
        dirs = tuple(range(len(sh)))
    Dd = len(dirs)
    S = pxo.Stencil(arg_shape=sh, kernel=kern, center=cen, mode="constant")
    f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(y)) * S
    f.diff_lipschitz = 1.0
    K = pxo.Gradient(arg_shape=sh, directions=dirs)
    h = lam * (pxo.L21Norm(arg_shape=(Dd, *sh)) if h_kind == "iso" else pxo.L1Norm(dim=Dd * N))
    g = {"none": None, "pos": pxo.PositiveOrthant(dim=N), "l1": 0.01 * pxo.L1Norm(dim=N)}[g_kind]
    host = dict(y=y, blur=dict(arg_shape=sh, kernel=kern, center=cen), dirs=dirs, Dd=Dd, lam=lam)
    return f, g, h, K, host


def _oracle(algo, host, g_kind, x0, tau, sigma, rho, n, h_kind, sh):
    dt = x0.dtype.type
    y, blur, dirs, Dd, lam = host["y"], host["blur"], host["dirs"], host["Dd"], host["lam"]
    grad_f = lambda v: orc.deblur_tv_grad(v, blur, y, 0.0, 1.0, dict(arg_shape=sh))
    Kf = lambda v: orc.gradient_apply(v, arg_shape=sh, directions=dirs)
    KT = lambda v: orc.gradient_adjoint(v, arg_shape=sh, directions=dirs)
    if h_kind == "iso":
        hp = lambda v, t: orc.l21_prox(v, t * dt(lam), (Dd, *sh))
    else:
        hp = lambda v, t: orc.l1_prox(v, t * dt(lam))
    fprox = lambda v, s: orc.fenchel_prox(hp, v, s)
    pg = {"none": None, "pos": lambda v, t: orc.positive_orthant_prox(v), "l1": lambda v, t: orc.l1_prox(v, t * dt(0.01))}[g_kind]
    if algo == "pd3o":
        x, z, _ = orc.pd3o(x0, grad_f, pg, Kf, KT, fprox, tau, sigma, rho, n)
    else:
        x, z = orc.condat_vu(x0, grad_f, pg, Kf, KT, fprox, tau, sigma, rho, n)
    return x, z


CASES = [
    # (shape, sigma, h, g, dtype, batch-as-axis)
    ((5, 7), 0.8, "l1", "none", np.float32, False),
    ((40, 68), 2.0, "iso", "pos", np.float32, False),
    ((70, 131), 2.5, "l1", "l1", np.float64, False),
    ((6, 9, 11), 0.8, "l1", "none", np.float32, False),
    ((17, 40, 70), 2.0, "l1", "none", np.float32, False),
    ((13, 33, 66), 1.0, "iso", "pos", np.float64, False),
    ((4, 33, 66), 2.0, "l1", "none", np.float32, True),
]


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{'x'.join(map(str, c[0]))}-s{c[1]}-{c[2]}-{c[3]}-{np.dtype(c[4]).name}{'-batch' if c[5] else ''}")
def test_pds_fused_vs_oracle(algo, case):
    sh, sigma, h_kind, g_kind, dt, batch = case
    N = int(np.prod(sh))
    x0 = np.random.default_rng(1).uniform(0, 1, N).astype(dt)
    n = 8
    with pxrt.Precision(W(dt)):
        f, g, h, K, host = _problem(sh, sigma, h_kind, g_kind, dt, batch_axis=batch)
        s = ALGOS[algo](f=f, g=g, h=h, K=K, show_progress=False)
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(n))
        assert s._plan is not None, "fused path not selected"
        x, z = to_NUMPY(s._mstate["x"]), to_NUMPY(s._mstate["z"])
        tau, sigma_, rho = s._mstate["tau"], s._mstate["sigma"], s._mstate["rho"]
    xr, zr = _oracle(algo, host, g_kind, x0, tau, sigma_, rho, n, h_kind, sh)
    assert rel_err(x, xr) <= TOL[dt], algo
    assert rel_err(z, zr) <= TOL[dt], algo


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
def test_pds_fused_matches_generic(algo):
    """Fused (3 launches) vs the generic rule-by-rule path (also HIP) on a multi-tile volume."""
    sh = (24, 64, 200)
    N = int(np.prod(sh))
    x0 = np.random.default_rng(2).uniform(0, 1, N).astype(np.float32)
    out = {}
    with pxrt.Precision(pxrt.Width.SINGLE):
        f, g, h, K, _ = _problem(sh, 2.0, "l1", "none", np.float32)
        for fused in (True, False):
            s = ALGOS[algo](f=f, g=g, h=h, K=K, show_progress=False)
            s.fit(x0=D(x0), stop_crit=pxst.MaxIter(10), fused=fused)
            assert (s._plan is not None) == fused
            out[fused] = (to_NUMPY(s._mstate["x"]), to_NUMPY(s._mstate["z"]))
    assert rel_err(out[True][0], out[False][0]) <= 1e-5
    assert rel_err(out[True][1], out[False][1]) <= 1e-5


def test_pds_axis0_segments_bit_exact():
    """Splitting the axis-0 march into segments recomputes the halo planes with the same arithmetic."""
    sh = (37, 40, 64)
    N = int(np.prod(sh))
    x0 = np.random.default_rng(3).uniform(0, 1, N).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        f, g, h, K, _ = _problem(sh, 2.0, "iso", "pos", np.float32)
        s = pxs.PD3O(f=f, g=g, h=h, K=K, show_progress=False)
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(3))
        p, m = s._plan, s._mstate
        outs = []
        for nseg in (1, 3, 37):
            xo, uo, zo = _dev.empty_like(m["x"]), _dev.empty_like(m["u"]), _dev.empty_like(m["z"])
            _dev.pds_step(0, p["pre"], None, m["u"], m["z"], p["hty"], xo, uo, zo, p["q"], p["w"], nseg=nseg)
            outs.append([to_NUMPY(t) for t in (xo, uo, zo)])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
def test_pds_fused_stacked_rows_and_no_input_mutation(algo):
    """(2, N) stacked initial points = two single solves; a user-held z0 is never overwritten."""
    sh = (9, 20, 36)
    N = int(np.prod(sh))
    rng = np.random.default_rng(4)
    x0 = rng.uniform(0, 1, (2, N)).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        f, g, h, K, _ = _problem(sh, 1.0, "l1", "none", np.float32)
        z0 = K(D(x0))
        z0_host = to_NUMPY(z0).copy()
        s = ALGOS[algo](f=f, g=g, h=h, K=K, show_progress=False)
        s.fit(x0=D(x0), z0=z0, stop_crit=pxst.MaxIter(5))
        assert s._plan is not None
        xs = to_NUMPY(s._mstate["x"])
        assert np.array_equal(to_NUMPY(z0), z0_host)
        for r in range(2):
            s1 = ALGOS[algo](f=f, g=g, h=h, K=K, show_progress=False)
            s1.fit(x0=D(x0[r]), stop_crit=pxst.MaxIter(5))
            assert rel_err(xs[r], to_NUMPY(s1._mstate["x"])) <= 1e-6


LA_CASES = [c for i, c in enumerate(CASES) if i in (0, 1, 2, 4, 5, 6)]


def _run(algo, case, n, lookahead, x0, interrupt=None):
    sh, sigma, h_kind, g_kind, dt, batch = case
    import pyxu_amd.abc as pxa

    with pxrt.Precision(W(dt)):
        f, g, h, K, _ = _problem(sh, sigma, h_kind, g_kind, dt, batch_axis=batch)
        s = ALGOS[algo](f=f, g=g, h=h, K=K, show_progress=False)
        s._LOOKAHEAD = lookahead
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(10 ** 6), mode=pxa.Mode.MANUAL)
        it = s.steps()
        for k in range(n):
            if interrupt is not None and k == interrupt:
                # a replaced state array (same values) invalidates the look-ahead: the step re-primes
                s._mstate["z"] = s._mstate["z"].clone()
            next(it)
        assert s._plan is not None and s._plan["la"] == lookahead
        return {k: to_NUMPY(v) for k, v in s._mstate.items() if k in ("x", "u", "z")}


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
@pytest.mark.parametrize("case", LA_CASES, ids=lambda c: f"{'x'.join(map(str, c[0]))}-s{c[1]}-{c[2]}-{c[3]}-{np.dtype(c[4]).name}{'-batch' if c[5] else ''}")
def test_pds_lookahead_matches_three_launch(algo, case):
    """pxa_pds_step_la (kernel B + kernel D: the dual update fused with the next march) against the
    three-launch step: the same expressions through the same device helpers, so the same bits."""
    N = int(np.prod(case[0]))
    x0 = np.random.default_rng(5).uniform(0, 1, N).astype(case[4])
    a = _run(algo, case, 6, True, x0)
    b = _run(algo, case, 6, False, x0)
    for k in a:
        assert np.array_equal(a[k], b[k]), (k, rel_err(a[k], b[k]))


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
def test_pds_lookahead_reprimes_after_state_change(algo):
    case = ((17, 40, 70), 2.0, "iso", "pos", np.float32, False)
    x0 = np.random.default_rng(6).uniform(0, 1, int(np.prod(case[0]))).astype(np.float32)
    a = _run(algo, case, 5, True, x0, interrupt=3)
    b = _run(algo, case, 5, True, x0)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("algo", [0, 1])
def test_pds_lookahead_segments_bit_exact(algo):
    """Kernel D's axis-0 segments recompute their halo planes (z, K^T z, v) with the same arithmetic."""
    sh = (37, 40, 64)
    N = int(np.prod(sh))
    x0 = np.random.default_rng(3).uniform(0, 1, N).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        f, g, h, K, _ = _problem(sh, 2.0, "iso", "pos", np.float32)
        s = (pxs.PD3O if algo == 0 else pxs.CondatVu)(f=f, g=g, h=h, K=K, show_progress=False)
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(3))
        p, m = s._plan, s._mstate
        outs = []
        for nseg in (1, 3, 37):
            x = _dev.copy(m["x"])
            u = _dev.copy(m["u"]) if algo == 0 else None
            xo, zo = _dev.empty_like(m["x"]), _dev.empty_like(m["z"])
            uo = _dev.empty_like(m["x"]) if algo == 0 else None
            kt = _dev.empty_like(m["x"]) if algo == 1 else None
            q = _dev.empty_like(m["x"])
            _dev.pds_step_la(algo, p["pre"], False, x, u, m["z"], p["hty"], xo, uo, zo, q, kt, p["w"], nseg=nseg)
            outs.append([to_NUMPY(t) for t in (x, xo, zo, q) + ((uo,) if algo == 0 else (kt,))])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
def test_pds_lookahead_two_positions_per_thread_bit_exact(algo):
    """Kernel D with two positions per thread (PXA_TUNE_PDS_MARCH bit 0) gives the default's bits."""
    case = ((17, 40, 70), 2.0, "iso", "pos", np.float32, False)
    x0 = np.random.default_rng(7).uniform(0, 1, int(np.prod(case[0]))).astype(np.float32)
    a = _run(algo, case, 4, True, x0)
    prev = _dev.tuning(_dev.TUNE_PDS_MARCH, 1)
    try:
        b = _run(algo, case, 4, True, x0)
    finally:
        _dev.tuning(_dev.TUNE_PDS_MARCH, prev)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("h_kind", ["l1", "iso"])
@pytest.mark.parametrize("sh", [(67, 129), (9, 33, 70), (5, 64, 128)], ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("relax", [0, 1])
def test_tv_dual_update_vs_oracle(dt, h_kind, sh, relax):
    """pxa_tv_dual_update (kernel C alone): relax(fenchel_prox_{sigma h}(z + sigma Grad w))
    against the oracle's reference arithmetic (operator.py:905-944, diff.py:1113-1265; pds.py:760 / 441)."""
    rng = np.random.default_rng(3)
    N = int(np.prod(sh))
    Dd = len(sh)
    w = rng.standard_normal(N).astype(dt)
    z = (0.05 * rng.standard_normal(Dd * N)).astype(dt)
    sigma, lam, rho = 0.37, 0.05, 0.7
    geom = (1, 1, *sh, 2) if Dd == 2 else (1, *sh, 3)
    out = to_NUMPY(_dev.tv_dual_update(D(w), D(z), geom, [-1.0] * 3, [1.0] * 3, sigma, lam, rho,
                                       0 if h_kind == "l1" else 1, relax=relax))
    d = np.dtype(dt).type
    if h_kind == "iso":
        hp = lambda v, t: orc.l21_prox(v, t * d(lam), (Dd, *sh))
    else:
        hp = lambda v, t: orc.l1_prox(v, t * d(lam))
    zin = z + d(sigma) * orc.gradient_apply(w, arg_shape=sh)
    zt = orc.fenchel_prox(hp, zin, sigma)
    ref = (d(1 - rho) * z + d(rho) * zt) if relax == 0 else (d(rho) * zt + d(1 - rho) * z)
    assert rel_err(out, ref) <= TOL[dt], rel_err(out, ref)


@pytest.mark.parametrize("rows", [1, 2, 4, 8, 9])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("h_kind", ["l1", "iso"])
@pytest.mark.parametrize("sh,stack", [((67, 129), 1), ((9, 33, 70), 1), ((5, 64, 128), 3), ((7, 37, 1024), 1),
                                      ((3, 1, 64), 2), ((6, 19, 260), 2)], ids=lambda s: "x".join(map(str, s)) if isinstance(s, tuple) else str(s))
def test_tv_dual_update_row_blocked_bit_exact(rows, dt, h_kind, sh, stack):
    """Kernel C with `rows` rows of w per thread (PXA_TUNE_DUAL_ROWS; 1: the one-row kernel without its next-plane
    prefetch; 2, 4: a thread's row + 1 neighbours are its own rows;
    8: the plane-block kernel, whose row + 1 / column + 1 neighbours come from an LDS image of the block, 3-D fp32)
    gives the one-row kernel's bits: odd row counts (the last block's missing rows), partial column blocks, a single
    row, stacks, 2-D and 3-D, both relaxations."""
    rng = np.random.default_rng(5)
    N = int(np.prod(sh))
    Dd = len(sh)
    w = rng.standard_normal(stack * N).astype(dt)
    z = (0.05 * rng.standard_normal(stack * Dd * N)).astype(dt)
    geom = (stack, 1, *sh, 2) if Dd == 2 else (stack, *sh, 3)
    for relax in (0, 1):
        args = (D(w), D(z), geom, [-1.0] * 3, [1.0] * 3, 0.37, 0.05, 0.7, 0 if h_kind == "l1" else 1)
        ref = to_NUMPY(_dev.tv_dual_update(*args, relax=relax))
        prev = _dev.tuning(_dev.TUNE_DUAL_ROWS, rows)
        try:
            got = to_NUMPY(_dev.tv_dual_update(*args, relax=relax))
        finally:
            _dev.tuning(_dev.TUNE_DUAL_ROWS, prev)
        assert np.array_equal(got, ref), (relax, rows)


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
def test_pds_lookahead_persistent_grid_bit_exact(algo):
    """Kernel D on a persistent grid (PXA_TUNE_PDS_MARCH bit 1: workgroups loop over the (segment, block) units)
    gives the one-workgroup-per-unit launch's bits.  512 in-plane blocks x the automatic segments: more units
    than resident workgroups, so the workgroups do loop."""
    case = ((40, 256, 512), 2.0, "iso", "pos", np.float32, False)
    x0 = np.random.default_rng(8).uniform(0, 1, int(np.prod(case[0]))).astype(np.float32)
    a = _run(algo, case, 4, True, x0)
    prev = _dev.tuning(_dev.TUNE_PDS_MARCH, 2)
    try:
        b = _run(algo, case, 4, True, x0)
    finally:
        _dev.tuning(_dev.TUNE_PDS_MARCH, prev)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
@pytest.mark.parametrize("slack", [0, 8])
def test_pds_lookahead_coupled_march_bit_exact(algo, slack):
    """Kernel D with the soft progress coupling of row neighbours (PXA_TUNE_PDS_MARCH bit 2; bits 3+ widen the
    allowed lag) gives the default launch's bits: the coupling only delays workgroups, it never changes what
    they compute.  256-wide rows (one block per row) and 512-wide ones (two), more units than resident
    workgroups, so some neighbours are not resident when others wait for them (the bounded spin)."""
    for shape in ((40, 256, 256), (24, 128, 512)):
        case = (shape, 2.0, "iso", "pos", np.float32, False)
        x0 = np.random.default_rng(9).uniform(0, 1, int(np.prod(shape))).astype(np.float32)
        a = _run(algo, case, 4, True, x0)
        prev = _dev.tuning(_dev.TUNE_PDS_MARCH, 4 | (slack << 3))
        try:
            b = _run(algo, case, 4, True, x0)
        finally:
            _dev.tuning(_dev.TUNE_PDS_MARCH, prev)
        for k in a:
            assert np.array_equal(a[k], b[k]), (shape, k)


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
@pytest.mark.parametrize("case", LA_CASES + [((40, 256, 512), 2.0, "iso", "pos", np.float32, False)],
                         ids=lambda c: "x".join(map(str, c[0])) + f"-{c[2]}-{np.dtype(c[4]).name}" if isinstance(c, tuple) else str(c))
def test_pds_lookahead_prefetch_march_bit_exact(algo, case):
    """Kernel D with every load of plane q + 1 issued before plane q is computed (the default: two planes of loads in
    flight per wave; PXA_TUNE_PDS_MARCH bit 9: three) gives the bits of the march without prefetch (bit 8): 2-D / 3-D,
    iso / aniso, fp32 / fp64, batch-as-axis."""
    N = int(np.prod(case[0]))
    x0 = np.random.default_rng(9).uniform(0, 1, N).astype(case[4])
    a = _run(algo, case, 5, True, x0)
    res = {}
    for v in (256, 512):
        prev = _dev.tuning(_dev.TUNE_PDS_MARCH, v)
        try:
            res[v] = _run(algo, case, 5, True, x0)
        finally:
            _dev.tuning(_dev.TUNE_PDS_MARCH, prev)
    for v, b in res.items():
        for k in a:
            assert np.array_equal(a[k], b[k]), (v, k)
