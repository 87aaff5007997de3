"""Pin the CPU oracle (oracle/pyxu_np.py) against goldens recorded from the reference itself."""
import numpy as np
import pytest

import oracle as orc
from conftest import golden_names, load_golden, rel_err

TOL = {np.float32: 1e-6, np.float64: 1e-13}


def _tol(a):
    return TOL[a.dtype.type]


def _kernels(g):
    ks = [g[f"kernel{i}"] for i in range(int(g["n_kernels"]))]
    return ks if bool(g["separable"]) else ks[0]


def _mode(g):
    m = g["mode"]
    return str(m) if m.ndim == 0 else tuple(str(s) for s in m)


@pytest.mark.parametrize("name", golden_names("stencil_"))
def test_stencil(name):
    g = load_golden(name)
    sh = tuple(g["arg_shape"])
    y = orc.stencil_apply(g["x"], sh, _kernels(g), g["center"], _mode(g))
    a = orc.stencil_adjoint(g["z"], sh, _kernels(g), g["center"], _mode(g))
    assert y.dtype == g["y"].dtype
    assert rel_err(y, g["y"]) <= _tol(y)
    assert rel_err(a, g["adj"]) <= _tol(a)


@pytest.mark.parametrize("name", golden_names("gaussian_"))
def test_gaussian(name):
    g = load_golden(name)
    dt = g["x"].dtype
    taps, c = orc.gaussian_taps(float(g["sigma"]), float(g["truncate"]), dt)
    np.testing.assert_array_equal(taps, g["taps"])
    sh = tuple(g["arg_shape"])
    y = orc.stencil_apply(g["x"], sh, [taps, taps], [c, c])
    a = orc.stencil_adjoint(g["z"], sh, [taps, taps], [c, c])
    assert rel_err(y, g["y"]) <= _tol(y)
    assert rel_err(a, g["adj"]) <= _tol(a)


@pytest.mark.parametrize("name", golden_names("convolve_"))
def test_convolve(name):
    g = load_golden(name)
    sh = tuple(g["arg_shape"])
    k = [g["kernel0"], g["kernel1"]]
    # Convolve = Stencil with flipped kernel / swapped fw-bw (stencil.py:794-887)
    kf = [np.flip(k[0]), np.flip(k[1])]
    cf = [k[0].size - g["center"][0] - 1, k[1].size - g["center"][1] - 1]
    y = orc.stencil_apply(g["x"], sh, kf, cf)
    a = orc.stencil_adjoint(g["z"], sh, kf, cf)
    assert rel_err(y, g["y"]) <= _tol(y)
    assert rel_err(a, g["adj"]) <= _tol(a)


@pytest.mark.parametrize("name", golden_names("gradient_"))
def test_gradient(name):
    g = load_golden(name)
    kw = dict(
        arg_shape=tuple(g["arg_shape"]),
        directions=tuple(g["directions"]),
        scheme=str(g["scheme"]),
        accuracy=int(g["accuracy"]),
        sampling=float(g["sampling"]),
        mode=str(g["mode"]),
    )
    y = orc.gradient_apply(g["x"], **kw)
    a = orc.gradient_adjoint(g["z"], **kw)
    assert rel_err(y, g["y"]) <= _tol(y)
    assert rel_err(a, g["adj"]) <= _tol(a)


@pytest.mark.parametrize("name", golden_names("norms_"))
def test_norms(name):
    g = load_golden(name)
    x, sh, lam = g["x"], tuple(g["arg_shape"]), float(g["lam"])
    np.testing.assert_array_equal(orc.l1_prox(x, 0.8), g["l1_prox"])
    np.testing.assert_array_equal(orc.l21_prox(x, 0.8, sh), g["l21_prox"])
    l1s = lambda a, t: orc.l1_prox(a, t * lam)
    l21s = lambda a, t: orc.l21_prox(a, t * lam, sh)
    assert rel_err(orc.fenchel_prox(l1s, x, 1.3), g["l1_fprox"]) <= _tol(x)
    assert rel_err(orc.fenchel_prox(l21s, x, 1.3), g["l21_fprox"]) <= _tol(x)
    assert rel_err(orc.moreau_grad(lambda a, t: orc.l21_prox(a, t, sh), x, 0.3), g["l21_moreau_grad"]) <= _tol(x)
    assert rel_err(orc.l21_apply(x, sh), g["l21_apply"]) <= _tol(x)
    np.testing.assert_array_equal(orc.positive_orthant_prox(x), g["po_prox"])


def test_known_answers_reference_tests():
    # src/pyxu_tests/operator/func/test_norm.py:36-74 (L1) and :376-414 (L21)
    x = np.array([-3.0, -2, -1, 0, 1])
    np.testing.assert_allclose(orc.l1_prox(x, 1.0), [-2, -1, 0, 0, 0])
    x = np.array([1.0, 2, -3, 0, -2, -4])
    np.testing.assert_allclose(orc.l21_apply(x, (2, 3)), [6 + 2 * np.sqrt(2)])
    np.testing.assert_allclose(orc.l21_prox(x, 4.0, (2, 3)), [0, 0, -3 / 5, 0, 0, -4 / 5], atol=1e-12)


def _deblur(g, dt):
    sh = tuple(g["arg_shape"])
    taps, c = orc.gaussian_taps(float(g["sigma"]), 3.0, dt)
    return dict(arg_shape=sh, kernel=[taps] * len(sh), center=[c] * len(sh), mode="constant")


@pytest.mark.parametrize("name", golden_names("pgd_") )
def test_pgd_trajectory(name):
    g = load_golden(name)
    if name.startswith("pgd_stacked"):
        dt = g["x0"].dtype
        blur = _deblur(g, dt)
        grad = lambda v: orc.deblur_tv_grad(v, blur, g["y"], 0, 0, None)
        prox = lambda z, t: orc.l1_prox(z, t * float(g["lam"]))
        x, _ = orc.pgd(g["x0"], grad, prox, dt.type(1 / dt.type(1.0)), 20)
        assert rel_err(x, g["x_20"]) <= 1e-6
        return
    dt = g["x0"].dtype
    sh = tuple(g["arg_shape"])
    blur = _deblur(g, dt)
    lam, mu = float(g["lam"]), float(g["mu"])
    variant = name.split("_")[1] if "tv_l1g" not in name else "tv_l1g"
    gk = dict(arg_shape=sh)
    if variant == "l1":
        grad = lambda v: orc.deblur_tv_grad(v, blur, g["y"], 0, 0, None)
    else:
        grad = lambda v: orc.deblur_tv_grad(v, blur, g["y"], lam, mu, gk)
    if variant == "tv":
        prox = lambda z, t: orc.positive_orthant_prox(z)
    else:
        prox = lambda z, t: orc.l1_prox(z, t * lam)
    tau = dt.type(1 / dt.type(float(g["diff_lipschitz"])))
    for n in (1, 10, 100):
        x, xp, hist = orc.pgd(g["x0"], grad, prox, tau, n, history=True)
        assert rel_err(x, g[f"x_{n}"]) <= _tol(x) * 10, n
        np.testing.assert_allclose(np.array(hist).ravel(), g[f"hist_{n}"][1:], rtol=1e-4)


@pytest.mark.parametrize("name", golden_names("pds_"))
def test_pds_trajectory(name):
    g = load_golden(name)
    dt = g["x0"].dtype
    sh = tuple(g["arg_shape"])
    D = len(sh)
    lam = float(g["lam"])
    blur = _deblur(g, dt)
    grad_f = lambda v: orc.deblur_tv_grad(v, blur, g["y"], 0, 0, None)
    K = lambda v: orc.gradient_apply(v, sh)
    KT = lambda v: orc.gradient_adjoint(v, sh)
    if name.startswith("pds_iso"):
        prox_h = lambda a, t: orc.l21_prox(a, t * lam, (D, *sh))
    else:
        prox_h = lambda a, t: orc.l1_prox(a, t * lam)
    fprox = lambda a, s: orc.fenchel_prox(prox_h, a, s)
    Lk = float(g["K_lipschitz"])
    tau, sigma, _, rho = orc.pd3o_step_sizes(1.0, Lk, dt)
    assert tau == g["pd3o_tau"] and sigma == g["pd3o_sigma"]
    tcv, scv, _, rcv = orc.condat_vu_step_sizes(1.0, Lk, dt)
    assert tcv == g["cv_tau"] and scv == g["cv_sigma"]
    for n in (1, 10, 100):
        x, z, _ = orc.pd3o(g["x0"], grad_f, None, K, KT, fprox, tau, sigma, rho, n)
        assert rel_err(x, g[f"pd3o_x_{n}"]) <= _tol(x) * 10, n
        assert rel_err(z, g[f"pd3o_z_{n}"]) <= _tol(x) * 10, n
        x, z = orc.condat_vu(g["x0"], grad_f, None, K, KT, fprox, tcv, scv, rcv, n)
        assert rel_err(x, g[f"cv_x_{n}"]) <= _tol(x) * 10, n
        assert rel_err(z, g[f"cv_z_{n}"]) <= _tol(x) * 10, n


@pytest.mark.parametrize("name", golden_names("admm_"))
def test_admm_trajectory(name):
    g = load_golden(name)
    dt = g["x0"].dtype
    tol = 2e-5 if dt == np.float32 else 1e-10
    for n in (1, 5, 30):
        x, u, z, _ = orc.admm_dense_l1(g["A"], g["y"], float(g["lam"]), g["x0"], float(g["tau"]), n)
        assert rel_err(x, g[f"x_{n}"]) <= tol, n
        assert rel_err(u, g[f"u_{n}"]) <= tol, n


def _diffop_args(g):
    d = g["directions"]
    directions = None if (d.ndim == 0 and int(d) == -1) else (int(d) if d.ndim == 0 else tuple(int(v) for v in d))
    return str(g["kind"]), tuple(int(v) for v in g["arg_shape"]), directions, str(g["scheme"]) or None


@pytest.mark.parametrize("name", golden_names("diffop_"))
def test_diffops(name):
    """Divergence / Laplacian / Hessian restatements vs the reference's own outputs (diff.py:1418-1936)."""
    g = load_golden(name)
    kind, sh, directions, scheme = _diffop_args(g)
    if kind == "divergence":
        kw = dict(directions=directions, scheme=scheme or "central")
        y, a = orc.divergence_apply(g["x"], sh, **kw), orc.divergence_adjoint(g["z"], sh, **kw)
    elif kind == "laplacian":
        y = orc.laplacian_apply(g["x"], sh)
        a = orc.laplacian_apply(g["z"], sh)  # the central second differences are symmetric
    else:
        dirs = "all" if directions is None else directions
        y, a = orc.hessian_apply(g["x"], sh, dirs), orc.hessian_adjoint(g["z"], sh, dirs)
    assert rel_err(y, g["y"]) <= _tol(y)
    assert rel_err(a, g["adj"]) <= _tol(a)


@pytest.mark.parametrize("name", golden_names("directional_"))
def test_directional(name):
    """Jacobian, Gaussian-derivative Gradient / Hessian / Laplacian / Divergence and the directional
    family restated on the oracle vs the reference's own outputs (diff.py:264-350, 1268-1416, 1938-2759)."""
    from _directional import case, oracle_fns

    g = load_golden(name)
    assert str(g["raises"]) == "", str(g["raises"])
    kind, kw = case(g)
    ap, ad = oracle_fns(kind, kw, g["x"].dtype)
    y, a = ap(g["x"]), ad(g["z"])
    assert rel_err(y, g["y"]) <= _tol(y), (kind, rel_err(y, g["y"]))
    assert rel_err(a, g["adj"]) <= _tol(a), (kind, rel_err(a, g["adj"]))
