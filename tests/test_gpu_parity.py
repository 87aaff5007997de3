"""
GPU parity: every hot-path operator / solver of pyxu_amd (HIP C-ABI) against the goldens recorded
from the reference and against the CPU oracle on the same seeded inputs.

Tolerances (north_star: 1e-5 relative in fp32): norm-wise relative error <= 1e-5 (fp32) or
1e-12 (fp64) for operators; trajectories after 100 iterations <= 1e-5 (fp32) / 1e-10 (fp64);
supports of the prox outputs identical outside the ulp tie band.
"""
import numpy as np
import pytest

import oracle as orc
from conftest import golden_names, load_golden, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd  # noqa: E402
import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402

OP_TOL = {np.float32: 1e-5, np.float64: 1e-12}
TRAJ_TOL = {np.float32: 1e-5, np.float64: 1e-10}


def W(dt):
    return pxrt.Width.SINGLE if np.dtype(dt) == np.float32 else pxrt.Width.DOUBLE


def D(a):
    return to_device(np.ascontiguousarray(a))


def test_native_library_is_the_compute_path():
    assert pyxu_amd.native_loaded()
    assert pyxu_amd.lib.pxa_version().decode().startswith("pyxu_amd")


# ----------------------------------------------------------------------------- operators vs goldens
def _kern(g):
    ks = [g[f"kernel{i}"] for i in range(int(g["n_kernels"]))]
    return ks if bool(g["separable"]) else ks[0]


def _mode(g):
    m = g["mode"]
    return str(m) if m.ndim == 0 else tuple(str(s) for s in m)


@pytest.mark.parametrize("name", golden_names("stencil_"))
def test_stencil_golden(name):
    g = load_golden(name)
    dt = g["x"].dtype.type
    with pxrt.Precision(W(dt)):
        op = pxo.Stencil(arg_shape=tuple(g["arg_shape"]), kernel=_kern(g), center=tuple(g["center"]), mode=_mode(g))
        y = to_NUMPY(op.apply(D(g["x"])))
        a = to_NUMPY(op.adjoint(D(g["z"])))
        assert np.isclose(float(op.lipschitz), float(g["lipschitz"]), rtol=1e-6)
    assert y.shape == g["y"].shape and y.dtype == g["y"].dtype
    assert rel_err(y, g["y"]) <= OP_TOL[dt]
    assert rel_err(a, g["adj"]) <= OP_TOL[dt]


@pytest.mark.parametrize("name", golden_names("gaussian_"))
def test_gaussian_golden(name):
    g = load_golden(name)
    dt = g["x"].dtype.type
    with pxrt.Precision(W(dt)):
        op = pxo.Gaussian(arg_shape=tuple(g["arg_shape"]), sigma=float(g["sigma"]), truncate=float(g["truncate"]))
        np.testing.assert_array_equal(op.kernel[0], g["taps"])
        assert rel_err(to_NUMPY(op.apply(D(g["x"]))), g["y"]) <= OP_TOL[dt]
        assert rel_err(to_NUMPY(op.adjoint(D(g["z"]))), g["adj"]) <= OP_TOL[dt]


@pytest.mark.parametrize("name", golden_names("convolve_"))
def test_convolve_golden(name):
    g = load_golden(name)
    dt = g["x"].dtype.type
    with pxrt.Precision(W(dt)):
        op = pxo.Convolve(arg_shape=tuple(g["arg_shape"]), kernel=[g["kernel0"], g["kernel1"]], center=tuple(g["center"]))
        assert rel_err(to_NUMPY(op.apply(D(g["x"]))), g["y"]) <= OP_TOL[dt]
        assert rel_err(to_NUMPY(op.adjoint(D(g["z"]))), g["adj"]) <= OP_TOL[dt]


@pytest.mark.parametrize("name", golden_names("gradient_"))
def test_gradient_golden(name):
    g = load_golden(name)
    dt = g["x"].dtype.type
    with pxrt.Precision(W(dt)):
        op = pxo.Gradient(arg_shape=tuple(g["arg_shape"]), directions=tuple(g["directions"]), mode=str(g["mode"]),
                          scheme=str(g["scheme"]), accuracy=int(g["accuracy"]), sampling=float(g["sampling"]))
        assert rel_err(to_NUMPY(op.apply(D(g["x"]))), g["y"]) <= OP_TOL[dt]
        assert rel_err(to_NUMPY(op.adjoint(D(g["z"]))), g["adj"]) <= OP_TOL[dt]
        assert np.isclose(float(op.lipschitz), float(g["lipschitz"]), rtol=1e-6)


@pytest.mark.parametrize("name", golden_names("norms_"))
def test_norms_golden(name):
    g = load_golden(name)
    dt = g["x"].dtype.type
    x = D(g["x"])
    sh = tuple(g["arg_shape"])
    N = int(np.prod(sh))
    lam = float(g["lam"])
    with pxrt.Precision(W(dt)):
        l1, l21 = pxo.L1Norm(dim=N), pxo.L21Norm(arg_shape=sh, l2_axis=(0,))
        sl2, po = pxo.SquaredL2Norm(dim=N), pxo.PositiveOrthant(dim=N)
        out = {
            "l1_apply": l1.apply(x), "l1_prox": l1.prox(x, 0.8), "l1_fprox": (lam * l1).fenchel_prox(x, 1.3),
            "l21_apply": l21.apply(x), "l21_prox": l21.prox(x, 0.8), "l21_fprox": (lam * l21).fenchel_prox(x, 1.3),
            "l21_moreau_grad": l21.moreau_envelope(0.3).grad(x), "l21_moreau_apply": l21.moreau_envelope(0.3).apply(x),
            "sl2_apply": sl2.apply(x), "sl2_grad": sl2.grad(x), "sl2_prox": sl2.prox(x, 0.8), "po_prox": po.prox(x, 0.8),
        }
    for k, v in out.items():
        v = to_NUMPY(v)
        assert v.shape == g[k].shape, k
        assert rel_err(v, g[k]) <= OP_TOL[dt] * 10, k
    # exact zero-sets for the thresholding proxes (no ties in these random inputs)
    for k in ("l1_prox", "l21_prox", "po_prox"):
        np.testing.assert_array_equal(to_NUMPY(out[k]) == 0, g[k] == 0)


@pytest.mark.parametrize("name", golden_names("dense_"))
def test_dense_golden(name):
    g = load_golden(name)
    dt = g["x"].dtype.type
    with pxrt.Precision(W(dt)):
        op = pxa.LinOp.from_array(D(g["A"]))
        assert rel_err(to_NUMPY(op.apply(D(g["x"]))), g["y"]) <= OP_TOL[dt] * 10
        assert rel_err(to_NUMPY(op.adjoint(D(g["z"]))), g["adj"]) <= OP_TOL[dt] * 10


# MFMA paths: the register-streamed kernel (B < 32, or rows not in whole 16-B chunks) and the LDS-staged
# kernel (B >= 32: 64- and 128-row workgroup tiles, several P tiles at B = 161, ragged P / Q, split-K)
@pytest.mark.parametrize("B", [2, 9, 32, 33, 64, 100, 128, 161])
@pytest.mark.parametrize("MN", [(96, 640), (300, 1030), (260, 1028), (2048, 4096)])
def test_dense_mfma_vs_fp64(MN, B):
    """fp32 matrix-core path of _ExplicitLinOp (B >= 2 stacked inputs) vs an fp64 host product.
    fp32 sums over K terms carry ~sqrt(K) eps inherent error: norm-wise 1e-5."""
    M, N = MN
    rng = np.random.default_rng(M + B)
    A = rng.standard_normal((M, N)).astype(np.float32)
    X = rng.standard_normal((B, N)).astype(np.float32)
    Z = rng.standard_normal((B, M)).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        op = pxa.LinOp.from_array(D(A))
        y = to_NUMPY(op.apply(D(X)))
        z = to_NUMPY(op.adjoint(D(Z)))
    A64 = A.astype(np.float64)
    assert rel_err(y, X.astype(np.float64) @ A64.T) <= 1e-5
    assert rel_err(z, Z.astype(np.float64) @ A64) <= 1e-5
    # stacked rows are independent: row b equals the single-RHS (GEMV path) product
    with pxrt.Precision(pxrt.Width.SINGLE):
        y1 = to_NUMPY(op.apply(D(X[-1])))
    assert rel_err(y[-1], y1) <= 1e-5


@pytest.mark.parametrize("trans", [0, 1])
def test_dense_lds_kernel_matches_register_kernel(trans):
    """PXA_TUNE_DENSE_KERNEL A/B: the LDS-staged MFMA kernel and the register-streamed one compute the same
    product (fp32, different summation split): norm-wise 1e-6 apart, both within 1e-5 of fp64."""
    M, N, B = 1024, 8192, 128
    rng = np.random.default_rng(9)
    A = rng.standard_normal((M, N)).astype(np.float32)
    X = rng.standard_normal((B, M if trans else N)).astype(np.float32)
    Ad, Xd = D(A), D(X)
    out = {}
    for knob in (0, 1):
        prev = _dev.tuning(_dev.TUNE_DENSE_KERNEL, knob)
        try:
            out[knob] = to_NUMPY(_dev.dense_matmat(Ad, Xd, trans))
        finally:
            _dev.tuning(_dev.TUNE_DENSE_KERNEL, prev)
    ref = X.astype(np.float64) @ (A.astype(np.float64) if trans else A.astype(np.float64).T)
    assert rel_err(out[0], ref) <= 1e-5 and rel_err(out[1], ref) <= 1e-5
    assert rel_err(out[0], out[1]) <= 1e-6


# ----------------------------------------------------------------------------- solver trajectories
def _deblur_f(g, dt, sh, lam=None, mu=None):
    N = int(np.prod(sh))
    H = pxo.Gaussian(arg_shape=sh, sigma=float(g["sigma"]), truncate=3.0)
    f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(g["y"])) * H
    if lam:
        f = f + lam * pxo.L21Norm(arg_shape=(len(sh), *sh)).moreau_envelope(mu) * pxo.Gradient(arg_shape=sh)
    return f


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", [n for n in golden_names("pgd_") if "stacked" not in n])
def test_pgd_trajectory_golden(name, fused):
    g = load_golden(name)
    dt = g["x0"].dtype.type
    sh = tuple(g["arg_shape"])
    N = int(np.prod(sh))
    lam, mu = float(g["lam"]), float(g["mu"])
    variant = "tv_l1g" if "tv_l1g" in name else name.split("_")[1]
    with pxrt.Precision(W(dt)):
        f = _deblur_f(g, dt, sh, None if variant == "l1" else lam, mu)
        g_ = pxo.PositiveOrthant(dim=N) if variant == "tv" else lam * pxo.L1Norm(dim=N)
        f.diff_lipschitz = float(g["diff_lipschitz"])
        for n in (1, 10, 100):
            s = pxs.PGD(f=f, g=g_, show_progress=False)
            s.fit(x0=D(g["x0"]), stop_crit=pxst.MaxIter(n), fused=fused)
            assert (s._plan is not None) == fused
            x = to_NUMPY(s.solution())
            assert x.dtype == g[f"x_{n}"].dtype
            assert rel_err(x, g[f"x_{n}"]) <= TRAJ_TOL[dt], (n, rel_err(x, g[f"x_{n}"]))


def test_pgd_stacked_golden():
    g = load_golden("pgd_stacked_f32")
    sh = tuple(g["arg_shape"])
    N = int(np.prod(sh))
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=float(g["sigma"]))
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(g["y"])) * H
        f.diff_lipschitz = 1.0
        for fused in (True, False):
            s = pxs.PGD(f=f, g=float(g["lam"]) * pxo.L1Norm(dim=N), show_progress=False)
            s.fit(x0=D(g["x0"]), stop_crit=pxst.MaxIter(20), fused=fused)
            assert rel_err(to_NUMPY(s.solution()), g["x_20"]) <= 1e-5


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", golden_names("pds_"))
def test_pds_trajectory_golden(name, fused):
    g = load_golden(name)
    dt = g["x0"].dtype.type
    sh = tuple(g["arg_shape"])
    Dd = len(sh)
    N = int(np.prod(sh))
    lam = float(g["lam"])
    with pxrt.Precision(W(dt)):
        f = _deblur_f(g, dt, sh)
        f.diff_lipschitz = float(g["diff_lipschitz"])
        K = pxo.Gradient(arg_shape=sh)
        h = lam * (pxo.L21Norm(arg_shape=(Dd, *sh)) if name.startswith("pds_iso") else pxo.L1Norm(dim=Dd * N))
        for key, klass in (("pd3o", pxs.PD3O), ("cv", pxs.CondatVu)):
            for n in (1, 10, 100):
                s = klass(f=f, g=None, h=h, K=K, show_progress=False)
                s.fit(x0=D(g["x0"]), stop_crit=pxst.MaxIter(n), fused=fused)
                assert (s._plan is not None) == fused
                assert s._mstate["tau"] == g[f"{key}_tau"] and s._mstate["sigma"] == g[f"{key}_sigma"]
                data, _ = s.stats()
                assert rel_err(to_NUMPY(data["x"]), g[f"{key}_x_{n}"]) <= TRAJ_TOL[dt], (key, n)
                assert rel_err(to_NUMPY(data["z"]), g[f"{key}_z_{n}"]) <= TRAJ_TOL[dt], (key, n)


@pytest.mark.parametrize("name", golden_names("admm_"))
def test_admm_trajectory_golden(name):
    g = load_golden(name)
    dt = g["x0"].dtype.type
    M, N = g["A"].shape
    tol = 2e-5 if dt == np.float32 else 1e-9
    with pxrt.Precision(W(dt)):
        K = pxa.LinOp.from_array(D(g["A"]))
        f = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(D(g["y"])) * K
        h = float(g["lam"]) * pxo.L1Norm(dim=N)
        for n in (1, 5, 30):
            s = pxs.ADMM(f=f, h=h, show_progress=False)
            s.fit(x0=D(g["x0"]), tau=float(g["tau"]), stop_crit=pxst.MaxIter(n))
            data, _ = s.stats()
            assert rel_err(to_NUMPY(data["x"]), g[f"x_{n}"]) <= tol, n
            assert rel_err(to_NUMPY(data["u"]), g[f"u_{n}"]) <= tol, n


# ----------------------------------------------------------------------------- oracle parity, odd sizes / edges
@pytest.mark.parametrize("sh", [(1, 1), (3, 5), (31, 65), (65, 31), (100, 257)])
@pytest.mark.parametrize("stack", [1, 3])
def test_fused_pgd_edges_vs_oracle(sh, stack):
    rng = np.random.default_rng(sum(sh) + stack)
    N = int(np.prod(sh))
    y = rng.standard_normal(N).astype(np.float32)
    x0 = rng.uniform(0, 1, (stack, N)).astype(np.float32) if stack > 1 else rng.uniform(0, 1, N).astype(np.float32)
    lam, mu = 0.05, 0.02
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=1.5)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(y)) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * pxo.Gradient(arg_shape=sh)
        f.diff_lipschitz = 1 + 8 * lam / mu
        s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=N), show_progress=False)
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(5))
        assert s._plan is not None
        x = to_NUMPY(s.solution())
    taps, c = orc.gaussian_taps(1.5, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
    ref, _ = orc.pgd(x0, grad, lambda z, t: orc.positive_orthant_prox(z), np.float32(1 / np.float32(f.diff_lipschitz)), 5)
    assert rel_err(x, ref) <= 1e-5


@pytest.mark.parametrize("sigma", [0.3, 1.0, 2.5])  # blur radius R = 1, 3, 8 (the kernel's range)
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("sh", [(7, 12), (40, 68), (70, 131)])  # n < 2R, one tile, ragged multi-tile
def test_fused_pgd_radius_dtype_vs_oracle(sigma, dt, sh):
    """Normal-operator kernel (H^T H yk - H^T y) incl. its boundary-row corrections, every radius."""
    rng = np.random.default_rng(int(10 * sigma) + sh[0])
    N = int(np.prod(sh))
    y = rng.standard_normal(N).astype(dt)
    x0 = rng.uniform(0, 1, N).astype(dt)
    lam, mu = 0.05, 0.02
    with pxrt.Precision(W(dt)):
        H = pxo.Gaussian(arg_shape=sh, sigma=sigma)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(y)) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * pxo.Gradient(arg_shape=sh)
        f.diff_lipschitz = 1 + 8 * lam / mu
        s = pxs.PGD(f=f, g=0.01 * pxo.L1Norm(dim=N), show_progress=False)
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(6))
        assert s._plan is not None
        x = to_NUMPY(s.solution())
    taps, c = orc.gaussian_taps(sigma, 3.0, dt)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
    tau = dt(1 / dt(f.diff_lipschitz))
    ref, _ = orc.pgd(x0, grad, lambda z, t: orc.l1_prox(z, t * dt(0.01)), tau, 6)
    assert rel_err(x, ref) <= (1e-5 if dt == np.float32 else 1e-12)


def test_batch_as_axis_fused_matches_per_image():
    """(B, n0, n1) with identity taps on axis 0 and Gradient(directions=(1,2)) == B independent images."""
    rng = np.random.default_rng(7)
    B, sh = 4, (40, 52)
    N = int(np.prod(sh))
    ys = rng.standard_normal((B, N)).astype(np.float32)
    lam, mu = 0.02, 0.01
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=(B, *sh), sigma=(0, 2.0, 2.0))
        G = pxo.Gradient(arg_shape=(B, *sh), directions=(1, 2))
        f = 0.5 * pxo.SquaredL2Norm(dim=B * N).asloss(D(ys.reshape(-1))) * H + lam * pxo.L21Norm(arg_shape=(2, B, *sh)).moreau_envelope(mu) * G
        f.diff_lipschitz = 1 + 8 * lam / mu
        res = {}
        for fused in (True, False):
            s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=B * N), show_progress=False)
            s.fit(x0=D(np.zeros(B * N, np.float32)), stop_crit=pxst.MaxIter(8), fused=fused)
            assert (s._plan is not None) == fused
            res[fused] = to_NUMPY(s.solution())
    assert rel_err(res[True], res[False]) <= 1e-5
    taps, c = orc.gaussian_taps(2.0, 3.0, np.float32)
    for b in range(B):
        blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
        grad = lambda v: orc.deblur_tv_grad(v, blur, ys[b], lam, mu, dict(arg_shape=sh))
        ref, _ = orc.pgd(np.zeros(N, np.float32), grad, lambda z, t: orc.positive_orthant_prox(z),
                         np.float32(1 / np.float32(1 + 8 * lam / mu)), 8)
        assert rel_err(res[True][b * N:(b + 1) * N], ref) <= 1e-5


# ----------------------------------------------------------------------------- full-size properties
def test_adjoint_identity_full_size():
    """<A x, z> = <x, A^T z> at the benchmark size (2048^2) for the blur and the gradient."""
    rng = np.random.default_rng(3)
    sh = (2048, 2048)
    N = int(np.prod(sh))
    with pxrt.Precision(pxrt.Width.DOUBLE):
        for op in (pxo.Gaussian(arg_shape=sh, sigma=2.0), pxo.Gradient(arg_shape=sh)):
            x = D(rng.standard_normal(N))
            z = D(rng.standard_normal(op.codim))
            lhs = float((op.apply(x) * z).sum().cpu())
            rhs = float((x * op.adjoint(z)).sum().cpu())
            assert abs(lhs - rhs) <= 1e-10 * max(abs(lhs), 1.0)


def test_fused_step_matches_generic_full_size():
    """One fused PGD-TV step at 2048^2 equals the rule-by-rule HIP path (independent kernels)."""
    rng = np.random.default_rng(4)
    sh = (2048, 2048)
    N = int(np.prod(sh))
    lam, mu = 0.01, 0.01
    with pxrt.Precision(pxrt.Width.SINGLE):
        y = D(rng.standard_normal(N).astype(np.float32))
        x0 = D(rng.uniform(0, 1, N).astype(np.float32))
        H = pxo.Gaussian(arg_shape=sh, sigma=2.0)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * pxo.Gradient(arg_shape=sh)
        f.diff_lipschitz = 1 + 8 * lam / mu
        res = {}
        for fused in (True, False):
            s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=N), show_progress=False)
            s.fit(x0=x0, stop_crit=pxst.MaxIter(3), fused=fused)
            res[fused] = to_NUMPY(s.solution())
    assert rel_err(res[True], res[False]) <= 1e-5


def test_xp_shim_numpy_semantics():
    """NDArrayInfo.MI355X.module(): NumPy-named functions computed by the HIP kernels."""
    from pyxu_amd.info.deps import NDArrayInfo

    xp = NDArrayInfo.MI355X.module()
    rng = np.random.default_rng(9)
    a = rng.standard_normal((3, 257)).astype(np.float32)
    t = D(a)
    np.testing.assert_array_equal(to_NUMPY(xp.fabs(t)), np.fabs(a))
    np.testing.assert_array_equal(to_NUMPY(xp.fmax(t, 0.25)), np.fmax(a, np.float32(0.25)))
    np.testing.assert_array_equal(to_NUMPY(xp.fmin(t, 0.25)), np.fmin(a, np.float32(0.25)))
    np.testing.assert_array_equal(to_NUMPY(xp.clip(t, -0.5, 0.5)), np.clip(a, -0.5, 0.5))
    for ord_ in (None, 1, np.inf):
        ref = np.linalg.norm(a.astype(np.float64), ord=ord_, axis=-1, keepdims=True)
        assert rel_err(to_NUMPY(xp.linalg.norm(t, ord=ord_, axis=-1, keepdims=True)), ref) <= 1e-6
    assert NDArrayInfo.from_obj(t) is NDArrayInfo.MI355X


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_row_ratio_bits(dt):
    """pxa_row_ratio: (dtype)(num / den) in float64 on the device == the host's numpy division + cast
    (the CG alpha / beta of cg.py:125-153), bit for bit, incl. a zero denominator."""
    from pyxu_amd import _dev

    rng = np.random.default_rng(3)
    num = np.abs(rng.standard_normal(1000)) * 10.0 ** rng.integers(-30, 30, 1000)
    den = np.abs(rng.standard_normal(1000)) * 10.0 ** rng.integers(-30, 30, 1000)
    den[7] = 0.0
    like = D(np.zeros(1, dtype=dt))
    out = to_NUMPY(_dev.row_ratio(D(num), D(den), like))
    with np.errstate(divide="ignore", over="ignore"):  # f32 overflow -> inf on both sides
        ref = (num / den).astype(dt)
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("rows", [1, 3])
def test_cg_stacked_vs_oracle(rows):
    """CG (opt/solver/cg.py:72-165) on an SPD dense operator, single and stacked right-hand sides
    (per-row alpha / beta through pxa_axpy_rows), fp64, against the oracle's restatement."""
    rng = np.random.default_rng(7 + rows)
    N = 96
    Kh = rng.standard_normal((64, N))
    Ah = Kh.T @ Kh + 0.5 * np.eye(N)
    b = rng.standard_normal((rows, N)) if rows > 1 else rng.standard_normal(N)
    with pxrt.Precision(pxrt.Width.DOUBLE):
        A = pxa.LinOp.from_array(D(Ah))
        s = pxs.CG(A=A, show_progress=False)
        s.fit(b=D(b), stop_crit=pxst.MaxIter(200) | pxst.AbsError(eps=1e-4, var="residual", f=None, norm=2, satisfy_all=True))
        x = to_NUMPY(s.solution())
    ref, _ = orc.cg(lambda v: v @ Ah.T, b, eps=1e-4, max_iter=200)
    assert rel_err(x, ref) <= 1e-7  # fp64; CG amplifies reduction-order rounding (kappa ~ 600)
    assert rel_err(x, np.linalg.solve(Ah, b.T).T) <= 1e-3


@pytest.mark.parametrize("name", golden_names("diffop_"))
def test_diffop_golden(name):
    """Divergence / Laplacian / Hessian (diff.py:1418-1936) through the HIP stencil path vs the
    reference's own outputs (tests/golden/make_goldens.py gen_diffops)."""
    g = load_golden(name)
    dt = g["x"].dtype.type
    kind = str(g["kind"])
    sh = tuple(int(v) for v in g["arg_shape"])
    d = g["directions"]
    directions = None if (d.ndim == 0 and int(d) == -1) else (int(d) if d.ndim == 0 else tuple(int(v) for v in d))
    with pxrt.Precision(W(dt)):
        if kind == "divergence":
            kw = {"scheme": str(g["scheme"])} if str(g["scheme"]) else {}
            op = pxo.Divergence(arg_shape=sh, directions=directions, **kw)
        elif kind == "laplacian":
            op = pxo.Laplacian(arg_shape=sh)
        else:
            op = pxo.Hessian(arg_shape=sh, directions="all" if directions is None else directions)
        assert op.shape == (g["y"].shape[-1], g["x"].shape[-1])
        assert rel_err(to_NUMPY(op.apply(D(g["x"]))), g["y"]) <= OP_TOL[dt]
        assert rel_err(to_NUMPY(op.adjoint(D(g["z"]))), g["adj"]) <= OP_TOL[dt]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(1,), (7,), (4096 * 3 + 5,), (3, 1000), (2, 1, 2048 * 2048 // 64)])
def test_relerr_stats_one_pass(shape, dtype):
    """pxa_relerr_stats == (row_reduce DIFFSQ, row_reduce SUMSQ) bit for bit, the copy == x, and the
    statistics match an fp64 NumPy restatement of RelError (stop.py:365-371)."""
    from pyxu_amd import _dev

    rng = np.random.default_rng(5)
    x = rng.standard_normal(shape).astype(dtype)
    p = rng.standard_normal(shape).astype(dtype)
    xd, pd = to_device(x), to_device(p)
    rows = int(np.prod(shape[:-1])) if len(shape) > 1 else 1
    st = _dev.empty_f64((2, rows), xd)
    xc = _dev.relerr_stats(xd, pd, st)
    a = _dev.row_reduce(_dev.RED_DIFFSQ, xd.reshape(-1, shape[-1]), pd.reshape(-1, shape[-1]))
    b = _dev.row_reduce(_dev.RED_SUMSQ, pd.reshape(-1, shape[-1]))
    got = to_NUMPY(st)
    assert np.array_equal(got[0], to_NUMPY(a).reshape(-1)) and np.array_equal(got[1], to_NUMPY(b).reshape(-1))
    assert np.array_equal(to_NUMPY(xc), x) and xc.data_ptr() != xd.data_ptr()
    x2, p2 = x.reshape(rows, -1).astype(np.float64), p.reshape(rows, -1).astype(np.float64)
    assert np.allclose(got[0], ((x2 - p2) ** 2).sum(-1), rtol=1e-12)
    assert np.allclose(got[1], (p2**2).sum(-1), rtol=1e-12)
