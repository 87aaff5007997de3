"""
Long trajectories on the INTERIOR tile paths the bench times (VERDICT r02 "parity depth"): 100 PGD
iterations at 512^2 (interior tiles of pgd_tv2d_kernel<float, 6>) and 20 PD3O / Condat-Vu iterations at
128^3 (interior march + plane tiles), compared with the oracle's restatement of the reference m_step
(oracle/pyxu_np.py, pinned to the reference goldens by tests/test_oracle_golden.py) at checkpoints.

The fused kernels round differently from the reference's NumPy order (the normal-operator form
G yk - H^T y, __builtin_amdgcn_rsqf for 1/|v|, fma in the momentum / update), so drift over a realistic run
is what this pins.  Tolerances (north_star): norm-wise relative error <= 1e-5 in fp32 at EVERY checkpoint;
prox zero-sets identical outside the fp32 tie band (an entry may be zero on one side only if the other
side's value is within 1e-6 of the iterate's max-abs).
"""
import numpy as np
import pytest

import oracle as orc
from conftest import rel_err
from test_gpu_bench_shapes import D, _blurred, zero_set_ok

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
from pyxu_amd.util import to_NUMPY  # noqa: E402

TOL = 1e-5
PGD_CHECKS = (1, 10, 50, 100)
PDS_CHECKS = (1, 10, 20)


@pytest.mark.parametrize("g_kind", ["pos", "l1"])
def test_pgd_tv_512_100_iterations(g_kind):
    """PGD 512^2: Gaussian(sigma=2) deblur + 0.01 env_0.01(L21 o Grad) TV with g = PositiveOrthant or
    0.01 L1; 100 iterations of the fused one-launch step, checked at k = 1, 10, 50, 100."""
    sh = (512, 512)
    N = sh[0] * sh[1]
    lam, mu, gw = 0.01, 0.01, 0.01
    rng = np.random.default_rng(77)
    y, blur = _blurred(sh, 2.0, rng)
    got = {}
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=2.0)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(y)) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * pxo.Gradient(arg_shape=sh)
        L = 1.0 + 8 * lam / mu
        f.diff_lipschitz = L
        g = pxo.PositiveOrthant(dim=N) if g_kind == "pos" else gw * pxo.L1Norm(dim=N)
        s = pxs.PGD(f=f, g=g, show_progress=False)
        s.fit(x0=D(np.zeros(N, np.float32)), stop_crit=pxst.MaxIter(max(PGD_CHECKS)), mode=pxa.Mode.MANUAL)
        assert s._plan is not None
        for k, _ in enumerate(s.steps(), start=1):
            if k in PGD_CHECKS:
                got[k] = to_NUMPY(_dev.copy(s._mstate["x"]))
    snap = dict.fromkeys(PGD_CHECKS)
    grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
    prox = (lambda z, t: orc.positive_orthant_prox(z)) if g_kind == "pos" else (lambda z, t: orc.l1_prox(z, t * np.float32(gw)))
    orc.pgd(np.zeros(N, np.float32), grad, prox, np.float32(1 / np.float32(L)), max(PGD_CHECKS), snap=snap)
    for k in PGD_CHECKS:
        err = rel_err(got[k], snap[k])
        assert err <= TOL, (k, err)
        assert zero_set_ok(got[k], snap[k]), k


@pytest.mark.parametrize("algo", ["pd3o", "cv"])
def test_pds_aniso_tv_128cube_20_iterations(algo):
    """PD3O / Condat-Vu at 128^3 (Gaussian(sigma=2) blur + 0.01 L1 o Grad, g = None), 20 iterations of the
    solver's default fused step (the look-ahead step, pxa_pds_step_la: kernel B + kernel D per iteration),
    x and z checked at k = 1, 10, 20."""
    sh = (128, 128, 128)
    N = int(np.prod(sh))
    lam = 0.01
    rng = np.random.default_rng(5)
    y, blur = _blurred(sh, 2.0, rng)
    x0 = np.zeros(N, np.float32)
    got = {}
    with pxrt.Precision(pxrt.Width.SINGLE):
        S = pxo.Stencil(arg_shape=sh, kernel=blur["kernel"], center=blur["center"], mode="constant")
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(y)) * S
        f.diff_lipschitz = 1.0
        K = pxo.Gradient(arg_shape=sh)
        h = lam * pxo.L1Norm(dim=3 * N)
        cls = pxs.PD3O if algo == "pd3o" else pxs.CondatVu
        s = cls(f=f, h=h, K=K, show_progress=False)
        s.fit(x0=D(x0), stop_crit=pxst.MaxIter(max(PDS_CHECKS)), mode=pxa.Mode.MANUAL)
        assert s._plan is not None, "fused PDS step not selected"
        tau, sigma_, rho = s._mstate["tau"], s._mstate["sigma"], s._mstate["rho"]
        for k, _ in enumerate(s.steps(), start=1):
            if k in PDS_CHECKS:
                got[k] = (to_NUMPY(_dev.copy(s._mstate["x"])), to_NUMPY(_dev.copy(s._mstate["z"])))
    grad_f = lambda v: orc.deblur_tv_grad(v, blur, y, 0.0, 1.0, dict(arg_shape=sh))
    Kf = lambda v: orc.gradient_apply(v, arg_shape=sh)
    KT = lambda v: orc.gradient_adjoint(v, arg_shape=sh)
    hp = lambda v, t: orc.l1_prox(v, t * np.float32(lam))
    fprox = lambda v, s_: orc.fenchel_prox(hp, v, s_)
    snap = dict.fromkeys(PDS_CHECKS)
    if algo == "pd3o":
        orc.pd3o(x0, grad_f, None, Kf, KT, fprox, tau, sigma_, rho, max(PDS_CHECKS), snap=snap)
    else:
        orc.condat_vu(x0, grad_f, None, Kf, KT, fprox, tau, sigma_, rho, max(PDS_CHECKS), snap=snap)
    for k in PDS_CHECKS:
        (x, z), (xr, zr) = got[k], snap[k]
        assert rel_err(x, xr) <= TOL, (k, rel_err(x, xr))
        assert rel_err(z, zr) <= TOL, (k, rel_err(z, zr))
