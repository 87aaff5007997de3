"""
Stencil filters (operator/linop/filter.py: DifferenceOfGaussians / DoG, Laplace, Sobel, Prewitt,
Scharr, StructureTensor, MovingAverage) and the proximal-splitting aliases (opt/solver/pds.py:
ChambollePock, LorisVerhoeven, DavisYin, DouglasRachford, ForwardBackward, ProximalPoint) on the
MI355X, against the reference's own outputs (tests/golden/filters_*.npz, aliases_*.npz, generated
by tests/golden/make_goldens.py gen_filters / gen_aliases).

Tolerances: the filters are sums of stencil passes evaluated in a different association order than
the reference's NumPy correlate: <= 1e-5 (fp32) / 1e-12 (fp64) norm-wise relative; alias-solver
trajectories after 1 / 10 / 50 iterations: <= 1e-5 (fp32) / 1e-10 (fp64).
"""
import numpy as np
import pytest

from conftest import load_golden, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402

OP_TOL = {"f32": 1e-5, "f64": 1e-12}
TRAJ_TOL = {"f32": 1e-5, "f64": 1e-10}
WIDTH = {"f32": pxrt.Width.SINGLE, "f64": pxrt.Width.DOUBLE}


def D(a):
    return to_device(np.ascontiguousarray(a))


def _filters(sh):
    return {
        "dog": pxo.DifferenceOfGaussians(arg_shape=sh, low_sigma=1.0),
        "dog_s": pxo.DoG(arg_shape=sh, low_sigma=0.7, high_sigma=1.3, mode="reflect", sampling=2.0),
        "laplace": pxo.Laplace(arg_shape=sh),
        "laplace_w": pxo.Laplace(arg_shape=sh, mode="wrap", sampling=2.0),
        "sobel0": pxo.Sobel(arg_shape=sh, axis=0),
        "sobel": pxo.Sobel(arg_shape=sh),
        "prewitt1": pxo.Prewitt(arg_shape=sh, axis=1, mode="edge"),
        "prewitt": pxo.Prewitt(arg_shape=sh, mode="symmetric"),
        "scharr": pxo.Scharr(arg_shape=sh, sampling=0.5),
        "scharr01": pxo.Scharr(arg_shape=sh, axis=(0, 1)),
        "st": pxo.StructureTensor(arg_shape=sh),
        "st_nos": pxo.StructureTensor(arg_shape=sh, smooth_sigma=0, mode="reflect"),
        "mavg": pxo.MovingAverage(arg_shape=sh, size=3, center=None, mode="constant"),
    }


@pytest.mark.parametrize("w", ["f32", "f64"])
@pytest.mark.parametrize("tag", ["2d", "3d"])
def test_filters_golden(w, tag):
    g = load_golden(f"filters_{w}")
    sh = tuple(int(v) for v in g[f"shape_{tag}"])
    with pxrt.Precision(WIDTH[w]):
        for k, op in _filters(sh).items():
            key = f"{tag}_{k}"
            assert type(op).__name__ == str(g[f"{key}_cls"]), key
            assert op.shape == tuple(g[f"{key}_shape"]), key
            y = to_NUMPY(op.apply(D(g[f"{key}_x"])))
            assert y.dtype == g[f"{key}_y"].dtype, key
            assert rel_err(y, g[f"{key}_y"]) <= OP_TOL[w], (key, rel_err(y, g[f"{key}_y"]))
            if f"{key}_adj" in g:
                a = to_NUMPY(op.adjoint(D(g[f"{key}_z"])))
                assert rel_err(a, g[f"{key}_adj"]) <= OP_TOL[w], (key, rel_err(a, g[f"{key}_adj"]))


def test_edge_magnitude_jacobian_matches_finite_differences():
    """Sobel magnitude = sqrt(sum_d (S_d x)^2) / sqrt(D): its Jacobian (chain rule through the sqrt /
    square maps, operator/map.py) against central differences."""
    rng = np.random.default_rng(3)
    sh = (8, 9)
    with pxrt.Precision(pxrt.Width.DOUBLE):
        op = pxo.Sobel(arg_shape=sh)
        x = rng.uniform(1, 2, int(np.prod(sh)))
        v = rng.standard_normal(x.size)
        J = op.jacobian(D(x))
        jv = to_NUMPY(J.apply(D(v)))
        eps = 1e-6
        fd = (to_NUMPY(op.apply(D(x + eps * v))) - to_NUMPY(op.apply(D(x - eps * v)))) / (2 * eps)
        assert rel_err(jv, fd) <= 1e-6


def _alias_cases(g, sh):
    N = int(np.prod(sh))
    H = pxo.Gaussian(arg_shape=sh, sigma=float(g["sigma"]), truncate=3.0)
    f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(D(g["y"])) * H
    f.diff_lipschitz = 1.0
    lam = float(g["lam"])
    K = pxo.Gradient(arg_shape=sh)
    h = lam * pxo.L21Norm(arg_shape=(2, *sh))
    gp = pxo.PositiveOrthant(dim=N)
    l1 = lam * pxo.L1Norm(dim=N)
    return {
        "cp": lambda: pxs.CP(g=gp, h=h, K=K, show_progress=False),
        "cp_pd3o": lambda: pxs.CP(g=gp, h=h, K=K, base=pxs.PD3O, show_progress=False),
        "lv": lambda: pxs.LV(f=f, h=h, K=K, show_progress=False),
        "dy": lambda: pxs.DY(f=f, g=gp, h=l1, show_progress=False),
        "dr": lambda: pxs.DR(g=gp, h=l1, show_progress=False),
        "fb": lambda: pxs.FB(f=f, g=l1, show_progress=False),
        "pp": lambda: pxs.PP(g=l1, show_progress=False),
    }


@pytest.mark.parametrize("w", ["f32", "f64"])
def test_alias_solvers_trajectory_golden(w):
    g = load_golden(f"aliases_{w}")
    sh = tuple(int(v) for v in g["arg_shape"])
    with pxrt.Precision(WIDTH[w]):
        for name, mk in _alias_cases(g, sh).items():
            for n in (1, 10, 50):
                s = mk()
                assert type(s).__name__ == str(g[f"{name}_cls"]), name
                s.fit(x0=D(g["x0"]), stop_crit=pxst.MaxIter(n))
                data, _ = s.stats()
                err = rel_err(to_NUMPY(data["x"]), g[f"{name}_x_{n}"])
                assert err <= TRAJ_TOL[w], (name, n, err)
            for k in ("tau", "sigma", "rho"):
                assert np.isclose(float(s._mstate[k]), float(g[f"{name}_{k}"]), rtol=1e-12), (name, k)


def test_filters_are_linops_where_the_reference_says_so():
    with pxrt.Precision(pxrt.Width.SINGLE):
        ops = _filters((9, 11))
    for k in ("dog", "laplace", "sobel0", "prewitt1", "mavg"):
        assert isinstance(ops[k], pxa.LinOp), k
    for k in ("sobel", "scharr", "st"):
        assert not isinstance(ops[k], pxa.LinOp), k
