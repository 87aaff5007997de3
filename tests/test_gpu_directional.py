"""
Jacobian (diff.py:1268-1416), Gaussian-derivative differences (diff_method="gd", diff.py:264-350) in
Gradient / Hessian / Laplacian / Divergence, and DirectionalDerivative / DirectionalGradient /
DirectionalLaplacian / DirectionalHessian (diff.py:1938-2759) on the MI355X: the derivative stacks run on
the HIP stencil / gradient kernels, the directional weighting on pxa_dir_contract.

Checked against the reference's own outputs (tests/golden/directional_*.npz, make_goldens.py
gen_directional) and, at larger seeded sizes, against the oracle restatement (tests/_directional.py),
with the adjoint identity.  Tolerances: <= 1e-5 (fp32) / 1e-12 (fp64) norm-wise relative (the stencils
sum in another association order than NumPy's correlate; the contraction rounds each product, then adds
in the reference's order).
"""
import numpy as np
import pytest

from _directional import case, make_op, oracle_fns
from conftest import golden_names, load_golden, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402

TOL = {np.float32: 1e-5, np.float64: 1e-12}
WIDTH = {np.float32: pxrt.Width.SINGLE, np.float64: pxrt.Width.DOUBLE}


def _run(op, x, adjoint=False):
    out = op.adjoint(to_device(np.ascontiguousarray(x))) if adjoint else op.apply(to_device(np.ascontiguousarray(x)))
    return to_NUMPY(out)


@pytest.mark.parametrize("name", golden_names("directional_"))
def test_directional_golden(name):
    g = load_golden(name)
    kind, kw = case(g)
    dt = g["x"].dtype.type
    with pxrt.Precision(WIDTH[dt]):
        op = make_op(pxo, kind, kw, dt)
        assert tuple(op.shape) == tuple(int(v) for v in g["shape"])
        y, a = _run(op, g["x"]), _run(op, g["z"], adjoint=True)
    assert y.dtype == dt and a.dtype == dt
    assert rel_err(y, g["y"]) <= TOL[dt], (kind, rel_err(y, g["y"]))
    assert rel_err(a, g["adj"]) <= TOL[dt], (kind, rel_err(a, g["adj"]))
    # the step-size input of the PDS solvers: the reference's Lipschitz constant of the same operator
    L_ref = float(g["lipschitz"])
    if np.isinf(L_ref):
        assert np.isinf(op.lipschitz), (kind, op.lipschitz)
    else:
        assert abs(float(op.lipschitz) - L_ref) <= 1e-6 * L_ref, (kind, float(op.lipschitz), L_ref)


BIG = [
    ("jacobian", dict(arg_shape=(96, 130), n_channels=3)),
    ("gradient_gd", dict(arg_shape=(40, 36, 52), sigma=(1.5, 1.0, 2.0))),
    ("hessian_gd", dict(arg_shape=(96, 130), sigma=1.2)),
    ("laplacian_gd", dict(arg_shape=(96, 130), sigma=2.0)),
    ("divergence_gd", dict(arg_shape=(96, 130), sigma=1.0, sampling=0.5)),
    ("dirderiv", dict(arg_shape=(96, 130), order=1, dirs=[(0.3, -1.2)], varying=True)),
    ("dirderiv", dict(arg_shape=(96, 130), order=2, dirs=[(0.3, -1.2), (1.0, 0.5)], varying=True)),
    ("dirgrad", dict(arg_shape=(40, 36, 52), dirs=[(0.1, 2.0, 1.0), (2.0, 1.0, 0.1), (1.0, 1.0, 1.0)], varying=False)),
    ("dirlap", dict(arg_shape=(96, 130), dirs=[(0.3, -1.2), (1.0, 0.5), (0.0, 1.0)], weights=(0.1, 0.7, 2.0),
                    varying=True)),
    ("dirhess", dict(arg_shape=(40, 36, 52), dirs=[(0.1, 2.0, 1.0), (2.0, 1.0, 0.1)], varying=True, sigma=0.9)),
]


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("kind,kw", BIG, ids=[f"{k}{i}" for i, (k, _) in enumerate(BIG)])
def test_directional_vs_oracle_and_adjoint(kind, kw, dt):
    rng = np.random.default_rng(5)
    with pxrt.Precision(WIDTH[dt]):
        op = make_op(pxo, kind, kw, dt)
        x = rng.standard_normal((2, op.dim)).astype(dt)
        z = rng.standard_normal((2, op.codim)).astype(dt)
        y, a = _run(op, x), _run(op, z, adjoint=True)
    ap, ad = oracle_fns(kind, kw, dt)
    assert rel_err(y, ap(x)) <= TOL[dt], (kind, rel_err(y, ap(x)))
    assert rel_err(a, ad(z)) <= TOL[dt], (kind, rel_err(a, ad(z)))
    lhs = np.sum(y.astype(np.float64) * z.astype(np.float64))
    rhs = np.sum(x.astype(np.float64) * a.astype(np.float64))
    assert abs(lhs - rhs) <= 50 * TOL[dt] * max(abs(lhs), 1.0)
