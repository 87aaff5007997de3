"""
Pad / SubSample / Trim public LinOps (operator/linop/pad.py, select.py) on the MI355X against the
reference's own outputs (tests/golden/padselect_*.npz, make_goldens.py gen_padselect): every pad
mode incl. mixed per-axis modes, and SubSample with steps, negative steps, index lists with repeats
(adjoint keeps numpy's last write), boolean masks and broadcast index pairs.

Pad.apply and every SubSample are pure data movement: bit-exact.  Pad.adjoint folds the borders
back with a few additions per sample whose association may differ from the reference's slice
updates: <= 1e-6 (fp32) / 1e-14 (fp64) norm-wise relative.
"""
import numpy as np
import pytest

from conftest import load_golden, rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402

PADS = {
    "c1": ((7,), 3, "constant"),
    "w2": ((5, 6), ((2, 1), (0, 3)), "wrap"),
    "r2": ((5, 6), (2, 3), "reflect"),
    "s3": ((4, 5, 6), 2, "symmetric"),
    "e2": ((5, 6), ((3, 0), (1, 4)), "edge"),
    "mix": ((5, 6, 4), ((1, 2), (3, 3), (0, 2)), ("edge", "wrap", "reflect")),
}
SELS = {
    "slice": ((10,), (slice(1, None, 3),)),
    "cols": ((3, 40), (slice(None), [1, 3, -1])),
    "mask": ((3, 5, 4), (0, np.r_[True, False, False, True, False])),
    "rep": ((8, 6), ([2, 5, 2, 7],)),
    "pairs": ((6, 7), ([0, 2, 5], [1, 1, 6])),
    "neg": ((9, 8), (slice(None, None, -2), slice(2, 7))),
    "trim": ((9, 8, 5), None),
}


def _sel(sh, idx):
    if idx is None:
        return pxo.Trim(arg_shape=sh, trim_width=((1, 2), (0, 3), (2, 1)))
    return pxo.SubSample(sh, *idx)


def D(a):
    return to_device(np.ascontiguousarray(a))


@pytest.mark.parametrize("w", ["f32", "f64"])
def test_pad_golden(w):
    g = load_golden(f"padselect_{w}")
    with pxrt.Precision(pxrt.Width.SINGLE if w == "f32" else pxrt.Width.DOUBLE):
        for k, (sh, pw, mode) in PADS.items():
            op = pxo.Pad(arg_shape=sh, pad_width=pw, mode=mode)
            assert op.shape == tuple(g[f"pad_{k}_shape"]), k
            assert np.isclose(float(op.lipschitz), float(g[f"pad_{k}_lip"]), rtol=1e-12), k
            assert np.array_equal(to_NUMPY(op.apply(D(g[f"pad_{k}_x"]))), g[f"pad_{k}_y"]), k
            assert np.array_equal(to_NUMPY(op.apply(D(g[f"pad_{k}_x"][0]))), g[f"pad_{k}_y"][0]), k
            a = to_NUMPY(op.adjoint(D(g[f"pad_{k}_z"])))
            assert rel_err(a, g[f"pad_{k}_adj"]) <= (1e-6 if w == "f32" else 1e-14), k


@pytest.mark.parametrize("w", ["f32", "f64"])
def test_subsample_golden(w):
    g = load_golden(f"padselect_{w}")
    with pxrt.Precision(pxrt.Width.SINGLE if w == "f32" else pxrt.Width.DOUBLE):
        for k, (sh, idx) in SELS.items():
            op = _sel(sh, idx)
            assert op.shape == tuple(g[f"sel_{k}_shape"]), k
            assert np.array_equal(to_NUMPY(op.apply(D(g[f"sel_{k}_x"]))), g[f"sel_{k}_y"]), k
            assert np.array_equal(to_NUMPY(op.adjoint(D(g[f"sel_{k}_z"]))), g[f"sel_{k}_adj"]), k
            G = op.gram()  # orthogonal projection: idempotent
            x = D(g[f"sel_{k}_x"])
            assert np.array_equal(to_NUMPY(G.apply(G.apply(x))), to_NUMPY(G.apply(x))), k


def test_pad_constant_gram_is_identity_and_cogram_projects():
    with pxrt.Precision(pxrt.Width.DOUBLE):
        op = pxo.Pad(arg_shape=(5, 6), pad_width=2)
        x = np.random.default_rng(0).standard_normal(op.dim)
        assert np.array_equal(to_NUMPY(op.gram().apply(D(x))), x)
        z = to_NUMPY(op.apply(D(x)))
        assert np.array_equal(to_NUMPY(op.cogram().apply(D(z))), z)
