"""
GPU parity of the FFT path of Stencil / Convolve (large non-separable zero-boundary kernels: zero-pad to
a smooth length >= n + K - 1, Stockham FFT, spectrum product, inverse FFT, crop) against the CPU
restatement of the reference's direct correlation (stencil.py:441-461 -> oracle.stencil_apply /
stencil_adjoint) and against this package's own direct-stencil kernel (same operator with the FFT
path switched off).  The adjoint uses the conjugate spectrum; <Ax, y> = <x, A*y> is checked too.
Tolerance: norm-wise relative 1e-5 (fp32) / 1e-12 (fp64).
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

import oracle.pyxu_np as ora  # noqa: E402
import pyxu_amd.operator as pxo  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd.util import to_device, to_NUMPY  # noqa: E402

TOL = {np.float32: 1e-5, np.float64: 1e-12}
WIDTH = {np.float32: pxrt.Width.SINGLE, np.float64: pxrt.Width.DOUBLE}

CASES = [  # (arg_shape, kernel shape, center)
    ((64, 80), (17, 17), (8, 8)),
    ((96, 70), (21, 15), (0, 14)),
    ((33, 40, 28), (7, 7, 7), (3, 2, 6)),
    ((300, 257), (31, 31), (15, 15)),
]


def _stencil(arg_shape, K, center, fft, seed=0):
    rng = np.random.default_rng(seed)
    k = rng.standard_normal(K)
    op = pxo.Stencil(arg_shape=arg_shape, kernel=k, center=center, mode="constant")
    op.FFT_MIN_TAPS = 1 if fft else 1 << 60  # force either path (the default threshold depends on ndim)
    return op, k


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("arg_shape,K,center", CASES)
def test_fft_stencil_matches_oracle(arg_shape, K, center, dtype):
    rng = np.random.default_rng(1)
    N = int(np.prod(arg_shape))
    x = rng.standard_normal((2, N))
    y = rng.standard_normal((2, N))
    with pxrt.Precision(WIDTH[dtype]):
        op, k = _stencil(arg_shape, K, center, fft=True)
        got = to_NUMPY(op.apply(to_device(x.astype(dtype))))
        gadj = to_NUMPY(op.adjoint(to_device(y.astype(dtype))))
        assert op._fft_plan(to_device(x.astype(dtype))) is not None, "FFT path not taken"
    for s in range(2):
        ref = ora.stencil_apply(x[s], arg_shape, k, center, mode="constant")
        assert rel_err(got[s], ref) < TOL[dtype]
        ref = ora.stencil_adjoint(y[s], arg_shape, k, center, mode="constant")
        assert rel_err(gadj[s], ref) < TOL[dtype]
    lhs = np.sum(got.astype(np.float64) * y)
    rhs = np.sum(x * gadj.astype(np.float64))
    assert abs(lhs - rhs) <= 10 * TOL[dtype] * np.linalg.norm(got) * np.linalg.norm(y)


@pytest.mark.parametrize("arg_shape,K,center", CASES)
def test_fft_stencil_matches_direct_kernel(arg_shape, K, center):
    rng = np.random.default_rng(2)
    N = int(np.prod(arg_shape))
    x = to_device(rng.standard_normal(N).astype(np.float32))
    with pxrt.Precision(pxrt.Width.SINGLE):
        a, _ = _stencil(arg_shape, K, center, fft=True)
        b, _ = _stencil(arg_shape, K, center, fft=False)
        assert rel_err(to_NUMPY(a.apply(x)), to_NUMPY(b.apply(x))) < 1e-5
        assert rel_err(to_NUMPY(a.adjoint(x)), to_NUMPY(b.adjoint(x))) < 1e-5


def test_fft_path_not_taken_for_small_or_separable_or_nonzero_boundary():
    x = to_device(np.zeros(64 * 64, dtype=np.float32))
    with pxrt.Precision(pxrt.Width.SINGLE):
        small = pxo.Stencil(arg_shape=(64, 64), kernel=np.ones((5, 5)), center=(2, 2))
        sep = pxo.Stencil(arg_shape=(64, 64), kernel=[np.ones(31), np.ones(31)], center=(15, 15))
        refl = pxo.Stencil(arg_shape=(64, 64), kernel=np.ones((31, 31)), center=(15, 15), mode="reflect")
        for op in (small, sep, refl):
            assert op._fft_plan(x) is None
