"""pxa_stencil_nd_box: the LDS-tiled N-D stencil kernel (PXA_TUNE_STENCIL_ND 0, default where it applies)
against the generic one-thread-per-output kernel (1) through the public Stencil operator -- same sums in the
same tap order, so the same bits -- for 2-D / 3-D non-separable kernels, off-centre centres, constant mode
(the fused Trim o S o Pad pass) and the other boundary modes (explicit padding, zero_partial), stacks, and
apply / adjoint, fp32 / fp64; plus NumPy (scipy.ndimage.correlate, the reference's own test oracle) at fp32
tolerance."""
import numpy as np
import pytest
import scipy.ndimage as ndi
import torch

import pyxu_amd.operator as pxo
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

pytestmark = pytest.mark.gpu


def run(op, x, adjoint, mode):
    old = _dev.tuning(_dev.TUNE_STENCIL_ND, mode)
    try:
        out = op.adjoint(x) if adjoint else op.apply(x)
        return out.cpu().numpy()
    finally:
        _dev.tuning(_dev.TUNE_STENCIL_ND, old)


CASES = [((96, 130), (5, 7), (2, 3), "constant"), ((64, 64), (15, 15), (7, 7), "constant"),
         ((33, 200), (3, 31), (0, 30), "constant"), ((40, 70), (9, 9), (4, 4), "reflect"),
         ((20, 24, 40), (3, 5, 5), (1, 2, 2), "constant"), ((18, 20, 36), (3, 3, 3), (1, 1, 1), "wrap"),
         ((50, 80), (7, 45), (3, 22), "constant")]


@pytest.mark.parametrize("shape,ksh,center,mode", CASES)
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("stack", [1, 2])
def test_stencil_nd_tile_matches_generic(shape, ksh, center, mode, dt, stack):
    rng = np.random.default_rng(sum(shape) + sum(ksh) + stack)
    kern = rng.standard_normal(ksh)
    x = rng.standard_normal((stack, *shape))
    width = pxrt.Width.SINGLE if dt == np.float32 else pxrt.Width.DOUBLE
    with pxrt.Precision(width):
        op = pxo.Stencil(arg_shape=shape, kernel=kern.astype(dt), center=center, mode=mode)
        op.FFT_MIN_TAPS = 1 << 60  # the direct kernels
        xt = torch.tensor(x.reshape(stack, -1), dtype=torch.float32 if dt == np.float32 else torch.float64,
                          device="cuda")
        for adjoint in (False, True):
            a, b = run(op, xt, adjoint, 0), run(op, xt, adjoint, 1)
            assert np.array_equal(a, b), (adjoint, float(np.max(np.abs(a - b))))
        if mode == "constant" and stack == 1:
            # correlate with the kernel anchored at `center` (stencil.py: y[i] = sum_k kern[k] x[i + k - center])
            origin = [c - (k // 2) for c, k in zip(center, ksh)]
            ref = ndi.correlate(x[0], kern, mode="constant", cval=0.0, origin=origin)
            got = run(op, xt, False, 0).reshape(shape)
            tol = 2e-5 if dt == np.float32 else 1e-12
            assert np.max(np.abs(got - ref)) <= tol * np.max(np.abs(ref)), float(np.max(np.abs(got - ref)))


SEP_CASES = [((96, 130), 2.0, "constant"), ((64, 64), 1.5, "reflect"), ((20, 24, 40), 1.0, "constant"),
             ((18, 20, 36), 1.0, "wrap"), ((33, 37), 2.0, "constant")]


@pytest.mark.parametrize("shape,sigma,mode", SEP_CASES)
@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("stack", [1, 3])
def test_separable_vector_pass_matches_scalar(shape, sigma, mode, dt, stack):
    """separable-axis passes (Gaussian: pxa_stencil_sep in constant mode, pxa_stencil_axis on the padded array
    otherwise): the default (LDS-tiled off-last-axis passes, vector last-axis pass), the vector kernel alone
    (PXA_TUNE_STENCIL_ND bit 2) and the scalar one (bit 1), bit for bit; rows whose length is not a multiple of the vector width take
    the scalar kernel either way"""
    rng = np.random.default_rng(sum(shape) + stack)
    x = rng.standard_normal((stack, int(np.prod(shape))))
    width = pxrt.Width.SINGLE if dt == np.float32 else pxrt.Width.DOUBLE
    with pxrt.Precision(width):
        op = pxo.Gaussian(arg_shape=shape, sigma=sigma, truncate=3.0, mode=mode)
        xt = torch.tensor(x, dtype=torch.float32 if dt == np.float32 else torch.float64, device="cuda")
        for adjoint in (False, True):
            a, b, c = run(op, xt, adjoint, 0), run(op, xt, adjoint, 2), run(op, xt, adjoint, 4)
            assert np.array_equal(a, b), (adjoint, float(np.max(np.abs(a - b))))
            assert np.array_equal(c, b), (adjoint, "vector", float(np.max(np.abs(c - b))))
        if mode == "constant":
            got = run(op, xt, False, 0)
            ref = np.stack([ndi.gaussian_filter(x[s].reshape(shape), sigma, mode="constant", cval=0.0, truncate=3.0)
                            for s in range(stack)]).reshape(stack, -1)
            tol = 1e-5 if dt == np.float32 else 1e-12
            assert np.max(np.abs(got - ref)) <= tol * np.max(np.abs(ref))
