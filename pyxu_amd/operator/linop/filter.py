"""Stencil-based filters (reference operator/linop/filter.py): Gaussian, MovingAverage."""
import numpy as np

import pyxu_amd.runtime as pxrt
from pyxu_amd.operator.linop.stencil import Stencil

__all__ = ["Gaussian", "MovingAverage", "gaussian_kernel1d"]


def gaussian_kernel1d(sigma: float, order: int, radius: int) -> np.ndarray:
    """Restatement of scipy.ndimage._filters._gaussian_kernel1d (scipy>=1.11,<2; reference call site
    filter.py:305): float64 Gaussian on [-radius, radius], normalised by its sum; derivatives of
    order n via the polynomial recursion of the published algorithm."""
    if order < 0:
        raise ValueError("order must be non-negative")
    exponent_range = np.arange(order + 1)
    sigma2 = sigma * sigma
    x = np.arange(-radius, radius + 1)
    phi_x = np.exp(-0.5 / sigma2 * x**2)
    phi_x = phi_x / phi_x.sum()
    if order == 0:
        return phi_x
    q = np.zeros(order + 1)
    q[0] = 1
    D = np.diag(exponent_range[1:], 1)
    P = np.diag(np.ones(order) / -sigma2, -1)
    Q_deriv = D + P
    for _ in range(order):
        q = Q_deriv.dot(q)
    q = (x[:, None] ** exponent_range).dot(q)
    return q * phi_x


def _canon(v, arg_shape):
    v = np.atleast_1d(v)
    if v.size == 1:
        v = np.repeat(v, len(arg_shape))
    assert v.size == len(arg_shape)
    return v.tolist()


def Gaussian(arg_shape, sigma=1.0, truncate=3.0, order=0, mode="constant", sampling=1, gpu=True, dtype=None):
    """Separable Gaussian filter (filter.py:187-311).  `gpu`/`dtype` kept for signature parity."""
    arg_shape = tuple(arg_shape) if not np.isscalar(arg_shape) else (int(arg_shape),)
    dtype = pxrt.getPrecision().value if dtype is None else dtype
    sigma, truncate, order, sampling = (_canon(v, arg_shape) for v in (sigma, truncate, order, sampling))
    kernel = [np.array([1], dtype=dtype)] * len(arg_shape)
    center = [0] * len(arg_shape)
    for i, (s, t, o, h) in enumerate(zip(sigma, truncate, order, sampling)):
        if s:
            s_pix = s / h
            radius = int(t * float(s_pix) + 0.5)
            k = np.asarray(np.flip(gaussian_kernel1d(s_pix, int(o), radius)), dtype=dtype)
            k /= h**o
            kernel[i] = k
            center[i] = radius
    op = Stencil(arg_shape=arg_shape, kernel=kernel, center=center, mode=mode)
    op._name = "Gaussian"
    return op


def MovingAverage(arg_shape, size, center=None, mode="constant", gpu=True, dtype=None):
    """Uniform (box) filter (filter.py:74-184)."""
    arg_shape = tuple(arg_shape)
    dtype = pxrt.getPrecision().value if dtype is None else dtype
    size = _canon(size, arg_shape)
    center = [s // 2 for s in size] if center is None else list(center)
    kernel = [np.ones(int(s), dtype=dtype) / s for s in size]
    op = Stencil(arg_shape=arg_shape, kernel=kernel, center=center, mode=mode)
    op._name = "MovingAverage"
    return op
