"""Stencil-based filters (reference operator/linop/filter.py): MovingAverage, Gaussian,
DifferenceOfGaussians, Laplace, Sobel / Prewitt / Scharr and StructureTensor, all on the HIP stencil
kernels (separable passes or the N-D kernel)."""
import functools
import itertools

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.operator.linop.stencil import Stencil

__all__ = ["Gaussian", "MovingAverage", "DifferenceOfGaussians", "DoG", "Laplace", "Sobel", "Prewitt", "Scharr",
           "StructureTensor", "gaussian_kernel1d"]


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
    if center is None:
        assert all(s % 2 == 1 for s in size), \
            "Can only infer center for odd `size`s. For even `size`s, please provide the desired `center`s."
        center = [s // 2 for s in size]
    kernel = [np.ones(int(s), dtype=dtype) for s in size]  # separable box, scaled once as the reference
    op = (1 / np.prod(size)) * Stencil(arg_shape=arg_shape, kernel=kernel, center=list(center), mode=mode)
    op._name = "MovingAverage"
    return op


def _to_canonical_form(v, arg_shape):
    """filter.py:42-47: a scalar is repeated per axis; a sequence must give one value per axis."""
    if np.isscalar(v) or not hasattr(v, "__len__"):
        return (v,) * len(arg_shape)
    assert len(v) == len(arg_shape)
    return tuple(v)


def DifferenceOfGaussians(arg_shape, low_sigma=1.0, high_sigma=None, low_truncate=3.0, high_truncate=3.0,
                          mode="constant", sampling=1, gpu=True, dtype=None):
    """Gaussian(low_sigma) - Gaussian(high_sigma), high_sigma = 1.6 low_sigma by default (filter.py:314-440)."""
    arg_shape = tuple(arg_shape)
    low_sigma = _to_canonical_form(low_sigma, arg_shape)
    if high_sigma is None:
        high_sigma = tuple(s * 1.6 for s in low_sigma)
    high_sigma = _to_canonical_form(high_sigma, arg_shape)
    low_truncate = _to_canonical_form(low_truncate, arg_shape)
    high_truncate = _to_canonical_form(high_truncate, arg_shape)
    kw = dict(arg_shape=arg_shape, order=0, mode=mode, gpu=gpu, dtype=dtype, sampling=sampling)
    op = Gaussian(sigma=low_sigma, truncate=low_truncate, **kw) - Gaussian(sigma=high_sigma, truncate=high_truncate, **kw)
    op._name = "DifferenceOfGaussians"
    return op


DoG = DifferenceOfGaussians


def Laplace(arg_shape, mode="constant", sampling=1, gpu=True, dtype=None):
    """Sum over axes of the [1, -2, 1] / h_d second difference (filter.py:443-533): one N-D stencil per
    axis, summed by the operator algebra in axis order."""
    arg_shape = tuple(arg_shape)
    ndim = len(arg_shape)
    dtype = pxrt.getPrecision().value if dtype is None else dtype
    sampling = _to_canonical_form(sampling, arg_shape)
    ops = []
    for dim in range(ndim):
        k = (np.array([1.0, -2.0, 1.0]).reshape([-1 if i == dim else 1 for i in range(ndim)]) / sampling[dim])
        c = [1 if i == dim else 0 for i in range(ndim)]
        ops.append(Stencil(arg_shape=arg_shape, kernel=k.astype(dtype), center=c, mode=mode))
    op = functools.reduce(lambda x, y: x + y, ops)
    op._name = "Laplace"
    return op


def _get_axes(axis, ndim):
    if axis is None:
        return list(range(ndim))
    if np.isscalar(axis):
        return [axis]
    return list(axis)


def _EdgeFilter(arg_shape, smooth_kernel, filter_name, axis=None, mode="constant", sampling=1, gpu=True, dtype=None):
    """filter.py:791-828: [-1, 0, 1] / h along each edge axis, the smoothing kernel / h along the others;
    several axes give the magnitude sqrt(sum_d (S_d x)^2) / sqrt(ndim)."""
    from pyxu_amd.operator.map import sqrt, square

    arg_shape = tuple(arg_shape)
    ndim = len(arg_shape)
    dtype = pxrt.getPrecision().value if dtype is None else dtype
    sampling = _to_canonical_form(sampling, arg_shape)
    axes = _get_axes(axis, ndim)
    magnitude = len(axes) > 1
    ops = []
    for edge_dim in axes:
        kernel = [np.array(1.0, dtype=dtype)] * ndim
        center = np.ones(ndim, dtype=int)
        kernel[edge_dim] = np.array([-1, 0, 1], dtype=dtype) / sampling[edge_dim]
        for smooth_dim in set(range(ndim)) - {edge_dim}:
            kernel[smooth_dim] = np.asarray(smooth_kernel, dtype=dtype) / sampling[smooth_dim]
        st = Stencil(arg_shape=arg_shape, kernel=kernel, center=center, mode=mode)
        ops.append(square(st) if magnitude else st)
    op = functools.reduce(lambda x, y: x + y, ops)
    if magnitude:
        op = (1 / np.sqrt(ndim)) * sqrt(op)
    op._name = filter_name
    return op


def Sobel(arg_shape, axis=None, mode="constant", sampling=1, gpu=True, dtype=None):
    """Sobel edge filter: smoothing [1, 2, 1] / 4 (filter.py:536-632)."""
    return _EdgeFilter(arg_shape, np.array([1, 2, 1]) / 4, "SobelFilter", axis, mode, sampling, gpu, dtype)


def Prewitt(arg_shape, axis=None, mode="constant", sampling=1, gpu=True, dtype=None):
    """Prewitt edge filter: smoothing [1, 1, 1] / 3 (filter.py:636-732)."""
    return _EdgeFilter(arg_shape, np.full((3,), 1 / 3), "Prewitt", axis, mode, sampling, gpu, dtype)


def Scharr(arg_shape, axis=None, mode="constant", sampling=1, gpu=True, dtype=None):
    """Scharr edge filter: smoothing [3, 10, 3] / 16 (filter.py:735-788)."""
    return _EdgeFilter(arg_shape, np.array([3, 10, 3]) / 16, "Scharr", axis, mode, sampling, gpu, dtype)


class StructureTensor(pxa.DiffMap):
    """Gaussian-smoothed outer products of the (central-difference) gradient, upper triangle in
    combinations_with_replacement order (filter.py:875-1042): (..., N) -> (..., D(D+1)/2 * N)."""

    def __init__(self, arg_shape, diff_method="fd", smooth_sigma=1.0, smooth_truncate=3.0, mode="constant", sampling=1,
                 gpu=True, dtype=None, parallel=False, **diff_kwargs):
        from pyxu_amd.operator.linop.base import IdentityOp
        from pyxu_amd.operator.linop.diff import Gradient

        self.arg_shape = tuple(arg_shape)
        size = int(np.prod(arg_shape))
        ndim = len(arg_shape)
        ntriu = (ndim * (ndim + 1)) // 2
        super().__init__(shape=(ntriu * size, size))
        self.directions = tuple(list(d) for d in itertools.combinations_with_replacement(range(ndim), 2))
        if diff_method == "fd":
            diff_kwargs.update({"scheme": diff_kwargs.pop("scheme", "central")})
        self.grad = Gradient(arg_shape=arg_shape, directions=None, mode=mode, gpu=gpu, dtype=dtype, sampling=sampling,
                             parallel=parallel, **diff_kwargs)
        if smooth_sigma:
            self.smooth = Gaussian(arg_shape=arg_shape, sigma=smooth_sigma, truncate=smooth_truncate, order=0, mode=mode,
                                   sampling=sampling, gpu=gpu, dtype=dtype)
        else:
            self.smooth = IdentityOp(dim=size)

    def unravel(self, arr):
        return arr.reshape(*arr.shape[:-1], -1, *self.arg_shape)

    def ravel(self, arr):
        return arr.reshape(*arr.shape[: -1 - len(self.arg_shape)], -1)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        sh = x.shape[:-1]
        S = int(np.prod(sh)) if len(sh) else 1
        N = int(np.prod(self.arg_shape))
        D = len(self.arg_shape)
        g = _dev.require(self.grad(x)).reshape(S, D, N)
        out = _dev.empty((S, len(self.directions) * N), x)
        for k, (i, j) in enumerate(self.directions):
            gi = _dev.take_cols(g.reshape(S, D * N), i * N, N)
            gj = _dev.take_cols(g.reshape(S, D * N), j * N, N)
            p = _dev.require(self.smooth(_dev.mul(gi, gj)))  # smooth(grad_i * grad_j)
            _dev.copy2d(p, out, S, N, N, len(self.directions) * N, dst_off=k * N)
        return out.reshape(*sh, -1)
