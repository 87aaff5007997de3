"""
NumPy-named array module of the MI355X backend: ``NDArrayInfo.MI355X.module()``.

The reference's hot-path code calls a handful of array-module functions on whatever backend the
input lives on (``xp.fmax``, ``xp.fabs``, ``xp.sign``, ``xp.clip``,
``xp.linalg.norm``, ``xp.zeros`` ...).  This shim gives those names NumPy semantics on torch-ROCm
tensors.  Allocation helpers use torch (memory only); every arithmetic function routes through the
HIP C-ABI (``pyxu_amd._dev``).  Functions without a kernel here raise NotImplementedError rather
than silently computing elsewhere.
"""
import types

import numpy as np

from pyxu_amd import _dev

__all__ = [
    "zeros", "ones", "full", "empty", "zeros_like", "empty_like", "asarray", "array", "arange", "eye",
    "fabs", "abs", "sign", "fmax", "fmin", "maximum", "minimum", "clip", "sqrt", "where", "isnan", "any", "all",
    "concatenate", "stack", "pad", "broadcast_to", "linalg",
]


def _torch():
    import torch

    return torch


def _dt(dtype):
    torch = _torch()
    if dtype is None:
        import pyxu_amd.runtime as pxrt

        dtype = pxrt.getPrecision().value
    return {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}.get(np.dtype(dtype), None) or \
        getattr(torch, np.dtype(dtype).name)


def _dev_index():
    return _torch().device("cuda", _torch().cuda.current_device())


# ------------------------------------------------------------------ allocation (memory only)
def zeros(shape, dtype=None):
    return _torch().zeros(shape, dtype=_dt(dtype), device=_dev_index())


def ones(shape, dtype=None):
    return _torch().ones(shape, dtype=_dt(dtype), device=_dev_index())


def full(shape, fill_value, dtype=None):
    return _torch().full(shape, fill_value, dtype=_dt(dtype), device=_dev_index())


def empty(shape, dtype=None):
    return _torch().empty(shape, dtype=_dt(dtype), device=_dev_index())


def zeros_like(x):
    return _torch().zeros_like(x)


def empty_like(x):
    return _dev.empty_like(x)


def asarray(x, dtype=None):
    from pyxu_amd.util import to_device

    return to_device(x, dtype=None if dtype is None else _dt(dtype))


array = asarray


def arange(*args, dtype=None):
    return asarray(np.arange(*args, dtype=dtype))


def eye(N, M=None, k=0, dtype=None):
    M = N if M is None else M
    out = zeros((N, M), dtype=dtype)
    rows = min(N, M - k) if k >= 0 else min(N + k, M)
    if rows > 0:
        _dev.set_diag(out, rows, M + 0, k if k >= 0 else -k * M, 1.0)
    return out


# ------------------------------------------------------------------ arithmetic (HIP kernels)
def fabs(x):
    return _dev.unary(_dev.UN_ABS, x)


abs = fabs  # noqa: A001


def sign(x):
    """numpy.sign: -1 / 0 / +1 (NaN stays NaN)."""
    return _dev.unary(_dev.UN_SIGN, x)


def sqrt(x, out=None):
    return _dev.unary(_dev.UN_SQRT, x, out=out)


def _bin(op, x, y, out=None):
    if np.isscalar(x) and np.isscalar(y):
        raise TypeError("pyxu_amd.xp: at least one operand must be a device array")
    return _dev.binary(op, x, y, out=out)


def fmax(x, y, out=None):
    """numpy.fmax (NaN-ignoring), array-array or array-scalar."""
    return _bin(_dev.BIN_FMAX, x, y, out)


def fmin(x, y, out=None):
    return _bin(_dev.BIN_FMIN, x, y, out)


def maximum(x, y, out=None):
    """numpy.maximum (NaN-propagating)."""
    return _bin(_dev.BIN_MAXIMUM, x, y, out)


def minimum(x, y, out=None):
    return _bin(_dev.BIN_MINIMUM, x, y, out)


def clip(x, a_min, a_max=None):
    return _dev.clip(x, float(a_min) if a_min is not None else -np.inf, None if a_max is None else float(a_max))


def where(cond, x, y):
    """numpy.where(cond, x, y) with x / y device arrays of cond's shape or scalars."""
    like = x if not np.isscalar(x) else (y if not np.isscalar(y) else None)
    if like is None:
        raise TypeError("pyxu_amd.xp.where: at least one of x, y must be a device array")
    return _dev.where(cond, x, y, like=like)


def isnan(x):
    return _dev.isnan(x)


def any(x, axis=None):  # noqa: A001
    if axis is not None:
        raise NotImplementedError("pyxu_amd.xp.any: axis=None only")
    return _dev.bool_reduce(x, 0)


def all(x, axis=None):  # noqa: A001
    if axis is not None:
        raise NotImplementedError("pyxu_amd.xp.all: axis=None only")
    return _dev.bool_reduce(x, 1)


# ------------------------------------------------------------------ joins / shape (HIP copies)
def concatenate(arrays, axis=0):
    """numpy.concatenate for device arrays: each part is viewed as (outer, k_i * inner) around `axis`
    and copied into its column band of the (outer, sum k_i * inner) result (pxa_copy2d)."""
    arrays = [_dev.require(a) for a in arrays]
    nd = arrays[0].ndim
    ax = axis % nd
    shp = list(arrays[0].shape)
    outer = int(np.prod(shp[:ax])) if ax > 0 else 1
    inner = int(np.prod(shp[ax + 1:])) if ax + 1 < nd else 1
    total = sum(a.shape[ax] for a in arrays)
    shp[ax] = total
    out = _dev.empty(tuple(shp), arrays[0])
    off = 0
    for a in arrays:
        assert a.ndim == nd and a.dtype == arrays[0].dtype
        w = a.shape[ax] * inner
        _dev.copy2d(a, out, outer, w, w, total * inner, dst_off=off)
        off += w
    return out


def stack(arrays, axis=0):
    arrays = [_dev.require(a) for a in arrays]
    nd = arrays[0].ndim + 1
    ax = axis % nd
    return concatenate([a.reshape(*a.shape[:ax], 1, *a.shape[ax:]) for a in arrays], axis=ax)


def pad(x, pad_width, mode="constant"):
    """numpy.pad over every axis of x (modes of operator/linop/pad.py: constant (0), wrap, reflect,
    symmetric, edge) through pxa_pad."""
    x = _dev.require(x)
    # numpy's pad_width forms: int, (n,), (before, after) for every axis, or ((before, after), ...) per axis
    pw = np.broadcast_to(np.asarray(pad_width, dtype=np.int64), (x.ndim, 2))
    pad_width = [(int(a), int(b)) for a, b in pw]
    lo = [p[0] for p in pad_width]
    hi = [p[1] for p in pad_width]
    y = _dev.pad(x, 1, tuple(x.shape), lo, hi, [mode] * x.ndim)
    return y.reshape(*[n + l + h for n, l, h in zip(x.shape, lo, hi)])


def broadcast_to(x, shape):
    """Read-only broadcast VIEW (numpy.broadcast_to semantics: no data is written)."""
    return x.expand(*shape)


# ------------------------------------------------------------------ linalg
def _norm(x, ord=None, axis=None, keepdims=False):
    """numpy.linalg.norm for vectors along the last axis (any ord >= 0 and inf)."""
    if axis not in (None, -1, x.ndim - 1):
        raise NotImplementedError("pyxu_amd.xp.linalg.norm: only axis=-1 (row norms) has a kernel")
    if axis is None and x.ndim != 1:
        x = x.reshape(-1)
    if ord in (None, 2):
        v = _dev.unary(_dev.UN_SQRT, _dev.row_reduce(_dev.RED_SUMSQ, x))
    elif ord == 1:
        v = _dev.row_reduce(_dev.RED_ABS, x)
    elif ord in (np.inf, float("inf")):
        v = _dev.row_reduce(_dev.RED_MAXABS, x)
    elif ord == 0:
        v = _dev.row_reduce_pow(0.0, x)
    else:  # any other p > 0: (sum |x|^p)^(1/p)
        v = _dev.binary(_dev.BIN_POW, _dev.row_reduce_pow(float(ord), x), 1.0 / float(ord))
    v = _dev.cast(v, x)
    if keepdims:
        v = v.reshape(*x.shape[:-1], 1)
    elif x.ndim == 1:
        v = v.reshape(())
    return v


linalg = types.SimpleNamespace(norm=_norm)
