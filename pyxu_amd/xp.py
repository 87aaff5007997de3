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
    "zeros", "ones", "full", "empty", "zeros_like", "empty_like", "asarray", "array", "arange",
    "fabs", "abs", "sign", "fmax", "fmin", "clip", "sqrt", "linalg",
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


# ------------------------------------------------------------------ arithmetic (HIP kernels)
def fabs(x):
    """|x| = x - 2 min(x, 0), from the clip / axpby kernels."""
    return _dev.axpby(1.0, x, -2.0, _neg_part(x))


abs = fabs  # noqa: A001


def _neg_part(x):
    # min(x, 0) = -clip(-x, 0)
    return _dev.axpby(-1.0, _dev.clip(_dev.axpby(-1.0, x), 0.0))


def fmax(x, y):
    if np.isscalar(x) and not np.isscalar(y):
        x, y = y, x
    if np.isscalar(y):
        return _dev.clip(x, float(y))
    raise NotImplementedError("pyxu_amd.xp.fmax: only an array-scalar form has a kernel")


def fmin(x, y):
    if np.isscalar(x) and not np.isscalar(y):
        x, y = y, x
    if np.isscalar(y):  # min(x, c) = -max(-x, -c)
        return _dev.axpby(-1.0, _dev.clip(_dev.axpby(-1.0, x), -float(y)))
    raise NotImplementedError("pyxu_amd.xp.fmin: only an array-scalar form has a kernel")


def clip(x, a_min, a_max=None):
    return _dev.clip(x, float(a_min) if a_min is not None else -np.inf, None if a_max is None else float(a_max))


def sign(x):
    raise NotImplementedError("pyxu_amd.xp.sign: no standalone kernel (L1Norm.prox fuses sign into pxa_prox_l1)")


def sqrt(x, out=None):
    raise NotImplementedError("pyxu_amd.xp.sqrt: no standalone kernel (fused into the L21 kernels)")


# ------------------------------------------------------------------ linalg
def _norm(x, ord=None, axis=None, keepdims=False):
    """numpy.linalg.norm for vectors along the last axis (ord in {None, 1, 2, inf})."""
    if axis not in (None, -1, x.ndim - 1):
        raise NotImplementedError("pyxu_amd.xp.linalg.norm: only axis=-1 (row norms) has a kernel")
    if axis is None and x.ndim != 1:
        x = x.reshape(-1)
    if ord in (None, 2):
        v = _dev.row_reduce(_dev.RED_SUMSQ, x).sqrt_()
    elif ord == 1:
        v = _dev.row_reduce(_dev.RED_ABS, x)
    elif ord in (np.inf, float("inf")):
        v = _dev.row_reduce(_dev.RED_MAXABS, x)
    else:
        raise NotImplementedError(f"pyxu_amd.xp.linalg.norm: ord={ord}")
    v = v.to(x.dtype)
    if keepdims:
        v = v.reshape(*x.shape[:-1], 1)
    elif x.ndim == 1:
        v = v.reshape(())
    return v


linalg = types.SimpleNamespace(norm=_norm)
