"""Linear-algebra helpers (reference pyxu.math.linalg.norm :14-22) on device tensors."""
import numpy as np

from pyxu_amd import _dev

__all__ = ["norm"]


def norm(x, ord=None, axis=None, keepdims=False):
    """Vector norm over the last axis (the only form the hot path uses)."""
    if axis not in (None, -1, x.ndim - 1):
        raise NotImplementedError("pyxu_amd.math.norm: last-axis norms only.")
    x2 = x.reshape(-1, x.shape[-1]) if axis is not None else x.reshape(1, -1)
    if ord in (None, 2):
        r = _dev.unary(_dev.UN_SQRT, _dev.row_reduce(_dev.RED_SUMSQ, x2))
    elif ord == 1:
        r = _dev.row_reduce(_dev.RED_ABS, x2)
    elif ord == np.inf:
        r = _dev.row_reduce(_dev.RED_MAXABS, x2)
    else:
        raise NotImplementedError(f"ord={ord}")
    r = _dev.cast(r, x)
    if axis is None:
        return r.reshape(()) if not keepdims else r.reshape((1,) * x.ndim)
    return r.reshape(*x.shape[:-1], 1) if keepdims else r.reshape(x.shape[:-1])
