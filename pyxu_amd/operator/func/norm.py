"""Norm functionals (mirrors reference operator/func/norm.py): L1, L2, SquaredL2, L21, LInfinity."""
import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["L1Norm", "L2Norm", "SquaredL2Norm", "L21Norm", "LInfinityNorm", "PositiveL1Norm"]


def _row(arr, op, y=None):
    """(..., N) -> (..., 1) in arr.dtype: device row reduction (double accumulation)."""
    x2 = arr.reshape(-1, arr.shape[-1])
    r = _dev.row_reduce(op, x2, None if y is None else y.reshape(x2.shape))
    return _dev.cast(r, arr).reshape(*arr.shape[:-1], 1)


class _ShiftLossMixin:
    def asloss(self, data=None):
        from pyxu_amd.operator.func.loss import shift_loss

        return shift_loss(op=self, data=data)


class L1Norm(_ShiftLossMixin, pxa.ProxFunc):
    """||x||_1 (norm.py:33-52)."""

    def __init__(self, dim):
        super().__init__(shape=(1, dim))
        self.lipschitz = np.sqrt(dim)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _row(arr, _dev.RED_ABS)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        return _dev.prox_l1(arr, tau)

    @pxrt.enforce_precision(i=("arr", "sigma"))
    def fenchel_prox(self, arr, sigma):
        return _dev.fenchel_prox_l1(arr, sigma, 1.0)


class L2Norm(_ShiftLossMixin, pxa.ProxFunc):
    """||x||_2 (norm.py:55-77)."""

    def __init__(self, dim):
        super().__init__(shape=(1, dim))
        self.lipschitz = 1
        self.diff_lipschitz = np.inf if False else np.inf

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        r = _dev.unary(_dev.UN_SQRT, _dev.row_reduce(_dev.RED_SUMSQ, arr.reshape(-1, arr.shape[-1])))
        return _dev.cast(r, arr).reshape(*arr.shape[:-1], 1)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        # x * (1 - tau / fmax(||x||, tau)): the L21 kernel with a single group spanning the row
        S = int(np.prod(arr.shape[:-1])) if arr.ndim > 1 else 1
        return _dev.prox_l21(arr, tau, S, arr.shape[-1], 1).reshape(arr.shape)


class SquaredL2Norm(pxa.QuadraticFunc):
    """||x||_2^2 (norm.py:80-112)."""

    def __init__(self, dim):
        super().__init__(shape=(1, dim))
        self.lipschitz = np.inf
        self.diff_lipschitz = 2

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _row(arr, _dev.RED_SUMSQ)

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        return _dev.axpby(2.0, arr)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        return _dev.div(arr, 2 * tau + 1)

    def _quad_spec(self):
        from pyxu_amd.operator.linop import HomothetyOp, NullFunc

        return (HomothetyOp(dim=self.dim, cst=2), NullFunc(dim=self.dim), 0)


class LInfinityNorm(_ShiftLossMixin, pxa.ProxFunc):
    """||x||_inf (norm.py:241-293); prox is outside the hot path."""

    def __init__(self, dim):
        super().__init__(shape=(1, dim))
        self.lipschitz = 1

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _row(arr, _dev.RED_MAXABS)

    def prox(self, arr, tau):
        raise NotImplementedError("pyxu_amd: LInfinityNorm.prox (root finding) is outside the hot-path scope.")


class L21Norm(_ShiftLossMixin, pxa.ProxFunc):
    """Mixed l2-l1 norm (norm.py:296-364): l2 over `l2_axis`, l1 over the rest."""

    def __init__(self, arg_shape, l2_axis=(0,)):
        arg_shape = (int(arg_shape),) if np.isscalar(arg_shape) else tuple(int(a) for a in arg_shape)
        assert all(a > 0 for a in arg_shape)
        N = len(arg_shape)
        assert N >= 2
        l2_axis = np.unique(np.atleast_1d(l2_axis))
        assert np.all((-N <= l2_axis) & (l2_axis < N))
        l2_axis = (l2_axis + N) % N
        super().__init__(shape=(1, int(np.prod(arg_shape))))
        self.lipschitz = np.inf
        self._arg_shape = arg_shape
        self._l2_axis = l2_axis
        self._l1_axis = np.setdiff1d(np.arange(N), l2_axis)
        a0, a1 = int(l2_axis.min()), int(l2_axis.max())
        self._contig = (a1 - a0 + 1) == len(l2_axis)
        if self._contig:
            self._outer = int(np.prod(arg_shape[:a0]))
            self._group = int(np.prod(arg_shape[a0:a1 + 1]))
            self._inner = int(np.prod(arg_shape[a1 + 1:]))
        self._perm = tuple(self._l1_axis.tolist()) + tuple(l2_axis.tolist())

    def _grouped(self, arr, fn):
        """Apply a (outer, group, inner) kernel on arr (..., N); permutes if l2 axes are not contiguous."""
        sh = arr.shape[:-1]
        S = int(np.prod(sh)) if len(sh) else 1
        x = _dev.require(arr)
        if self._contig:
            return fn(x, S * self._outer, self._group, self._inner).reshape(arr.shape)
        # bring the l2 axes last (layout plumbing), run grouped kernel, restore
        nd = len(self._arg_shape)
        xt = x.reshape(S, *self._arg_shape).permute(0, *[p + 1 for p in self._perm]).contiguous()
        g = int(np.prod([self._arg_shape[a] for a in self._l2_axis]))
        y = fn(xt, xt.numel() // g, g, 1).reshape(xt.shape)
        inv = np.argsort((0,) + tuple(p + 1 for p in self._perm))
        return y.permute(*inv.tolist()).contiguous().reshape(arr.shape)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        sh = arr.shape[:-1]
        S = int(np.prod(sh)) if len(sh) else 1
        if self._contig:
            n = _dev.group_norm(_dev.require(arr), S * self._outer, self._group, self._inner)
        else:
            x = _dev.require(arr).reshape(S, *self._arg_shape).permute(0, *[p + 1 for p in self._perm]).contiguous()
            g = int(np.prod([self._arg_shape[a] for a in self._l2_axis]))
            n = _dev.group_norm(x, x.numel() // g, g, 1)
        r = _dev.row_reduce(_dev.RED_SUM, n.reshape(S, -1))
        return _dev.cast(r, arr).reshape(*sh, 1)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        return self._grouped(arr, lambda x, o, g, i: _dev.prox_l21(x, tau, o, g, i))

    @pxrt.enforce_precision(i=("arr", "sigma"))
    def fenchel_prox(self, arr, sigma):
        return self._grouped(arr, lambda x, o, g, i: _dev.fenchel_prox_l21(x, sigma, 1.0, o, g, i))


class PositiveL1Norm(_ShiftLossMixin, pxa.ProxFunc):
    """||x||_1 + indicator(x >= 0) (norm.py:367-403)."""

    def __init__(self, dim):
        super().__init__(shape=(1, dim))
        from pyxu_amd.operator.func.indicator import PositiveOrthant

        self._indicator = PositiveOrthant(dim=dim)
        self._l1norm = L1Norm(dim=dim)
        self.lipschitz = np.inf

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _dev.axpby(1.0, self._indicator(arr), 1.0, self._l1norm(arr))

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        # fmax(0, arr - tau)
        return _dev.clip(_dev.add_scalar(arr, -tau), 0.0)
