"""Element-wise maps used by the stencil filters (mirrors reference operator/map/ufunc.py:660-771):
``sqrt(op)`` and ``square(op)`` as ``_Sqrt * op`` / ``_Square * op`` compositions.  Evaluated by the
HIP unary kernels (pxa_unary: sqrt, x * x)."""
import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["sqrt", "square"]


class _Sqrt(pxa.DiffMap):
    def __init__(self, dim):
        super().__init__(shape=(dim, dim))
        self.lipschitz = np.inf
        self.diff_lipschitz = np.inf

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _dev.unary(_dev.UN_SQRT, arr)

    def jacobian(self, arr):
        from pyxu_amd.operator.linop.base import DiagonalOp

        v = _dev.axpby(2.0, self.apply(arr))
        return DiagonalOp(_dev.unary(_dev.UN_RECIP, v))


class _Square(pxa.DiffMap):
    def __init__(self, dim):
        super().__init__(shape=(dim, dim))
        self.lipschitz = np.inf
        self.diff_lipschitz = 2

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _dev.unary(_dev.UN_SQUARE, arr)  # arr ** 2 == arr * arr exactly

    def jacobian(self, arr):
        from pyxu_amd.operator.linop.base import DiagonalOp

        return DiagonalOp(_dev.axpby(2.0, _dev.require(arr)))


def sqrt(op):
    """Element-wise non-negative square root of op's output (ufunc.py:678-694)."""
    return _Sqrt(op.codim) * op


def square(op):
    """Element-wise square of op's output (ufunc.py:754-770)."""
    return _Square(op.codim) * op
