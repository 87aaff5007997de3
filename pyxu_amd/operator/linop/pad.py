"""Pad (reference operator/linop/pad.py:16-416) as a public LinOp on the HIP pad kernels:
apply = pxa_pad (core copy + per-axis border fills, axes last to first), adjoint = pxa_pad_adjoint
(border folds in reverse axis order, then the core)."""
import collections.abc as cabc

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["Pad"]

_MODES = ("constant", "wrap", "reflect", "symmetric", "edge")


def _canonical_widths(width, ndim, what):
    """int | (int, ...) | ((int, int), ...) -> ((lo, hi), ...)   (pad.py:178-188, select.py:234-242)"""
    if not isinstance(width, cabc.Sequence):
        width = ((width, width),) * ndim
    assert len(width) == ndim, f"arg_shape/{what} are length-mismatched."
    if not isinstance(width[0], cabc.Sequence):
        width = tuple((w, w) for w in width)
    return tuple((int(lo), int(hi)) for lo, hi in width)


class Pad(pxa.LinOp):
    """Multi-dimensional padding: (..., prod(arg_shape)) -> (..., prod(arg_shape + lo + hi))."""

    def __init__(self, arg_shape, pad_width, mode="constant"):
        self._arg_shape = tuple(int(n) for n in arg_shape)
        assert all(n > 0 for n in self._arg_shape)
        ndim = len(self._arg_shape)
        self._pad_width = _canonical_widths(pad_width, ndim, "pad_width")
        assert all(0 <= min(lo, hi) for lo, hi in self._pad_width)
        if isinstance(mode, str):
            mode = (mode,) * ndim
        elif isinstance(mode, cabc.Sequence):
            assert len(mode) == ndim, "arg_shape/mode are length-mismatched."
        else:
            raise ValueError(f"Unkwown mode encountered: {mode}.")
        self._mode = tuple(m.strip().lower() for m in mode)
        assert set(self._mode) <= set(_MODES), "Unknown mode(s) encountered."
        self._pad_shape = tuple(n + lo + hi for n, (lo, hi) in zip(self._arg_shape, self._pad_width))
        super().__init__(shape=(int(np.prod(self._pad_shape)), int(np.prod(self._arg_shape))))
        for i, (n, m, (lo, hi)) in enumerate(zip(self._arg_shape, self._mode, self._pad_width)):
            w_max = dict(constant=np.inf, wrap=n, reflect=n - 1, symmetric=n, edge=np.inf)[m]
            assert max(lo, hi) <= w_max, f"pad_width along dim-{i} is limited to {w_max}."
        self.lipschitz = self.estimate_lipschitz(__rule=True)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        sh = x.shape[:-1]
        stack = int(np.prod(sh))
        lo = [w[0] for w in self._pad_width]
        hi = [w[1] for w in self._pad_width]
        y = _dev.pad(x, stack, self._arg_shape, lo, hi, self._mode)
        return y.reshape(*sh, self.codim)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        x = _dev.require(arr)
        sh = x.shape[:-1]
        stack = int(np.prod(sh))
        lo = [w[0] for w in self._pad_width]
        hi = [w[1] for w in self._pad_width]
        y = _dev.pad_adjoint(x, stack, self._arg_shape, lo, hi, self._mode)
        return y.reshape(*sh, self.dim)

    def estimate_lipschitz(self, **kwargs):
        """Product of the per-axis bounds (pad.py:377-394) for the rule; else the generic estimate."""
        if "__rule" in kwargs:
            L = []
            for n, m, (lo, hi) in zip(self._arg_shape, self._mode, self._pad_width):
                if m == "constant":
                    L.append(1)
                elif m in ("wrap", "symmetric"):
                    L.append(np.sqrt(1 + np.ceil((lo + hi) / n)))
                elif m == "reflect":
                    L.append(np.sqrt(1 + np.ceil((lo + hi) / (n - 2))))
                else:
                    L.append(np.sqrt(1 + max(lo, hi)))
            return np.prod(L)
        return super().estimate_lipschitz(**kwargs)

    def gram(self):
        if all(m == "constant" for m in self._mode):
            from pyxu_amd.operator.linop.base import IdentityOp

            return IdentityOp(dim=self.dim)
        return super().gram()

    def cogram(self):
        if all(m == "constant" for m in self._mode):
            from pyxu_amd.operator.linop.select import Trim

            return Trim(arg_shape=self._pad_shape, trim_width=self._pad_width).gram()
        return super().cogram()
