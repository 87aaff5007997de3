"""Elementary LinOps and the dense explicit LinOp (reference operator/linop/base.py)."""
import warnings

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.operator.interop import from_source
from pyxu_amd.util import is_device_array, to_device

__all__ = ["IdentityOp", "NullOp", "NullFunc", "HomothetyOp", "DiagonalOp", "Sum", "_ExplicitLinOp"]


def _view(arr):
    # a view signals "do not modify in place" to copy_if_unsafe (reference returns read-only views)
    return arr.view(arr.shape)


class IdentityOp(pxa.OrthProjOp):
    """Identity (base.py:24-59)."""

    def __init__(self, dim):
        super().__init__(shape=(dim, dim))

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _view(arr)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        return _view(arr)

    def svdvals(self, **kwargs):
        return np.ones(kwargs.get("k", 1), dtype=pxrt.getPrecision().value)

    @pxrt.enforce_precision(i=("arr", "damp"))
    def pinv(self, arr, damp, **kwargs):
        return _dev.div(arr, 1 + damp)

    def gram(self):
        return self

    def cogram(self):
        return self

    @pxrt.enforce_precision()
    def trace(self, **kwargs):
        return float(self.dim)


class NullOp(pxa.LinOp):
    """Null operator (base.py:62-113)."""

    def __init__(self, shape):
        super().__init__(shape=shape)
        self.lipschitz = 0

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return _dev.zeros((*arr.shape[:-1], self.codim), arr)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        return _dev.zeros((*arr.shape[:-1], self.dim), arr)

    def gram(self):
        return NullOp(shape=(self.dim, self.dim)).asop(pxa.SelfAdjointOp).squeeze()

    def cogram(self):
        return NullOp(shape=(self.codim, self.codim)).asop(pxa.SelfAdjointOp).squeeze()

    @pxrt.enforce_precision()
    def trace(self, **kwargs):
        return 0


def NullFunc(dim):
    """Null functional (base.py:116-124)."""
    op = NullOp(shape=(1, dim)).squeeze()
    op._name = "NullFunc"
    return op


def HomothetyOp(dim, cst):
    """``cst * I`` (base.py:127-210)."""
    assert np.isscalar(cst)
    if np.isclose(cst, 0):
        return NullOp(shape=(dim, dim))
    if np.isclose(cst, 1):
        return IdentityOp(dim=dim)

    @pxrt.enforce_precision(i="arr")
    def op_apply(_, arr):
        return _dev.axpby(_._cst, arr)

    @pxrt.enforce_precision(i=("arr", "damp"))
    def op_pinv(_, arr, damp, **kwargs):
        return _dev.div(_dev.axpby(_._cst, arr), _._cst**2 + damp)

    op = from_source(
        cls=pxa.PosDefOp if cst > 0 else pxa.SelfAdjointOp,
        shape=(dim, dim),
        embed=dict(_name="HomothetyOp", _cst=float(cst), _lipschitz=float(abs(cst))),
        apply=op_apply,
        pinv=op_pinv,
        estimate_lipschitz=lambda _, **kw: abs(_._cst),
        gram=lambda _: HomothetyOp(dim=_.dim, cst=_._cst**2),
        cogram=lambda _: HomothetyOp(dim=_.dim, cst=_._cst**2),
        trace=lambda _, **kw: float(_._cst * _.dim),
    )
    op.adjoint = op.apply
    return op


def DiagonalOp(vec, enable_warnings=True):
    """Element-wise scaling by a device vector (base.py:213-331)."""
    vec = to_device(vec) if not is_device_array(vec) else vec
    dim = vec.numel()

    @pxrt.enforce_precision(i="arr")
    def op_apply(_, arr):
        v = pxrt.coerce(_._vec)
        return _dev.mul(arr, v.expand_as(arr).contiguous()) if arr.ndim > 1 else _dev.mul(arr, v)

    op = from_source(cls=pxa.SelfAdjointOp, shape=(dim, dim), embed=dict(_name="DiagonalOp", _vec=vec), apply=op_apply)
    op.adjoint = op.apply
    op.lipschitz = float(_dev.row_reduce(_dev.RED_MAXABS, vec.reshape(1, -1)).cpu()[0])
    return op


def Sum(arg_shape, axis=None):
    """Sum over all entries (reference operator/linop/reduce.py) — the full-reduction case only."""
    dim = int(np.prod(arg_shape))
    if axis is not None and tuple(np.atleast_1d(axis)) != tuple(range(len(arg_shape))):
        raise NotImplementedError("pyxu_amd: Sum over a subset of axes is outside the hot-path scope.")

    @pxrt.enforce_precision(i="arr")
    def op_apply(_, arr):
        from pyxu_amd.abc.operator import _rowsum

        return _rowsum(arr)

    @pxrt.enforce_precision(i="arr")
    def op_adjoint(_, arr):
        z = _dev.require(arr)
        rows = z.numel()
        out = _dev.empty((*z.shape[:-1], _.dim), z)
        return _dev.copy2d(z, out, rows, _.dim, 1, _.dim, col_stride=0)  # each row's scalar repeated

    op = from_source(cls=pxa.LinFunc, shape=(1, dim), embed=dict(_name="Sum"), apply=op_apply, adjoint=op_adjoint)
    op.lipschitz = np.sqrt(dim)
    return op


def _like(tdt):
    """A 1-element device tensor of torch dtype `tdt` (dtype carrier for _dev.cast)."""
    import torch

    return torch.empty((1,), dtype=tdt, device="cuda")


def _ExplicitLinOp(cls, mat, enable_warnings=True):
    """Dense-matrix operator of class `cls` (LinOp / LinFunc / SquareOp ...) (base.py:334-512).

    ``apply`` = A.dot(x) per stacked row, ``adjoint`` = A^T.dot(z), on the MI355X (pxa_dense_matmat).
    """
    if not is_device_array(mat):
        mat = to_device(np.asarray(mat))
    if mat.ndim != 2:
        raise ValueError("pyxu_amd: from_array expects a 2-D dense matrix.")
    mat = mat.contiguous()
    cache = {}

    def _mat_as(_, dtype):
        m = cache.get(dtype)
        if m is None:
            if _._mat.dtype != dtype and _._enable_warnings:
                warnings.warn("Computation may not be performed at the requested precision.")
            m = _._mat if _._mat.dtype == dtype else _dev.cast(_._mat, _like(dtype))
            cache[dtype] = m
        return m

    def _matmat(_, arr, trans):
        sh = arr.shape[:-1]
        x = arr.reshape(-1, arr.shape[-1]).contiguous()
        y = _dev.dense_matmat(_mat_as(_, x.dtype), x, trans)
        return y.reshape(*sh, -1)

    @pxrt.enforce_precision(i="arr")
    def op_apply(_, arr):
        return _matmat(_, arr, 0)

    @pxrt.enforce_precision(i="arr")
    def op_adjoint(_, arr):
        return _matmat(_, arr, 1)

    def op_asarray(_, xp=None, dtype=None):
        dtype = pxrt.getPrecision().value if dtype is None else np.dtype(dtype)
        tdt = pxrt.Width(np.dtype(dtype)).torch
        A = _._mat if _._mat.dtype == tdt else _dev.cast(_._mat, _like(tdt))
        return A.cpu().numpy() if xp is np else A

    klass = cls
    if klass is pxa.LinOp and mat.shape[0] == mat.shape[1]:
        klass = pxa.SquareOp
    op = from_source(
        cls=klass,
        shape=tuple(mat.shape),
        embed=dict(_name="_ExplicitLinOp", _mat=mat, _enable_warnings=bool(enable_warnings)),
        apply=op_apply,
        adjoint=op_adjoint,
        asarray=op_asarray,
    )
    return op
