"""SubSample / Trim (reference operator/linop/select.py:18-251) as public LinOps.

The index specifier is resolved once on the host: numpy's own indexing of ``arange(N)`` gives the
flat source position of every output sample in output order, so integers, slices (any step),
integer lists (with numpy's advanced-index broadcasting) and boolean masks all reduce to one
int64 vector on the device.  apply = pxa_gather_cols, adjoint = zero fill + pxa_scatter_cols;
a box selection (unit-step slices only, the Trim case) runs on pxa_trim instead."""
import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["SubSample", "Trim"]


class SubSample(pxa.LinOp):
    """(..., prod(arg_shape)) -> (..., prod(sub_shape)) = arr[..., *indices]; Lipschitz 1."""

    def __init__(self, arg_shape, *indices):
        if np.isscalar(arg_shape):
            arg_shape = (arg_shape,)
        self._arg_shape = tuple(int(n) for n in arg_shape)
        assert 1 <= len(indices) <= len(self._arg_shape)
        idx = [slice(None)] * len(self._arg_shape)
        for i, s in enumerate(indices):
            if isinstance(s, (int, np.integer)):
                s = slice(int(s), int(s) + 1)
            elif not isinstance(s, slice):
                from pyxu_amd.util import to_NUMPY

                s = to_NUMPY(s) if hasattr(s, "device") else np.asarray(s)
            idx[i] = s
        self._idx = tuple(idx)
        pos = np.arange(int(np.prod(self._arg_shape)), dtype=np.int64).reshape(self._arg_shape)[self._idx]
        self._sub_shape = np.atleast_1d(pos).shape
        super().__init__(shape=(int(np.prod(self._sub_shape)), int(np.prod(self._arg_shape))))
        self.lipschitz = 1
        pos = np.ascontiguousarray(pos.reshape(-1))
        # box fast path: every axis a unit-step slice -> the pad/trim kernel
        self._box = None
        if all(isinstance(s, slice) and s.step in (None, 1) for s in self._idx):
            lo, hi = [], []
            for s, n in zip(self._idx, self._arg_shape):
                a, b, _ = s.indices(n)
                b = max(a, b)
                lo.append(a)
                hi.append(n - b)
            if all(n - l - h > 0 for n, l, h in zip(self._arg_shape, lo, hi)):
                self._box = (lo, hi)
        # adjoint: numpy's `out[idx] = arr` keeps the LAST write of a repeated position
        _, last = np.unique(pos[::-1], return_index=True)
        keep = np.sort(pos.size - 1 - last)
        self._pos_host = pos
        self._uniq = keep.size == pos.size
        self._keep_host = keep
        self._dev_cache = {}

    def _dev_idx(self, like, which):
        key = (which, like.device)
        if key not in self._dev_cache:
            from pyxu_amd.util import to_device

            host = {"pos": self._pos_host, "keep": self._keep_host,
                    "upos": np.ascontiguousarray(self._pos_host[self._keep_host])}[which]
            self._dev_cache[key] = to_device(host)
        return self._dev_cache[key]

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        sh = x.shape[:-1]
        stack = int(np.prod(sh))
        if self._box is not None:
            y = _dev.trim(x, stack, self._arg_shape, self._box[0], self._box[1], embed=False)
            return y.reshape(*sh, self.codim)
        return _dev.gather_cols(x, self._dev_idx(x, "pos"))

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        y = _dev.require(arr)
        sh = y.shape[:-1]
        stack = int(np.prod(sh))
        if self._box is not None:
            big = tuple(self._arg_shape)
            out = _dev.trim(y, stack, big, self._box[0], self._box[1], embed=True)
            return out.reshape(*sh, self.dim)
        if self._uniq:
            return _dev.scatter_cols(y, self._dev_idx(y, "pos"), self.dim)
        # a repeated position keeps only its last write: scatter the surviving columns
        return _dev.scatter_cols(_dev.gather_cols(y, self._dev_idx(y, "keep")), self._dev_idx(y, "upos"), self.dim)

    def svdvals(self, **kwargs):
        return pxa.UnitOp.svdvals(self, **kwargs)

    def gram(self):
        return _SubSampleGram(self)

    def cogram(self):
        from pyxu_amd.operator.linop.base import IdentityOp

        return IdentityOp(dim=self.codim).squeeze()

    @pxrt.enforce_precision(i=("arr", "damp"))
    def pinv(self, arr, damp, **kwargs):
        return _dev.div(self.adjoint(arr), 1 + damp)

    def dagger(self, damp, **kwargs):
        return self.T / (1 + damp)


class _SubSampleGram(pxa.OrthProjOp):
    """S^T S: the orthogonal projection onto the selected samples (select.py:173-186)."""

    def __init__(self, op):
        super().__init__(shape=(op.dim, op.dim))
        self._op = op

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._op.adjoint(self._op.apply(arr))


def Trim(arg_shape, trim_width):
    """Trim each axis by (head, tail) samples: a SubSample with unit-step slices (select.py:205-251)."""
    from pyxu_amd.operator.linop.pad import _canonical_widths

    arg_shape = tuple(arg_shape)
    widths = _canonical_widths(trim_width, len(arg_shape), "trim_width")
    return SubSample(arg_shape, *[slice(h, n - t) for (h, t), n in zip(widths, arg_shape)])
