"""
Block operators (mirrors reference ``pyxu.operator.blocks``, src/pyxu/operator/blocks.py:1-1008):
``stack`` / ``vstack`` / ``hstack`` / ``block_diag`` / ``block`` / ``coo_block``.

Same construction rules, property inference, Lipschitz bounds and evaluation order as the
reference's ``_COOBlock`` (blocks.py:474-1008): a block reads its column band ``arr[..., off:off+dim]``
of the input and its result is summed into its row band of the output, blocks of one row summed in
insertion order starting from 0 (the reference's Python ``sum``), row bands concatenated along the
last axis.  On the MI355X the data movement is done in place by ``pxa_copy2d`` (csrc/array.hip):
column bands of a 1-D input are views (no copy), stacked inputs are gathered with one strided copy,
and each block result is written / accumulated directly into its band of the preallocated output,
so ``vstack.apply`` / ``hstack.adjoint`` cost one pass per block and no ``concatenate``.  The
reference's ``parallel=True`` (Dask threads, blocks.py:474-509) is accepted and ignored: every
block already runs on the whole GPU.
"""
import collections
import itertools
import types

import numpy as np

import pyxu_amd.abc.operator as pxo
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["stack", "vstack", "hstack", "block_diag", "block", "coo_block"]


def stack(ops, axis, **kwargs):
    """vstack (axis=0) or hstack (axis=1) (blocks.py:30-71)."""
    axis = int(axis)
    assert axis in {0, 1}, f"axis: out-of-bounds axis '{axis}'."
    return {0: vstack, 1: hstack}[axis](ops, **kwargs)


def vstack(ops, **kwargs):
    """[O_1; ...; O_N] (blocks.py:74-137): (c1 + ... + cN, d)."""
    n = len(ops)
    op = _COOBlock((ops, (tuple(range(n)), [0] * n)), grid_shape=(n, 1), parallel=kwargs.get("parallel", False)).op()
    if hasattr(op, "_block"):
        op._expr = types.MethodType(lambda _: ("vstack", *[_._block[(r, 0)] for r in range(_._grid_shape[0])]), op)
    return op


def hstack(ops, **kwargs):
    """[O_1, ..., O_N] (blocks.py:140-201): (c, d1 + ... + dN)."""
    n = len(ops)
    op = _COOBlock((ops, ([0] * n, tuple(range(n)))), grid_shape=(1, n), parallel=kwargs.get("parallel", False)).op()
    if hasattr(op, "_block"):
        op._expr = types.MethodType(lambda _: ("hstack", *[_._block[(0, c)] for c in range(_._grid_shape[1])]), op)
    return op


def block_diag(ops, **kwargs):
    """diag(O_1, ..., O_N) (blocks.py:204-313)."""
    n = len(ops)
    op = _COOBlock((ops, (tuple(range(n)), tuple(range(n)))), grid_shape=(n, n), parallel=kwargs.get("parallel", False)).op()
    if not hasattr(op, "_block"):
        return op

    def op_svdvals(_, **kw):
        if not _.has(pxo.Property.LINEAR):
            raise NotImplementedError
        k = kw.get("k", 1)
        if kw.get("which", "LM").upper() == "SM":
            return _.__class__.svdvals(_, **kw)
        parts = np.concatenate([np.atleast_1d(np.asarray(o.svdvals(**kw))) for o in _._block.values()])
        return np.sort(parts, axis=None)[-k:]

    @pxrt.enforce_precision(i=("arr", "damp"))
    def op_pinv(_, arr, damp, **kw):
        if not _.has(pxo.Property.LINEAR):
            raise NotImplementedError
        x = _dev.require(arr)
        out = _dev.empty((*x.shape[:-1], _.dim), x)
        rows = x.numel() // max(x.shape[-1], 1)
        for idx in sorted(_._block):
            o = _._block[idx]
            r_off = _._block_offset[idx][0]
            c_off = _._block_offset[idx][1]
            p = _dev.require(o.pinv(_dev.take_cols(x, r_off, o.codim), damp, **kw))
            _dev.copy2d(p, out, rows, o.dim, o.dim, _.dim, dst_off=c_off)
        return out

    @pxrt.enforce_precision()
    def op_trace(_, **kw):
        if not _.has(pxo.Property.LINEAR_SQUARE):
            raise NotImplementedError
        if all(o.has(pxo.Property.LINEAR_SQUARE) for o in _._block.values()):
            return sum(o.trace(**kw) for o in _._block.values())
        return pxo.SquareOp.trace(_, **kw)

    op.svdvals = types.MethodType(op_svdvals, op)
    op.pinv = types.MethodType(op_pinv, op)
    op.trace = types.MethodType(op_trace, op)
    op._expr = types.MethodType(lambda _: ("block_diag", *[_._block[k] for k in sorted(_._block)]), op)
    return op


def block(ops, order, **kwargs):
    """Dense block-defined operator (blocks.py:316-383): order 0 = vstack inner, hstack outer; 1 = the
    converse."""
    order = int(order)
    assert order in {0, 1}, f"order: out-of-bounds order '{order}'."
    inner = {0: vstack, 1: hstack}[order]
    outer = {0: hstack, 1: vstack}[order]
    return outer([inner(row, **kwargs) for row in ops], **kwargs)


def coo_block(ops, grid_shape, *, parallel=False):
    """(Sparse) block-defined operator in COOrdinate format (blocks.py:387-471)."""
    return _COOBlock(ops=ops, grid_shape=grid_shape, parallel=parallel).op()


# ----------------------------------------------------------------------------- device helpers
def _lead(x):
    return x.shape[:-1], (x.numel() // max(x.shape[-1], 1) if x.numel() else int(np.prod(x.shape[:-1])))


def _band_sum(out, rows, ld, off, parts):
    """out[..., off:off + n] = 0 + p_0 + p_1 + ... (device, in order): the reference's sum(rows[r])."""
    for k, p in enumerate(parts):
        p = _dev.require(p)
        n = p.shape[-1] if p.ndim else 1
        _dev.copy2d(p, out, rows, n, n, ld, dst_off=off, accumulate=2 if k == 0 else 1)


class _COOBlock:
    """See coo_block() (blocks.py:474-1008)."""

    def __init__(self, ops, grid_shape, parallel=False):
        self._grid_shape = tuple(int(g) for g in grid_shape)
        self._parallel = bool(parallel)
        self._init_spec(ops)

    def op(self):
        blk = self._block
        if len(blk) == 1:
            _, op = blk.popitem()
            return op
        from pyxu_amd.abc import arithmetic

        op = self._infer_op()
        op._block = self._block
        op._block_offset = self._block_offset
        op._grid_shape = self._grid_shape
        op._parallel = self._parallel
        for p in op.properties():
            for name in p.arithmetic_methods():
                func = getattr(self.__class__, name, None)
                if func is not None:
                    setattr(op, name, types.MethodType(func, op))
        arithmetic.Rule._propagate_constants(op)
        return op

    def _init_spec(self, ops):
        data, (i, j) = ops
        n_row, n_col, n_block = *self._grid_shape, len(data)
        msg = "Incorrect COO parametrization"
        assert n_block == len(i) == len(j), msg
        assert 0 < n_block <= n_row * n_col, msg
        assert 0 <= min(i) <= max(i) < n_row, msg
        assert 0 <= min(j) <= max(j) < n_col, msg
        row = collections.defaultdict(list)
        col = collections.defaultdict(list)
        for d, _i, _j in zip(data, i, j):
            row[_i].append(d)
            col[_j].append(d)
        for k, v in row.items():
            assert len({o.codim for o in v}) == 1, f"All sub-operators on row {k} must have same codomain size."
        for k, v in col.items():
            assert len({o.dim for o in v}) == 1, f"All sub-operators on column {k} must have same domain size."
        assert len(row) == n_row, "Coarse grid contains empty rows: cannot infer fine-grid dimensions."
        assert len(col) == n_col, "Coarse grid contains empty columns: cannot infer fine-grid dimensions."
        self._block = {(int(_i), int(_j)): d.squeeze() for d, _i, _j in zip(data, i, j)}
        row_off = np.cumsum([row[k][0].codim for k in range(n_row)])
        col_off = np.cumsum([col[k][0].dim for k in range(n_col)])
        self._block_offset = {
            (r, c): (0 if r == 0 else int(row_off[r - 1]), 0 if c == 0 else int(col_off[c - 1]))
            for r in range(n_row) for c in range(n_col)
        }

    def _infer_op(self):
        blk = self._block
        row = collections.defaultdict(list)
        col = collections.defaultdict(list)
        for (r, c), o in blk.items():
            row[r].append(o)
            col[c].append(o)
        n_row, n_col = len(row), len(col)
        codim = sum(v[0].codim for v in row.values())
        dim = sum(v[0].dim for v in col.values())
        P = pxo.Property
        props = set.intersection(*[set(o.properties()) for o in blk.values()])
        if codim > 1:
            props -= {P.FUNCTIONAL, P.PROXIMABLE, P.DIFFERENTIABLE_FUNCTION, P.QUADRATIC}
        if n_row == n_col == len(blk) and all((r, r) in blk for r in range(n_row)):
            pass  # block_diag
        elif codim == 1:  # hstack of functionals: quadratic iff quadratics + linear terms
            if all(o.has(P.QUADRATIC) for o in blk.values()):
                props.add(P.QUADRATIC)
            elif any(o.has(P.QUADRATIC) for o in blk.values()):
                if all(o.has(P.LINEAR) for o in blk.values() if not o.has(P.QUADRATIC)):
                    props.add(P.QUADRATIC)
        else:
            props &= {P.CAN_EVAL, P.DIFFERENTIABLE, P.LINEAR}
            if codim == dim and P.LINEAR in props:
                props.add(P.LINEAR_SQUARE)
        klass = pxo.Operator._infer_operator_type(props)
        return klass(shape=(codim, dim))

    # ------------------------------------------------------------------ arithmetic methods (bound)
    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        lead, rows = _lead(x)
        out = _dev.empty((*lead, self.codim), x)
        parts = collections.defaultdict(list)
        for idx, o in self._block.items():
            parts[idx[0]].append(o.apply(_dev.take_cols(x, self._block_offset[idx][1], o.dim)))
        for r in range(len(parts)):
            _band_sum(out, rows, self.codim, self._block_offset[(r, 0)][0], parts[r])
        return out

    def __call__(self, arr):
        return self.apply(arr)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        if not self.has(pxo.Property.LINEAR):
            raise NotImplementedError
        z = _dev.require(arr)
        lead, rows = _lead(z)
        out = _dev.empty((*lead, self.dim), z)
        parts = collections.defaultdict(list)
        for idx, o in self._block.items():
            parts[idx[1]].append(o.adjoint(_dev.take_cols(z, self._block_offset[idx][0], o.codim)))
        for c in range(len(parts)):
            _band_sum(out, rows, self.dim, self._block_offset[(0, c)][1], parts[c])
        return out

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        if not self.has(pxo.Property.PROXIMABLE):
            raise NotImplementedError
        x = _dev.require(arr)
        lead, rows = _lead(x)
        out = _dev.empty(x.shape, x)
        for c in range(len(self._block)):
            o = self._block[(0, c)]
            off = self._block_offset[(0, c)][1]
            p = _dev.require(o.prox(_dev.take_cols(x, off, o.dim), tau))
            _dev.copy2d(p, out, rows, o.dim, o.dim, self.dim, dst_off=off)
        return out

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        if not self.has(pxo.Property.DIFFERENTIABLE_FUNCTION):
            raise NotImplementedError
        x = _dev.require(arr)
        lead, rows = _lead(x)
        out = _dev.empty(x.shape, x)
        for c in range(len(self._block)):
            o = self._block[(0, c)]
            off = self._block_offset[(0, c)][1]
            p = _dev.require(o.grad(_dev.take_cols(x, off, o.dim)))
            _dev.copy2d(p, out, rows, o.dim, o.dim, self.dim, dst_off=off)
        return out

    def jacobian(self, arr):
        if not self.has(pxo.Property.DIFFERENTIABLE):
            raise NotImplementedError
        if self.has(pxo.Property.LINEAR):
            return self
        data, i, j = [], [], []
        for (r, c), o in self._block.items():
            off = self._block_offset[(r, c)][1]
            data.append(o.jacobian(arr[off:off + o.dim]))
            i.append(r)
            j.append(c)
        return _COOBlock(ops=(data, (i, j)), grid_shape=self._grid_shape, parallel=self._parallel).op()

    def _quad_spec(self):
        if not self.has(pxo.Property.QUADRATIC):
            raise NotImplementedError
        from pyxu_amd.operator.linop import NullOp

        parts = dict()
        for idx, o in self._block.items():
            if o.has(pxo.Property.QUADRATIC):
                parts[idx] = o._quad_spec()
            else:  # necessarily LINEAR
                parts[idx] = (NullOp(shape=(o.dim, o.dim)).asop(pxo.PosDefOp), o, 0)
        Q, c, t = zip(*[parts[k] for k in sorted(parts)])
        return block_diag(Q), hstack(c), sum(t)

    def estimate_lipschitz(self, **kwargs):
        Ls = np.zeros(self._grid_shape)
        if "__rule" in kwargs:
            for (r, c), o in self._block.items():
                Ls[r, c] = float(o.lipschitz) ** 2
        elif self.has(pxo.Property.LINEAR):
            return self.__class__.estimate_lipschitz(self, **kwargs)
        else:
            for (r, c), o in self._block.items():
                Ls[r, c] = float(o.estimate_lipschitz(**kwargs)) ** 2
        if np.allclose(Ls.sum(), np.trace(Ls)):  # block-diagonal: max; otherwise the sum bound
            return float(np.sqrt(Ls.max()))
        return float(np.sqrt(Ls.sum()))

    def estimate_diff_lipschitz(self, **kwargs):
        if not self.has(pxo.Property.DIFFERENTIABLE):
            raise NotImplementedError
        dLs = np.zeros(self._grid_shape)
        if "__rule" in kwargs:
            for (r, c), o in self._block.items():
                dLs[r, c] = float(o.diff_lipschitz) ** 2
        elif self.has(pxo.Property.QUADRATIC):
            return pxo.QuadraticFunc.estimate_diff_lipschitz(self, **kwargs)
        elif self.has(pxo.Property.LINEAR):
            return 0
        else:
            for (r, c), o in self._block.items():
                dLs[r, c] = float(o.estimate_diff_lipschitz(**kwargs)) ** 2
        if np.allclose(dLs.sum(), np.trace(dLs)):
            return float(np.sqrt(dLs.max()))
        return float(np.sqrt(dLs.sum()))

    def asarray(self, xp=None, dtype=None):
        if not self.has(pxo.Property.LINEAR):
            raise NotImplementedError
        import torch

        dtype = pxrt.getPrecision().value if dtype is None else np.dtype(dtype)
        A = torch.zeros(self.shape, dtype=pxrt.Width(np.dtype(dtype)).torch, device="cuda")
        for idx, o in self._block.items():
            p = _dev.require(o.asarray(dtype=dtype))
            r_o, c_o = self._block_offset[idx]
            r_s, c_s = o.shape
            _dev.copy2d(p, A, r_s, c_s, c_s, self.dim, dst_off=r_o * self.dim + c_o)
        return A.cpu().numpy() if xp is np else A

    def _expr(self):
        head = "coo_block[" + ", ".join(map(str, self._grid_shape)) + "]"
        return (head, *[o for _, o in sorted(self._block.items())])

    def gram(self):
        if not self.has(pxo.Property.LINEAR):
            raise NotImplementedError
        blk = self._block
        n_row, n_col = self._grid_shape
        ops = collections.defaultdict(list)
        for r, c in itertools.product(range(n_col), repeat=2):
            for k in range(n_row):
                if (k, r) in blk and (k, c) in blk:
                    ops[(r, c)].append(blk[(k, r)].gram() if r == c else blk[(k, r)].T * blk[(k, c)])
        data, i, j = [], [], []
        for (r, c), lst in ops.items():
            acc = lst[0]
            for o in lst[1:]:
                acc = acc + o
            data.append(acc)
            i.append(r)
            j.append(c)
        G = _COOBlock(ops=(data, (i, j)), grid_shape=(n_col, n_col), parallel=self._parallel).op()
        return G.asop(pxo.SelfAdjointOp).squeeze()

    def cogram(self):
        if not self.has(pxo.Property.LINEAR):
            raise NotImplementedError
        return (self * self.T).asop(pxo.SelfAdjointOp).squeeze()
