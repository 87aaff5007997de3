"""
Operator class lattice (mirrors reference ``pyxu.abc.operator``, src/pyxu/abc/operator.py).

Same class names, Property tags, arithmetic API and Lipschitz bookkeeping as the reference; every
numerical method evaluates on MI355X device tensors through ``pyxu_amd._dev`` (HIP C-ABI).
"""
import collections
import copy
import enum
import types
import warnings

import numpy as np

import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.util import copy_if_unsafe

__all__ = [
    "Property",
    "Operator",
    "Map",
    "Func",
    "DiffMap",
    "DiffFunc",
    "ProxFunc",
    "ProxDiffFunc",
    "QuadraticFunc",
    "LinOp",
    "LinFunc",
    "SquareOp",
    "NormalOp",
    "SelfAdjointOp",
    "UnitOp",
    "ProjOp",
    "OrthProjOp",
    "PosDefOp",
]


class Property(enum.Enum):
    """Mathematical properties (operator.py:20-73)."""

    CAN_EVAL = enum.auto()
    FUNCTIONAL = enum.auto()
    PROXIMABLE = enum.auto()
    DIFFERENTIABLE = enum.auto()
    DIFFERENTIABLE_FUNCTION = enum.auto()
    LINEAR = enum.auto()
    LINEAR_SQUARE = enum.auto()
    LINEAR_NORMAL = enum.auto()
    LINEAR_IDEMPOTENT = enum.auto()
    LINEAR_SELF_ADJOINT = enum.auto()
    LINEAR_POSITIVE_DEFINITE = enum.auto()
    LINEAR_UNITARY = enum.auto()
    QUADRATIC = enum.auto()

    def arithmetic_methods(self) -> frozenset:
        data = collections.defaultdict(list)
        data[self.CAN_EVAL].extend(["apply", "__call__", "estimate_lipschitz", "_expr"])
        data[self.FUNCTIONAL].append("asloss")
        data[self.PROXIMABLE].append("prox")
        data[self.DIFFERENTIABLE].extend(["jacobian", "estimate_diff_lipschitz"])
        data[self.DIFFERENTIABLE_FUNCTION].append("grad")
        data[self.LINEAR].extend(["adjoint", "asarray", "svdvals", "pinv", "gram", "cogram"])
        data[self.LINEAR_SQUARE].append("trace")
        data[self.QUADRATIC].append("_quad_spec")
        return frozenset(data[self])


def _is_real(x) -> bool:
    if isinstance(x, (int, float, np.integer, np.floating)) and not isinstance(x, bool):
        return True
    if isinstance(x, np.ndarray) and x.size == 1:
        return True
    return False


# ----------------------------------------------------------------------------- small array helpers
def _rows(arr):
    """(..., M) -> (rows, M) contiguous view."""
    return arr.reshape(-1, arr.shape[-1])


def _rowsum(arr):
    """sum over the last axis, keepdims, in arr's dtype (device)."""
    s = _dev.row_reduce(_dev.RED_SUM, _rows(arr))
    return _dev.cast(s, arr).reshape(*arr.shape[:-1], 1)


def _dot(a, b):
    s = _dev.row_reduce(_dev.RED_DOT, _rows(a), _rows(b))
    return _dev.cast(s, a).reshape(*a.shape[:-1], 1)


class Operator:
    """Abstract base class of all operators (operator.py:76-501)."""

    __array_priority__ = np.inf

    def __init__(self, shape):
        shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        assert len(shape) == 2, f"shape: expected (N, M), got {shape}."
        self._shape = shape
        self._name = self.__class__.__name__

    # Public Interface ------------------------------------------------------
    @property
    def shape(self):
        return self._shape

    @property
    def dim(self) -> int:
        return self._shape[1]

    @property
    def codim(self) -> int:
        return self._shape[0]

    @classmethod
    def properties(cls) -> frozenset:
        return frozenset()

    @classmethod
    def has(cls, prop) -> bool:
        if isinstance(prop, Property):
            prop = (prop,)
        return frozenset(prop) <= cls.properties()

    def asop(self, cast_to):
        """Recast to another core operator class (operator.py:137-176)."""
        if cast_to not in _core_operators():
            raise ValueError(f"cast_to: expected a core base-class, got {cast_to}.")
        p_core = frozenset(self.properties())
        p_shell = frozenset(cast_to.properties())
        if p_shell <= p_core:
            return self
        op = cast_to(shape=self.shape)
        op._core = self
        for p in p_shell & p_core:
            for m in p.arithmetic_methods():
                setattr(op, m, getattr(self, m))
        # constants carry over
        if hasattr(self, "_lipschitz"):
            op._lipschitz = self._lipschitz
        if hasattr(self, "_diff_lipschitz") and op.has(Property.DIFFERENTIABLE):
            op._diff_lipschitz = self._diff_lipschitz
        op._name = self._name
        return op

    # Arithmetic ------------------------------------------------------------
    def __add__(self, other):
        from pyxu_amd.abc import arithmetic

        if isinstance(other, Operator):
            return arithmetic.AddRule(lhs=self, rhs=other).op()
        return NotImplemented

    def __sub__(self, other):
        from pyxu_amd.abc import arithmetic

        if isinstance(other, Operator):
            return arithmetic.AddRule(lhs=self, rhs=-other).op()
        return NotImplemented

    def __neg__(self):
        from pyxu_amd.abc import arithmetic

        return arithmetic.ScaleRule(op=self, cst=-1).op()

    def __mul__(self, other):
        from pyxu_amd.abc import arithmetic

        if isinstance(other, Operator):
            return arithmetic.ChainRule(lhs=self, rhs=other).op()
        if _is_real(other):
            return arithmetic.ScaleRule(op=self, cst=float(other)).op()
        return NotImplemented

    def __rmul__(self, other):
        from pyxu_amd.abc import arithmetic

        if _is_real(other):
            return arithmetic.ScaleRule(op=self, cst=float(other)).op()
        return NotImplemented

    def __truediv__(self, other):
        from pyxu_amd.abc import arithmetic

        if _is_real(other):
            return arithmetic.ScaleRule(op=self, cst=float(1 / other)).op()
        return NotImplemented

    def __pow__(self, k):
        from pyxu_amd.abc import arithmetic

        if isinstance(k, (int, np.integer)) and k >= 0:
            return arithmetic.PowerRule(op=self, k=int(k)).op()
        return NotImplemented

    def __matmul__(self, other):
        return NotImplemented

    def __rmatmul__(self, other):
        return NotImplemented

    def argscale(self, scalar):
        from pyxu_amd.abc import arithmetic

        assert _is_real(scalar)
        return arithmetic.ArgScaleRule(op=self, cst=float(scalar)).op()

    def argshift(self, shift):
        from pyxu_amd.abc import arithmetic

        if _is_real(shift):
            shift = float(shift)
        return arithmetic.ArgShiftRule(op=self, cst=shift).op()

    # Internal helpers -------------------------------------------------------
    @staticmethod
    def _infer_operator_type(prop):
        prop = frozenset(prop)
        for op in _core_operators():
            if op.properties() == prop:
                return op
        raise ValueError(f"No operator found with properties {prop}.")

    def squeeze(self):
        """Cast to the right core sub-type given the codomain dimension (operator.py:395-415)."""
        p = set(self.properties())
        if self.codim == 1:
            p.add(Property.FUNCTIONAL)
            if Property.DIFFERENTIABLE in self.properties():
                p.add(Property.DIFFERENTIABLE_FUNCTION)
            if Property.LINEAR in self.properties():
                for p_ in Property:
                    if p_.name.startswith("LINEAR_"):
                        p.discard(p_)
                p.add(Property.PROXIMABLE)
        elif self.codim == self.dim:
            if Property.LINEAR in self.properties():
                p.add(Property.LINEAR_SQUARE)
        return self.asop(self._infer_operator_type(p))

    def __repr__(self) -> str:
        return f"{self._name}{self.shape}"

    def _expr(self) -> tuple:
        return (self,)

    def expr(self, level: int = 0, strip: bool = True) -> str:
        fmt = lambda obj, lvl: ("." * lvl) + str(obj)
        lines = []
        head, *tail = self._expr()
        head = f"{repr(head)}," if len(tail) == 0 else f"[{head}, ==> {repr(self)}"
        lines.append(fmt(head, level))
        for t in tail:
            if isinstance(t, Operator):
                lines += t.expr(level=level + 1, strip=False).split("\n")
            else:
                lines.append(fmt(f"{t},", level + 1))
        if len(tail) > 0:
            lines[-1] = lines[-1][:-1] + "],"
        out = "\n".join(lines)
        return out.strip(",") if strip else out


class Map(Operator):
    """Real-valued maps (operator.py:504-637)."""

    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.CAN_EVAL})

    def __init__(self, shape):
        super().__init__(shape=shape)
        self.lipschitz = np.inf

    def apply(self, arr):
        raise NotImplementedError

    def __call__(self, arr):
        return self.apply(arr)

    @property
    def lipschitz(self):
        if not hasattr(self, "_lipschitz"):
            self._lipschitz = self.estimate_lipschitz()
        return pxrt.coerce(self._lipschitz)

    @lipschitz.setter
    def lipschitz(self, L):
        assert L >= 0
        self._lipschitz = float(L)
        if not self.has(Property.LINEAR):

            def op_estimate_lipschitz(_, **kwargs):
                return _._lipschitz

            self.estimate_lipschitz = types.MethodType(op_estimate_lipschitz, self)

    def estimate_lipschitz(self, **kwargs):
        raise NotImplementedError


class Func(Map):
    """Real-valued functionals (operator.py:640-682)."""

    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.FUNCTIONAL})

    def __init__(self, shape):
        super().__init__(shape=shape)
        assert self.codim == 1, f"shape: expected (1, n), got {shape}."

    def asloss(self, data=None):
        raise NotImplementedError


class DiffMap(Map):
    """Differentiable maps (operator.py:685-844)."""

    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.DIFFERENTIABLE})

    def __init__(self, shape):
        super().__init__(shape=shape)
        self.diff_lipschitz = np.inf

    def jacobian(self, arr):
        raise NotImplementedError

    @property
    def diff_lipschitz(self):
        if not hasattr(self, "_diff_lipschitz"):
            self._diff_lipschitz = self.estimate_diff_lipschitz()
        return pxrt.coerce(self._diff_lipschitz)

    @diff_lipschitz.setter
    def diff_lipschitz(self, dL):
        assert dL >= 0
        self._diff_lipschitz = float(dL)
        if not self.has(Property.QUADRATIC):

            def op_estimate_diff_lipschitz(_, **kwargs):
                return _._diff_lipschitz

            self.estimate_diff_lipschitz = types.MethodType(op_estimate_diff_lipschitz, self)

    def estimate_diff_lipschitz(self, **kwargs):
        raise NotImplementedError


class ProxFunc(Func):
    """Proximable functionals (operator.py:847-1072)."""

    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.PROXIMABLE})

    def __init__(self, shape):
        super().__init__(shape=shape)

    def prox(self, arr, tau):
        raise NotImplementedError

    @pxrt.enforce_precision(i=("arr", "sigma"))
    def fenchel_prox(self, arr, sigma):
        """Moreau identity: ``arr - sigma prox_{f/sigma}(arr/sigma)`` (operator.py:905-944)."""
        out = self.prox(arr=_dev.div(arr, sigma), tau=1 / sigma)
        out = copy_if_unsafe(out)
        return _dev.axpby(-sigma, out, 1.0, arr, out=out)

    def moreau_envelope(self, mu):
        """Moreau envelope (operator.py:946-1072): a DiffFunc with grad ``(x - prox_{mu f}(x)) / mu``."""
        from pyxu_amd.operator.interop import from_source

        assert mu > 0, f"mu: expected positive, got {mu}"

        @pxrt.enforce_precision(i="arr")
        def op_apply(_, arr):
            x = self.prox(arr, tau=_._mu)
            out = copy_if_unsafe(self.apply(x))
            d = _dev.axpby(1.0, arr, -1.0, x)
            n2 = _dev.cast(_dev.row_reduce(_dev.RED_SUMSQ, _rows(d)), arr).reshape(*arr.shape[:-1], 1)
            return _dev.axpby(1.0, out, 0.5 / _._mu, n2)

        @pxrt.enforce_precision(i="arr")
        def op_grad(_, arr):
            x = _dev.axpby(1.0, arr, -1.0, self.prox(arr, tau=_._mu))
            return _dev.div(x, _._mu, out=x)

        op = from_source(
            cls=DiffFunc,
            shape=self.shape,
            embed=dict(_name="moreau_envelope", _mu=mu, _diff_lipschitz=float(1 / mu), _inner=self),
            apply=op_apply,
            grad=op_grad,
            _expr=lambda _: ("moreau_envelope", _._inner, _._mu),
        )
        return op


class DiffFunc(DiffMap, Func):
    """Differentiable functionals (operator.py:1075-1136)."""

    @classmethod
    def properties(cls):
        p = set()
        for klass in cls.__bases__:
            p |= klass.properties()
        p.add(Property.DIFFERENTIABLE_FUNCTION)
        return frozenset(p)

    def __init__(self, shape):
        DiffMap.__init__(self, shape)
        Func.__init__(self, shape)

    def jacobian(self, arr):
        return LinFunc.from_array(self.grad(arr))

    def grad(self, arr):
        raise NotImplementedError


class ProxDiffFunc(ProxFunc, DiffFunc):
    @classmethod
    def properties(cls):
        p = set()
        for klass in cls.__bases__:
            p |= klass.properties()
        return frozenset(p)

    def __init__(self, shape):
        ProxFunc.__init__(self, shape)
        DiffFunc.__init__(self, shape)


class QuadraticFunc(ProxDiffFunc):
    """``f(x) = 1/2 <x, Qx> + c^T x + t`` (operator.py:1169-1310); prox through CG."""

    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.QUADRATIC})

    def __init__(self, shape, Q=None, c=None, t=0):
        from pyxu_amd.operator.linop import IdentityOp, NullFunc

        super().__init__(shape=shape)
        self._Q = IdentityOp(dim=self.dim) if Q is None else Q
        self._c = NullFunc(dim=self.dim) if c is None else c
        self._t = t
        assert self._Q.shape == (self.dim, self.dim)
        assert self._c.shape == self.shape

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        Q, c, t = self._quad_spec()
        out = _dot(arr, Q.apply(arr))
        out = _dev.axpby(0.5, out, 1.0, c.apply(arr))
        return _dev.add_scalar(out, float(t), out=out)

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        Q, c, _ = self._quad_spec()
        out = copy_if_unsafe(Q.apply(arr))
        return _dev.axpby(1.0, out, 1.0, c.grad(arr), out=out)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        _, c, _ = self._quad_spec()
        b = _dev.div(arr, tau)
        b = _dev.axpby(1.0, b, -1.0, self._c_grad(c, arr), out=b)
        return self._prox_solve(b, tau)

    def _prox_cg(self, tau):
        """The CG sub-solver of prox(., tau) on Q + I / tau and its stop criterion (the default AbsError | a
        MaxIter(2 dim) sentinel), built once per (Q, tau) and reused by later calls: ADMM calls prox once per
        outer iteration with the same tau; the solver's state and the criterion's are reset per solve."""
        from pyxu_amd.operator.linop import HomothetyOp
        from pyxu_amd.opt.solver import CG
        from pyxu_amd.opt.stop import MaxIter

        Q, _, _ = self._quad_spec()
        key = (id(Q), float(tau))
        memo = self.__dict__.setdefault("_prox_memo", {})
        hit = memo.get(key)
        if hit is None or hit[0] is not Q:
            A = Q + HomothetyOp(cst=1 / tau, dim=Q.dim)
            slvr = CG(A=A, show_progress=False, _internal=True)
            hit = memo[key] = (Q, slvr, slvr.default_stop_crit() | MaxIter(n=2 * A.dim))
        return hit[1], hit[2]

    def _prox_solve(self, b, tau, preset=None):
        """x = (Q + I / tau)^-1 b by CG from x0 = 0 (operator.py:1273-1291); `preset`: CG.m_init's _preset
        (the start vectors already written, see ADMM._m_step_l1)."""
        slvr, stop_crit = self._prox_cg(tau)
        # = slvr.fit(b=b, stop_crit=stop_crit), no side files
        slvr._solve_inline(b=b, stop_crit=stop_crit, **({} if preset is None else {"_preset": preset}))
        # = slvr.solution() (CG: the state's x), without the history flush stats() does first: nobody reads an
        # inline sub-solve's history, and flushing its ~13 deferred records cost ~50 us between ADMM's x-update
        # and the rest of its step (C4 device timeline, r05zd)
        return slvr._mstate["x"]

    def asloss(self, data=None):
        from pyxu_amd.operator.func.loss import shift_loss

        return shift_loss(op=self, data=data)

    def estimate_diff_lipschitz(self, **kwargs):
        Q, *_ = self._quad_spec()
        return Q.estimate_lipschitz(**kwargs)

    def _c_grad(self, c, arr):
        """c.grad(arr) of the linear term: a constant vector (a linear functional's gradient does not depend on
        where it is taken), evaluated once per (stack shape, dtype, device) and reused.  For a loss composed
        with a dense K (ADMM's x-update, QuadraticFunc.prox -> CG) it costs two adjoint passes over K, which
        the reference repeats on every prox call (operator.py:1257-1280)."""
        key = (id(c), tuple(arr.shape[:-1]), arr.dtype, str(arr.device))
        memo = self.__dict__.setdefault("_c_grad_memo", {})
        hit = memo.get(key)
        if hit is None or hit[0] is not c:  # (c is held by the entry, so its id cannot be reused meanwhile)
            hit = memo[key] = (c, _dev.copy(c.grad(arr)))  # own buffer: callers only read it
        return hit[1]

    def _quad_spec(self):
        return (self._Q, self._c, self._t)


class LinOp(DiffMap):
    """Linear operators (operator.py:1313-1830)."""

    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR})

    def __init__(self, shape):
        super().__init__(shape=shape)
        self.diff_lipschitz = 0

    def adjoint(self, arr):
        raise NotImplementedError

    def jacobian(self, arr):
        return self

    @property
    def T(self):
        from pyxu_amd.abc import arithmetic

        return arithmetic.TransposeRule(op=self).op()

    def estimate_lipschitz(self, **kwargs):
        """A Lipschitz constant of the operator (operator.py:1440-1498).

        method="trace" (the default, as in the reference): sqrt of the Hutch++ estimate of
        tr(A^T A) (or tr(A A^T) when codim < dim) = ||A||_F, an upper bound of ||A||_2, with m = 126
        queries (pyxu_amd.math.linalg.hutchpp; `m`, `seed` forwarded).
        method="svd": the optimal constant ||A||_2 by a device power iteration on A^T A (``n_iter``,
        ``tol``, ``seed``), which converges to what the reference's svdvals(k=1) returns.
        """
        method = str(kwargs.get("method", "trace")).lower().strip()
        if method == "trace":
            if self.shape == (1, 1):
                return self._power_lipschitz(**kwargs)
            from pyxu_amd.math.linalg import hutchpp

            op = self.gram() if (self.codim >= self.dim) else self.cogram()
            tr = hutchpp(op, m=int(kwargs.get("m", 126)), seed=kwargs.get("seed"))
            return float(np.sqrt(max(tr, 0.0)))
        if method == "svd":
            return self._power_lipschitz(**kwargs)
        raise NotImplementedError(f"method={method!r}")

    def _power_lipschitz(self, **kwargs):
        """||A||_2 by power iteration on A^T A, every product on the device."""
        n_iter = int(kwargs.get("n_iter", 200))
        tol = float(kwargs.get("tol", 1e-6))
        seed = int(kwargs.get("seed", 0) or 0)
        from pyxu_amd.util import to_device

        x = np.random.default_rng(seed).standard_normal(self.dim).astype(pxrt.getPrecision().value)
        x = to_device(x / np.linalg.norm(x))  # host start vector (synthetic), uploaded once
        L_prev = 0.0
        with pxrt.EnforcePrecision(False):
            for _ in range(n_iter):
                y = self.adjoint(self.apply(x))
                n = float(_dev.row_reduce(_dev.RED_SUMSQ, y.reshape(1, -1)).cpu()[0]) ** 0.5
                if n == 0:
                    return 0.0
                L = n**0.5
                x = _dev.div(y, n)
                if abs(L - L_prev) <= tol * L:
                    break
                L_prev = L
        return float(L)

    def svdvals(self, k=1, which="LM", **kwargs):
        if k != 1 or which.upper() != "LM":
            raise NotImplementedError("pyxu_amd: only the largest singular value (k=1, 'LM') is available on device.")
        return np.array([self._power_lipschitz(**kwargs)], dtype=pxrt.getPrecision().value)

    def asarray(self, xp=None, dtype=None):
        """Matrix representation (device tensor unless xp is numpy), built column-block-wise."""
        import torch

        dtype = pxrt.getPrecision().value if dtype is None else np.dtype(dtype)
        tdt = pxrt.Width(np.dtype(dtype)).torch
        At = torch.empty((self.dim, self.codim), dtype=tdt, device="cuda")  # A^T, built row block by row block
        blk = 4096
        with pxrt.EnforcePrecision(False):
            for j0 in range(0, self.dim, blk):
                j1 = min(self.dim, j0 + blk)
                E = _dev.fill(torch.empty((j1 - j0, self.dim), dtype=tdt, device="cuda"), 0.0)
                _dev.set_diag(E, j1 - j0, self.dim, j0, 1.0)  # identity columns j0 .. j1 - 1
                Y = _dev.require(self.apply(E)).reshape(j1 - j0, self.codim)
                _dev.copy2d(Y, At, j1 - j0, self.codim, self.codim, self.codim, dst_off=j0 * self.codim)
        A = _dev.transpose(At)
        if xp is np:
            return A.cpu().numpy()
        return A

    def gram(self):
        from pyxu_amd.abc.arithmetic import _set_expr

        op = self.T * self
        _set_expr(op, ("gram", self))
        return op.asop(SelfAdjointOp).squeeze()

    def cogram(self):
        from pyxu_amd.abc.arithmetic import _set_expr

        op = self * self.T
        _set_expr(op, ("cogram", self))
        return op.asop(SelfAdjointOp).squeeze()

    @pxrt.enforce_precision(i=("arr", "damp"))
    def pinv(self, arr, damp, kwargs_init=None, kwargs_fit=None):
        from pyxu_amd.operator.linop import HomothetyOp
        from pyxu_amd.opt.solver import CG
        from pyxu_amd.opt.stop import MaxIter

        kwargs_fit = dict() if kwargs_fit is None else dict(kwargs_fit)
        kwargs_init = dict() if kwargs_init is None else dict(kwargs_init)
        kwargs_init.update(show_progress=kwargs_init.get("show_progress", False))
        A = self.gram() if np.isclose(damp, 0) else self.gram() + HomothetyOp(cst=damp, dim=self.dim)
        cg = CG(A, **kwargs_init)
        if "stop_crit" not in kwargs_fit:
            kwargs_fit["stop_crit"] = cg.default_stop_crit() | MaxIter(n=20 * A.dim)
        cg.fit(b=self.adjoint(arr), **kwargs_fit)
        return cg.solution()

    def dagger(self, damp, kwargs_init=None, kwargs_fit=None):
        from pyxu_amd.operator.interop import from_source

        def op_apply(_, arr):
            return self.pinv(arr, damp=_._damp, kwargs_init=_._kwargs_init, kwargs_fit=_._kwargs_fit)

        def op_adjoint(_, arr):
            return self.T.pinv(arr, damp=_._damp, kwargs_init=_._kwargs_init, kwargs_fit=_._kwargs_fit)

        return from_source(
            cls=SquareOp if self.dim == self.codim else LinOp,
            shape=(self.dim, self.codim),
            embed=dict(_name="dagger", _damp=damp, _kwargs_init=copy.copy(kwargs_init or {}),
                       _kwargs_fit=copy.copy(kwargs_fit or {})),
            apply=op_apply,
            adjoint=op_adjoint,
            _expr=lambda _: (_._name, _, _._damp),
        )

    @classmethod
    def from_array(cls, A, enable_warnings: bool = True):
        """Dense LinOp from its matrix (operator.py:1790-1830 -> base.py _ExplicitLinOp)."""
        from pyxu_amd.operator.linop.base import _ExplicitLinOp

        return _ExplicitLinOp(cls, A, enable_warnings)


class SquareOp(LinOp):
    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR_SQUARE})

    def __init__(self, shape):
        super().__init__(shape=shape)
        assert self.dim == self.codim, f"shape: expected (M, M), got {self.shape}."

    @pxrt.enforce_precision()
    def trace(self, **kwargs):
        A = _dev.require(self.asarray())
        n = A.shape[0]
        d = _dev.empty((n,), A)
        _dev.copy2d(A, d, n, 1, n + 1, 1)  # the diagonal (stride n + 1)
        return float(_dev.row_reduce(_dev.RED_SUM, d.reshape(1, n)).cpu()[0])


class NormalOp(SquareOp):
    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR_NORMAL})

    def cogram(self):
        return self.gram()


class SelfAdjointOp(NormalOp):
    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR_SELF_ADJOINT})

    def adjoint(self, arr):
        return self.apply(arr)


class UnitOp(NormalOp):
    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR_UNITARY})

    def __init__(self, shape):
        super().__init__(shape=shape)
        self.lipschitz = 1

    def estimate_lipschitz(self, **kwargs):
        return 1

    @pxrt.enforce_precision(i=("arr", "damp"))
    def pinv(self, arr, damp, **kwargs):
        out = self.adjoint(arr)
        if not np.isclose(damp, 0):
            out = _dev.div(copy_if_unsafe(out), 1 + damp)
        return out

    def gram(self):
        from pyxu_amd.operator.linop import IdentityOp

        return IdentityOp(dim=self.dim).squeeze()


class ProjOp(SquareOp):
    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR_IDEMPOTENT})


class OrthProjOp(ProjOp, SelfAdjointOp):
    @classmethod
    def properties(cls):
        p = set()
        for klass in cls.__bases__:
            p |= klass.properties()
        return frozenset(p)

    def __init__(self, shape):
        super().__init__(shape=shape)
        self.lipschitz = 1

    def estimate_lipschitz(self, **kwargs):
        return 1

    def gram(self):
        return self.squeeze()

    def cogram(self):
        return self.squeeze()


class PosDefOp(SelfAdjointOp):
    @classmethod
    def properties(cls):
        return frozenset(set(super().properties()) | {Property.LINEAR_POSITIVE_DEFINITE})


class LinFunc(ProxDiffFunc, LinOp):
    """Linear functionals (operator.py:2044-2134)."""

    @classmethod
    def properties(cls):
        p = set()
        for klass in cls.__bases__:
            p |= klass.properties()
        return frozenset(p)

    def __init__(self, shape):
        super().__init__(shape=shape)

    def jacobian(self, arr):
        return LinOp.jacobian(self, arr)

    def estimate_lipschitz(self, **kwargs):
        import torch

        with pxrt.EnforcePrecision(False):
            g = self.grad(torch.ones((self.dim,), dtype=pxrt.getPrecision().torch, device="cuda"))
        return float(_dev.row_reduce(_dev.RED_SUMSQ, g.reshape(1, -1)).cpu()[0]) ** 0.5

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        x = _dev.fill(_dev.empty((*arr.shape[:-1], 1), arr), 1.0)
        return self.adjoint(x)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        out = copy_if_unsafe(self.grad(arr))
        return _dev.axpby(-tau, out, 1.0, arr, out=out)

    @pxrt.enforce_precision(i=("arr", "sigma"))
    def fenchel_prox(self, arr, sigma):
        return self.grad(arr)

    def cogram(self):
        from pyxu_amd.operator.linop import HomothetyOp

        L = self.lipschitz
        return HomothetyOp(cst=L**2, dim=1)

    def asarray(self, xp=None, dtype=None):
        import torch

        dtype = pxrt.getPrecision().value if dtype is None else np.dtype(dtype)
        with pxrt.EnforcePrecision(False):
            x = torch.ones((1, 1), dtype=pxrt.Width(np.dtype(dtype)).torch, device="cuda")
            A = self.adjoint(x)
        return A.cpu().numpy() if xp is np else A

    @classmethod
    def from_array(cls, A, enable_warnings: bool = True):
        if A.ndim == 1:
            A = A.reshape((1, -1))
        return super().from_array(A, enable_warnings)


def _core_operators():
    return {
        Map, Func, DiffMap, DiffFunc, ProxFunc, ProxDiffFunc, QuadraticFunc, LinOp, LinFunc, SquareOp, NormalOp,
        SelfAdjointOp, UnitOp, ProjOp, OrthProjOp, PosDefOp,
    }


warnings.filterwarnings("default", module="pyxu_amd")
