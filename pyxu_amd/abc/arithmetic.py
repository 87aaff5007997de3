"""
Operator algebra (mirrors reference ``pyxu.abc.arithmetic``, src/pyxu/abc/arithmetic.py).

Each Rule synthesises an instance of the inferred core class and binds its own arithmetic methods
on it (so ``isinstance`` / ``Property`` queries behave as in the reference); Lipschitz constants are
propagated forward with the same ``__rule`` protocol (arithmetic.py:28-41).  Array arithmetic runs
through ``pyxu_amd._dev`` on MI355X device tensors.
"""
import types

import numpy as np

import pyxu_amd.abc.operator as pxo
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.util import copy_if_unsafe, is_device_array

__all__ = ["Rule", "ScaleRule", "ArgScaleRule", "ArgShiftRule", "AddRule", "ChainRule", "PowerRule", "TransposeRule"]


def _set_expr(op, expr):
    op._expr = types.MethodType(lambda _: expr, op)


def _infer_sum_shape(sh1, sh2):
    A, B = sh1
    C, D = sh2
    if B != D:
        raise ValueError(f"Addition of {sh1} and {sh2} operators forbidden.")
    if A == C:
        return sh1
    if 1 in (A, C):
        return (max(A, C), B)
    raise ValueError(f"Addition of {sh1} and {sh2} operators forbidden.")


def _infer_composition_shape(sh1, sh2):
    A, B = sh1
    C, D = sh2
    if B == C:
        return (A, D)
    raise ValueError(f"Composition of {sh1} and {sh2} operators forbidden.")


def _quad_Q(op):
    """Q of ``op._quad_spec()`` without materialising (c, t): Lipschitz bookkeeping at construction
    time must not evaluate anything (the reference evaluates t = f(shift) eagerly, arithmetic.py:625)."""
    head = op._expr()[0] if op.has(pxo.Property.CAN_EVAL) else None
    if head == "scale":
        return ScaleRule(op=_quad_Q(op._op), cst=op._cst).op()
    if head == "argshift":
        return _quad_Q(op._op)
    if head == "compose" and op._rhs.has(pxo.Property.LINEAR) and op._lhs.has(pxo.Property.QUADRATIC):
        return (op._rhs.T * _quad_Q(op._lhs) * op._rhs).asop(pxo.PosDefOp)
    return op._quad_spec()[0]


def _memo_quad_spec(func):
    """(Q, c, t) of a rule-built quadratic, computed once per precision: the operator is immutable, and
    the reference's re-evaluation on every QuadraticFunc.prox call (abc/arithmetic.py ChainRule /
    ArgShiftRule._quad_spec) rebuilds the operators and reads t = f(shift) back from the device -- a
    host sync per ADMM x-update."""

    def memo(self):
        key = pxrt.getPrecision()
        cache = self.__dict__.setdefault("_quad_spec_memo", {})
        if key not in cache:
            cache[key] = func(self)
        return cache[key]

    memo.__wrapped__ = func
    return memo


def _chain_quadratic(op):
    """The QuadraticFunc of a composed quadratic ``q(K x)`` (ChainRule, lhs quadratic, rhs linear) whose prox
    the composition's prox evaluates: one per (memoised) spec, so that its per-instance caches (the constant
    c.grad, the CG sub-solver) survive across prox calls (ADMM calls this once per outer iteration)."""
    Q, c, t = op._quad_spec()
    qf = op.__dict__.get("_quad_prox_fn")
    if qf is None or qf[0] is not Q or qf[1] is not c or qf[2] is not t:
        qf = op._quad_prox_fn = (Q, c, t, pxo.QuadraticFunc(shape=op.shape, Q=Q, c=c, t=t))
    return qf[3]


def quadratic_prox_target(op):
    """The QuadraticFunc whose prox ``op.prox(arr, tau)`` evaluates (CG on Q + I / tau from b = arr / tau -
    c.grad), or None when op's prox takes another route.  Follows the dispatch of ChainRule.prox
    (arithmetic.py:1009-1030 of the reference) without evaluating anything."""
    P = pxo.Property
    if not (op.has(P.PROXIMABLE) and op.has(P.QUADRATIC)):
        return None
    bound = op.__dict__.get("prox")
    if bound is None:
        return op if isinstance(op, pxo.QuadraticFunc) and type(op).prox is pxo.QuadraticFunc.prox else None
    if getattr(bound, "__func__", None) is not ChainRule.prox:
        return None
    if op._lhs.has(P.PROXIMABLE) and op._rhs.has(P.LINEAR_UNITARY):
        return None
    if op._lhs.has(P.QUADRATIC) and op._rhs.has(P.LINEAR):
        return _chain_quadratic(op)
    return None


class Rule:
    def op(self):
        raise NotImplementedError

    def _bind(self, op):
        for p in op.properties():
            for name in p.arithmetic_methods():
                func = getattr(self.__class__, name, None)
                if func is not None:
                    if name == "_quad_spec":
                        func = _memo_quad_spec(func)
                    setattr(op, name, types.MethodType(func, op))

    @staticmethod
    def _propagate_constants(op):
        if op.has(pxo.Property.CAN_EVAL):
            op._lipschitz = op.estimate_lipschitz(__rule=True)
        if op.has(pxo.Property.DIFFERENTIABLE):
            op._diff_lipschitz = op.estimate_diff_lipschitz(__rule=True)

    def __call__(self, arr):
        return self.apply(arr)

    def svdvals(self, **kwargs):
        return self.__class__.svdvals(self, **kwargs)

    def pinv(self, arr, damp, **kwargs):
        return self.__class__.pinv(self, arr=arr, damp=damp, **kwargs)

    def trace(self, **kwargs):
        return self.__class__.trace(self, **kwargs)


# ============================================================================ ScaleRule
class ScaleRule(Rule):
    """``cst * op`` (arithmetic.py:65-258)."""

    def __init__(self, op, cst):
        self._op = op.squeeze()
        self._cst = float(cst)

    def op(self):
        if np.isclose(self._cst, 0):
            from pyxu_amd.operator.linop import NullOp

            return NullOp(shape=self._op.shape).squeeze()
        if np.isclose(self._cst, 1):
            return self._op
        klass = self._infer_op_klass()
        op = klass(shape=self._op.shape)
        op._op, op._cst = self._op, self._cst
        op._name = self._op._name
        self._bind(op)
        self._propagate_constants(op)
        return op

    def _infer_op_klass(self):
        P = pxo.Property
        preserved = {P.CAN_EVAL, P.FUNCTIONAL, P.DIFFERENTIABLE, P.DIFFERENTIABLE_FUNCTION, P.LINEAR, P.LINEAR_SQUARE,
                     P.LINEAR_NORMAL, P.LINEAR_SELF_ADJOINT}
        if self._cst > 0:
            preserved |= {P.LINEAR_POSITIVE_DEFINITE, P.QUADRATIC, P.PROXIMABLE}
        if self._op.has(P.LINEAR):
            preserved.add(P.PROXIMABLE)
        if np.isclose(self._cst, -1):
            preserved.add(P.LINEAR_UNITARY)
        return pxo.Operator._infer_operator_type(self._op.properties() & preserved)

    def _expr(self):
        return ("scale", self._op, self._cst)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        out = copy_if_unsafe(self._op.apply(arr))
        return _dev.axpby(self._cst, out, out=out)

    def estimate_lipschitz(self, **kwargs):
        L = float(self._op.lipschitz) if "__rule" in kwargs else self._op.estimate_lipschitz(**kwargs)
        return L * abs(self._cst)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        return self._op.prox(arr, tau * self._cst)

    def _quad_spec(self):
        Q1, c1, t1 = self._op._quad_spec()
        return (ScaleRule(op=Q1, cst=self._cst).op(), ScaleRule(op=c1, cst=self._cst).op(), t1 * self._cst)

    def jacobian(self, arr):
        if self.has(pxo.Property.LINEAR):
            return self
        return self._op.jacobian(arr) * self._cst

    def estimate_diff_lipschitz(self, **kwargs):
        dL = float(self._op.diff_lipschitz) if "__rule" in kwargs else self._op.estimate_diff_lipschitz(**kwargs)
        return dL * abs(self._cst)

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        out = copy_if_unsafe(self._op.grad(arr))
        return _dev.axpby(self._cst, out, out=out)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        out = copy_if_unsafe(self._op.adjoint(arr))
        return _dev.axpby(self._cst, out, out=out)

    def asarray(self, **kwargs):
        xp = kwargs.pop("xp", None)
        A = _dev.axpby(self._cst, _dev.require(self._op.asarray(**kwargs)))
        return A.cpu().numpy() if xp is np else A

    def svdvals(self, **kwargs):
        return self._op.svdvals(**kwargs) * abs(self._cst)

    @pxrt.enforce_precision(i=("arr", "damp"))
    def pinv(self, arr, damp, **kwargs):
        out = copy_if_unsafe(self._op.pinv(arr, damp=damp / (self._cst**2), **kwargs))
        return _dev.div(out, self._cst, out=out)

    def gram(self):
        return self._op.gram() * (self._cst**2)

    def cogram(self):
        return self._op.cogram() * (self._cst**2)

    def trace(self, **kwargs):
        return self._op.trace(**kwargs) * self._cst

    def asloss(self, data=None):
        if not self.has(pxo.Property.FUNCTIONAL):
            raise NotImplementedError
        return self if data is None else self._op.asloss(data) * self._cst


# ============================================================================ ArgScaleRule
class ArgScaleRule(Rule):
    """``op(cst * x)`` (arithmetic.py:261-476)."""

    def __init__(self, op, cst):
        self._op = op.squeeze()
        self._cst = float(cst)

    def op(self):
        if np.isclose(self._cst, 1):
            return self._op
        if np.isclose(self._cst, 0):
            raise NotImplementedError("pyxu_amd: argscale(0) (ConstantValued) is outside the hot-path scope.")
        P = pxo.Property
        preserved = {P.CAN_EVAL, P.FUNCTIONAL, P.PROXIMABLE, P.DIFFERENTIABLE, P.DIFFERENTIABLE_FUNCTION, P.LINEAR,
                     P.LINEAR_SQUARE, P.LINEAR_NORMAL, P.LINEAR_SELF_ADJOINT, P.QUADRATIC}
        if self._cst > 0:
            preserved.add(P.LINEAR_POSITIVE_DEFINITE)
        if np.isclose(self._cst, -1):
            preserved.add(P.LINEAR_UNITARY)
        klass = pxo.Operator._infer_operator_type(self._op.properties() & preserved)
        op = klass(shape=self._op.shape)
        op._op, op._cst = self._op, self._cst
        op._name = self._op._name
        self._bind(op)
        self._propagate_constants(op)
        return op

    def _expr(self):
        return ("argscale", self._op, self._cst)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._op.apply(_dev.axpby(self._cst, arr))

    def estimate_lipschitz(self, **kwargs):
        L = float(self._op.lipschitz) if "__rule" in kwargs else self._op.estimate_lipschitz(**kwargs)
        return L * abs(self._cst)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        x = _dev.axpby(self._cst, arr)
        y = self._op.prox(x, (self._cst**2) * tau)
        return _dev.div(copy_if_unsafe(y), self._cst)

    def jacobian(self, arr):
        if self.has(pxo.Property.LINEAR):
            return self
        return self._op.jacobian(_dev.axpby(self._cst, arr)) * self._cst

    def estimate_diff_lipschitz(self, **kwargs):
        dL = float(self._op.diff_lipschitz) if "__rule" in kwargs else self._op.estimate_diff_lipschitz(**kwargs)
        return dL * (self._cst**2)

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        out = copy_if_unsafe(self._op.grad(_dev.axpby(self._cst, arr)))
        return _dev.axpby(self._cst, out, out=out)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        out = copy_if_unsafe(self._op.adjoint(arr))
        return _dev.axpby(self._cst, out, out=out)

    def asarray(self, **kwargs):
        xp = kwargs.pop("xp", None)
        A = _dev.axpby(self._cst, _dev.require(self._op.asarray(**kwargs)))
        return A.cpu().numpy() if xp is np else A

    def gram(self):
        return self._op.gram() * (self._cst**2)

    def cogram(self):
        return self._op.cogram() * (self._cst**2)

    def trace(self, **kwargs):
        return self._op.trace(**kwargs) * self._cst

    def _quad_spec(self):
        Q1, c1, t1 = self._op._quad_spec()
        return (ScaleRule(op=Q1, cst=self._cst**2).op(), ScaleRule(op=c1, cst=self._cst).op(), t1)

    def asloss(self, data=None):
        raise NotImplementedError


# ============================================================================ ArgShiftRule
class ArgShiftRule(Rule):
    """``op(x + shift)`` (arithmetic.py:479-664)."""

    def __init__(self, op, cst):
        self._op = op.squeeze()
        self._scalar = isinstance(cst, (int, float, np.number))
        if self._scalar:
            cst = float(cst)
        else:
            if not (type(cst).__module__.startswith("torch") and hasattr(cst, "data_ptr")):
                raise TypeError("pyxu_amd: argshift() expects a scalar or an MI355X device array.")
            assert cst.numel() == len(cst), f"cst: expected 1D array, got {tuple(cst.shape)}."
        self._cst = cst

    def op(self):
        if self._scalar:
            norm = abs(self._cst)
        elif is_device_array(self._cst):
            norm = float(_dev.row_reduce(_dev.RED_SUMSQ, self._cst.reshape(1, -1)).cpu()[0])
        else:  # host tensor: construction-only use (no compute is possible on it); keep the shift
            norm = 1.0
        if np.isclose(float(norm), 0):
            return self._op
        P = pxo.Property
        preserved = {P.CAN_EVAL, P.FUNCTIONAL, P.PROXIMABLE, P.DIFFERENTIABLE, P.DIFFERENTIABLE_FUNCTION, P.QUADRATIC}
        klass = pxo.Operator._infer_operator_type(self._op.properties() & preserved)
        if self._scalar:
            shape = self._op.shape
        else:
            if self._op.dim not in (None, self._cst.numel()):
                raise ValueError(f"Shifting {self._op} by {tuple(self._cst.shape)} forbidden.")
            shape = (self._op.codim, self._cst.numel())
        op = klass(shape=shape)
        op._op, op._cst = self._op, self._cst
        op._name = self._op._name
        self._bind(op)
        self._propagate_constants(op)
        return op

    def _expr(self):
        return ("argshift", self._op, (None,) if isinstance(self._cst, float) else tuple(self._cst.shape))

    def _shift(self, arr):
        if isinstance(self._cst, float):
            return _dev.add_scalar(arr, self._cst)
        return _dev.axpby_bcast(1.0, arr, 1.0, pxrt.coerce(self._cst))

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._op.apply(ArgShiftRule._shift(self, arr))

    def estimate_lipschitz(self, **kwargs):
        return self._op.lipschitz if "__rule" in kwargs else self._op.estimate_lipschitz(**kwargs)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        out = copy_if_unsafe(self._op.prox(ArgShiftRule._shift(self, arr), tau))
        if isinstance(self._cst, float):
            return _dev.add_scalar(out, -self._cst, out=out)
        return _dev.axpby_bcast(1.0, out, -1.0, pxrt.coerce(self._cst), out=out)

    def _quad_spec(self):
        from pyxu_amd.operator.linop import Sum

        Q1, c1, t1 = self._op._quad_spec()
        if isinstance(self._cst, float):
            c2 = c1 + (self._cst * (Sum(arg_shape=(Q1.dim,)) * Q1))
            import torch

            cst = torch.full((Q1.dim,), self._cst, dtype=pxrt.getPrecision().torch, device="cuda")
            t2 = float(self._op.apply(cst).cpu()[0])
        else:
            c2 = c1 + pxo.LinFunc.from_array(Q1.apply(pxrt.coerce(self._cst)), enable_warnings=False)
            t2 = float(self._op.apply(pxrt.coerce(self._cst)).cpu()[0])
        return (Q1, c2, t2)

    def jacobian(self, arr):
        return self._op.jacobian(ArgShiftRule._shift(self, arr))

    def estimate_diff_lipschitz(self, **kwargs):
        return self._op.diff_lipschitz if "__rule" in kwargs else self._op.estimate_diff_lipschitz(**kwargs)

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        return self._op.grad(ArgShiftRule._shift(self, arr))

    def asloss(self, data=None):
        if self.has(pxo.Property.FUNCTIONAL):
            raise ArithmeticError("The meaning of op.argshift().asloss() is ambiguous.")
        raise NotImplementedError


# ============================================================================ AddRule
class AddRule(Rule):
    """``lhs + rhs`` (arithmetic.py:667-1031)."""

    def __init__(self, lhs, rhs):
        self._lhs = lhs.squeeze()
        self._rhs = rhs.squeeze()

    def op(self):
        sh = _infer_sum_shape(self._lhs.shape, self._rhs.shape)
        klass = self._infer_op_klass()
        P = pxo.Property
        if klass.has(P.QUADRATIC):
            lin = lambda _: _.has(P.LINEAR)
            quad = lambda _: _.has(P.QUADRATIC)
            if quad(self._lhs) and quad(self._rhs):
                lQ, lc, lt = self._lhs._quad_spec()
                rQ, rc, rt = self._rhs._quad_spec()
                op = klass(shape=sh, Q=lQ + rQ, c=lc + rc, t=lt + rt)
            elif quad(self._lhs) and lin(self._rhs):
                lQ, lc, lt = self._lhs._quad_spec()
                op = klass(shape=sh, Q=lQ, c=lc + self._rhs, t=lt)
            elif lin(self._lhs) and quad(self._rhs):
                rQ, rc, rt = self._rhs._quad_spec()
                op = klass(shape=sh, Q=rQ, c=self._lhs + rc, t=rt)
            else:
                raise ValueError("Impossible scenario: something went wrong during klass inference.")
            op._lhs, op._rhs = self._lhs, self._rhs
        else:
            op = klass(shape=sh)
            op._lhs, op._rhs = self._lhs, self._rhs
            self._bind(op)
            self._propagate_constants(op)
        return op

    def _expr(self):
        return ("add", self._lhs, self._rhs)

    def _infer_op_klass(self):
        P = pxo.Property
        lhs_p, rhs_p = self._lhs.properties(), self._rhs.properties()
        base = set(lhs_p & rhs_p)
        for p in (P.LINEAR_NORMAL, P.LINEAR_UNITARY, P.LINEAR_IDEMPOTENT, P.PROXIMABLE):
            base.discard(p)
        if P.LINEAR_SELF_ADJOINT in base:
            base.add(P.LINEAR_NORMAL)
        if (({P.LINEAR_IDEMPOTENT, P.LINEAR_SELF_ADJOINT} < lhs_p) and (P.LINEAR_POSITIVE_DEFINITE in rhs_p)) or (
            ({P.LINEAR_IDEMPOTENT, P.LINEAR_SELF_ADJOINT} < rhs_p) and (P.LINEAR_POSITIVE_DEFINITE in lhs_p)
        ):
            base |= {P.LINEAR_SQUARE, P.LINEAR_NORMAL, P.LINEAR_SELF_ADJOINT, P.LINEAR_POSITIVE_DEFINITE}
        if P.LINEAR in base:
            sh = _infer_sum_shape(self._lhs.shape, self._rhs.shape)
            if (sh[0] == sh[1]) and (sh[0] > 1):
                base.add(P.LINEAR_SQUARE)
        if P.QUADRATIC in base:
            base.add(P.PROXIMABLE)
        if (P.PROXIMABLE in (lhs_p & rhs_p)) and ({P.QUADRATIC, P.LINEAR} < (lhs_p | rhs_p)):
            base.add(P.QUADRATIC)
        if (P.PROXIMABLE in (lhs_p & rhs_p)) and (P.LINEAR in (lhs_p | rhs_p)):
            base.add(P.PROXIMABLE)
        return pxo.Operator._infer_operator_type(base)

    @staticmethod
    def _add(a, b):
        """a + b with range broadcasting of a (..., 1) operand."""
        if a.shape == b.shape:
            return _dev.axpby(1.0, a, 1.0, b)
        if a.shape[-1] == 1:
            a, b = b, a
        # b is (..., 1): broadcast along the last axis
        import torch

        return _dev.axpby(1.0, a, 1.0, b.expand_as(a).contiguous())

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return AddRule._add(self._lhs.apply(arr), self._rhs.apply(arr))

    def estimate_lipschitz(self, **kwargs):
        if "__rule" in kwargs:
            L_lhs, L_rhs = self._lhs.lipschitz, self._rhs.lipschitz
        elif self.has(pxo.Property.LINEAR):
            return self.__class__.estimate_lipschitz(self, **kwargs)
        else:
            L_lhs, L_rhs = self._lhs.estimate_lipschitz(**kwargs), self._rhs.estimate_lipschitz(**kwargs)
        if self._lhs.codim < self._rhs.codim:
            L_lhs = L_lhs * np.sqrt(self._rhs.codim)
        elif self._lhs.codim > self._rhs.codim:
            L_rhs = L_rhs * np.sqrt(self._lhs.codim)
        return L_lhs + L_rhs

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        P_L, P_R = self._lhs.properties(), self._rhs.properties()
        if pxo.Property.LINEAR in (P_L | P_R):
            P, G = (self._rhs, self._lhs) if pxo.Property.LINEAR in P_L else (self._lhs, self._rhs)
            x = copy_if_unsafe(G.grad(arr))
            x = _dev.axpby(-tau, x, 1.0, arr, out=x)
            return P.prox(x, tau)
        raise NotImplementedError

    def jacobian(self, arr):
        if self.has(pxo.Property.LINEAR):
            return self
        return self._lhs.jacobian(arr) + self._rhs.jacobian(arr)

    def estimate_diff_lipschitz(self, **kwargs):
        if "__rule" in kwargs:
            dL_lhs, dL_rhs = self._lhs.diff_lipschitz, self._rhs.diff_lipschitz
        elif self.has(pxo.Property.LINEAR):
            dL_lhs = dL_rhs = 0
        else:
            dL_lhs, dL_rhs = self._lhs.estimate_diff_lipschitz(**kwargs), self._rhs.estimate_diff_lipschitz(**kwargs)
        if self._lhs.codim < self._rhs.codim:
            dL_lhs = dL_lhs * np.sqrt(self._rhs.codim)
        elif self._lhs.codim > self._rhs.codim:
            dL_rhs = dL_rhs * np.sqrt(self._lhs.codim)
        return dL_lhs + dL_rhs

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        out = copy_if_unsafe(self._lhs.grad(arr))
        return _dev.axpby(1.0, out, 1.0, self._rhs.grad(arr), out=out)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        from pyxu_amd.abc.operator import _rowsum

        arr_l = arr_r = arr
        if self._lhs.codim < self._rhs.codim:
            arr_l = _rowsum(arr)
        elif self._lhs.codim > self._rhs.codim:
            arr_r = _rowsum(arr)
        out = copy_if_unsafe(self._lhs.adjoint(arr_l))
        return _dev.axpby(1.0, out, 1.0, self._rhs.adjoint(arr_r), out=out)

    def asarray(self, **kwargs):
        xp = kwargs.pop("xp", None)
        L = _dev.require(self._lhs.asarray(**kwargs))
        Rm = _dev.require(self._rhs.asarray(**kwargs))
        if L.shape != Rm.shape:  # (1, N) + (M, N) range broadcasting (arithmetic.py:843-849)
            big, small = (L, Rm) if L.numel() >= Rm.numel() else (Rm, L)
            A = _dev.axpby_bcast(1.0, big, 1.0, small)
        else:
            A = _dev.axpby(1.0, L, 1.0, Rm)
        return A.cpu().numpy() if xp is np else A

    def gram(self):
        op = self._lhs.gram() + self._rhs.gram() + (self._lhs.T * self._rhs + self._rhs.T * self._lhs).asop(pxo.SelfAdjointOp)
        return op.squeeze()

    def cogram(self):
        op = self._lhs.cogram() + self._rhs.cogram() + (self._lhs * self._rhs.T + self._rhs * self._lhs.T).asop(pxo.SelfAdjointOp)
        return op.squeeze()

    def trace(self, **kwargs):
        return self._lhs.trace(**kwargs) + self._rhs.trace(**kwargs)

    def asloss(self, data=None):
        if data is None:
            return self
        return self._lhs.asloss(data) + self._rhs.asloss(data)


# ============================================================================ ChainRule
class ChainRule(Rule):
    """``lhs o rhs`` (arithmetic.py:1034-1344)."""

    def __init__(self, lhs, rhs):
        self._lhs = lhs.squeeze()
        self._rhs = rhs.squeeze()

    def op(self):
        sh = _infer_composition_shape(self._lhs.shape, self._rhs.shape)
        klass = self._infer_op_klass()
        op = klass(shape=sh)
        op._lhs, op._rhs = self._lhs, self._rhs
        op._name = "compose"
        self._bind(op)
        self._propagate_constants(op)
        return op

    def _expr(self):
        return ("compose", self._lhs, self._rhs)

    def _infer_op_klass(self):
        P = pxo.Property
        lhs_p, rhs_p = self._lhs.properties(), self._rhs.properties()
        props = {P.CAN_EVAL}
        if P.FUNCTIONAL in lhs_p:
            props.add(P.FUNCTIONAL)
        if (P.PROXIMABLE in lhs_p) and (P.LINEAR_UNITARY in rhs_p):
            props.add(P.PROXIMABLE)
        elif ({P.LINEAR, P.FUNCTIONAL} < lhs_p) and (P.PROXIMABLE in rhs_p):
            if self._lhs_scalar() > 0:
                props.add(P.PROXIMABLE)
                if P.QUADRATIC in rhs_p:
                    props.add(P.QUADRATIC)
        if P.DIFFERENTIABLE in (lhs_p & rhs_p):
            props.add(P.DIFFERENTIABLE)
        if (P.DIFFERENTIABLE_FUNCTION in lhs_p) and (P.DIFFERENTIABLE in rhs_p):
            props.add(P.DIFFERENTIABLE_FUNCTION)
        if (P.QUADRATIC in lhs_p) and (P.LINEAR in rhs_p):
            props |= {P.PROXIMABLE, P.QUADRATIC}
        if P.LINEAR in (lhs_p & rhs_p):
            props.add(P.LINEAR)
            if self._lhs.codim == 1:
                props.add(P.PROXIMABLE)
            if self._lhs.codim == self._rhs.dim > 1:
                props.add(P.LINEAR_SQUARE)
        if P.LINEAR_UNITARY in (lhs_p & rhs_p):
            props |= {P.LINEAR_NORMAL, P.LINEAR_UNITARY}
        return pxo.Operator._infer_operator_type(props)

    def _lhs_scalar(self):
        A = self._lhs.asarray()
        return float(A.reshape(-1)[0].cpu()) if not isinstance(A, np.ndarray) else float(A.reshape(-1)[0])

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._lhs.apply(self._rhs.apply(arr))

    def estimate_lipschitz(self, **kwargs):
        if "__rule" in kwargs:
            return self._lhs.lipschitz * self._rhs.lipschitz
        if self.has(pxo.Property.LINEAR):
            return self.__class__.estimate_lipschitz(self, **kwargs)
        return self._lhs.estimate_lipschitz(**kwargs) * self._rhs.estimate_lipschitz(**kwargs)

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        P = pxo.Property
        if self.has(P.PROXIMABLE):
            if self._lhs.has(P.PROXIMABLE) and self._rhs.has(P.LINEAR_UNITARY):
                return self._rhs.adjoint(self._lhs.prox(self._rhs.apply(arr), tau))
            if self._lhs.has(P.QUADRATIC) and self._rhs.has(P.LINEAR):
                return _chain_quadratic(self).prox(arr, tau)
            if self._lhs.has(P.LINEAR) and self._rhs.has(P.PROXIMABLE):
                return ScaleRule(op=self._rhs, cst=self._lhs_scalar()).op().prox(arr, tau)
            if P.LINEAR in (self._lhs.properties() & self._rhs.properties()):
                return pxo.LinFunc.prox(self, arr, tau)
        raise NotImplementedError

    def _quad_spec(self):
        P = pxo.Property
        if not self.has(P.QUADRATIC):
            raise NotImplementedError
        if self._lhs.has(P.LINEAR):
            return ScaleRule(op=self._rhs, cst=self._lhs_scalar()).op()._quad_spec()
        Q1, c1, t1 = self._lhs._quad_spec()
        Q2 = (self._rhs.T * Q1 * self._rhs).asop(pxo.PosDefOp)
        c2 = c1 * self._rhs
        return (Q2, c2, t1)

    def jacobian(self, arr):
        if self.has(pxo.Property.LINEAR):
            return self
        return self._lhs.jacobian(self._rhs.apply(arr)) * self._rhs.jacobian(arr)

    def estimate_diff_lipschitz(self, **kwargs):
        P = pxo.Property
        no_eval = "__rule" in kwargs
        if self.has(P.QUADRATIC):
            if no_eval:
                # reference: a freshly built QuadraticFunc(Q, c, t) reports diff_lipschitz = inf until set
                # (arithmetic.py:1266-1273)
                return np.inf
            return _quad_Q(self).estimate_lipschitz(**kwargs)
        if self._lhs.has(P.LINEAR) and self._rhs.has(P.LINEAR):
            return 0
        if self._lhs.has(P.LINEAR) and self._rhs.has(P.DIFFERENTIABLE):
            if no_eval:
                return self._lhs.lipschitz * self._rhs.diff_lipschitz
            return self._lhs.estimate_lipschitz(**kwargs) * self._rhs.estimate_diff_lipschitz(**kwargs)
        if self._lhs.has(P.DIFFERENTIABLE) and self._rhs.has(P.LINEAR):
            if no_eval:
                return self._lhs.diff_lipschitz * (self._rhs.lipschitz**2)
            return self._lhs.estimate_diff_lipschitz(**kwargs) * (self._rhs.estimate_lipschitz(**kwargs) ** 2)
        return np.inf

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        P = pxo.Property
        if {P.LINEAR, P.FUNCTIONAL} <= self._lhs.properties() and self._rhs.has(P.LINEAR):
            # a linear functional's gradient does not depend on where it is taken: skip rhs.apply(arr)
            # (the reference evaluates it and discards it; for ADMM's c o K that is a full pass over K
            # per QuadraticFunc.prox call; reference arithmetic.py:1288-1291)
            y = _dev.zeros((*arr.shape[:-1], self._rhs.codim), arr)
            return self._rhs.adjoint(self._lhs.grad(y))
        x = self._lhs.grad(self._rhs.apply(arr))
        if arr.ndim == 1 or self._rhs.has(pxo.Property.LINEAR):
            return self._rhs.jacobian(arr).adjoint(x)
        a2 = arr.reshape(-1, arr.shape[-1])
        x2 = x.reshape(a2.shape[0], -1)
        out = _dev.empty(a2.shape, a2)
        for r, (a, b) in enumerate(zip(a2, x2)):  # per-row Jacobians (non-linear rhs), rows written in place
            g = _dev.require(self._rhs.jacobian(a).adjoint(b))
            _dev.copy2d(g, out, 1, g.numel(), g.numel(), g.numel(), dst_off=r * a2.shape[1])
        return out.reshape(arr.shape)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        return self._rhs.adjoint(self._lhs.adjoint(arr))

    def asarray(self, **kwargs):
        xp = kwargs.pop("xp", None)
        L = _dev.require(self._lhs.asarray(**kwargs))
        Rm = _dev.require(self._rhs.asarray(**kwargs))
        A = _dev.dense_matmat(Rm, L, 1)  # rows of L times R (pxa_dense_matmat, trans = 1)
        return A.cpu().numpy() if xp is np else A

    def gram(self):
        return (self._rhs.T * self._lhs.gram() * self._rhs).asop(pxo.SelfAdjointOp).squeeze()

    def cogram(self):
        return (self._lhs * self._rhs.cogram() * self._lhs.T).asop(pxo.SelfAdjointOp).squeeze()

    def asloss(self, data=None):
        if self.has(pxo.Property.FUNCTIONAL):
            raise ArithmeticError("The meaning of (lhs * rhs).asloss() is ambiguous.")
        raise NotImplementedError


# ============================================================================ PowerRule
class PowerRule(Rule):
    """``op ** k`` (arithmetic.py:1347-1384)."""

    def __init__(self, op, k):
        assert op.codim == op.dim, f"PowerRule: expected endomorphism, got {op}."
        assert int(k) >= 0
        self._op = op.squeeze()
        self._k = int(k)

    def op(self):
        if self._k == 0:
            from pyxu_amd.operator.linop import IdentityOp

            return IdentityOp(dim=self._op.codim)
        op = self._op
        if pxo.Property.LINEAR_IDEMPOTENT not in self._op.properties():
            for _ in range(self._k - 1):
                op = ChainRule(self._op, op).op()
            _set_expr(op, ("exp", self._op, self._k))
        return op


# ============================================================================ TransposeRule
class TransposeRule(Rule):
    """``op.T`` (arithmetic.py:1387-1506)."""

    def __init__(self, op):
        self._op = op

    def op(self):
        klass = self._infer_op_klass()
        op = klass(shape=(self._op.dim, self._op.codim))
        op._op = self._op
        op._name = f"{self._op._name}.T"
        self._bind(op)
        self._propagate_constants(op)
        return op

    def _expr(self):
        return ("transpose", self._op)

    def _infer_op_klass(self):
        props = self._op.properties()
        if self._op.codim == self._op.dim == 1:
            return pxo.LinFunc
        if pxo.Property.FUNCTIONAL in props:
            return pxo.LinOp
        if self._op.dim == 1:
            return pxo.LinFunc
        return pxo.Operator._infer_operator_type(props)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._op.adjoint(arr)

    def estimate_lipschitz(self, **kwargs):
        return self._op.lipschitz if "__rule" in kwargs else self._op.estimate_lipschitz(**kwargs)

    def asloss(self, data=None):
        raise NotImplementedError

    @pxrt.enforce_precision(i=("arr", "tau"))
    def prox(self, arr, tau):
        return pxo.LinFunc.prox(self, arr, tau)

    def jacobian(self, arr):
        return self

    def estimate_diff_lipschitz(self, **kwargs):
        return 0

    @pxrt.enforce_precision(i="arr")
    def grad(self, arr):
        return pxo.LinFunc.grad(self, arr)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        return self._op.apply(arr)

    def asarray(self, **kwargs):
        xp = kwargs.pop("xp", None)
        A = _dev.transpose(_dev.require(self._op.asarray(**kwargs)))
        return A.cpu().numpy() if xp is np else A

    def gram(self):
        return self._op.cogram()

    def cogram(self):
        return self._op.gram()

    def svdvals(self, **kwargs):
        return self._op.svdvals(**kwargs)

    def trace(self, **kwargs):
        return self._op.trace(**kwargs)
