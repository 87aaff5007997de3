"""
Recognise ``A = s * K^T K + d * I`` (K one dense ``_ExplicitLinOp``) in an operator tree, so that CG
can evaluate ``A.apply(p)`` with ONE pass over K (``pxa_dense_normal``) instead of the rule-by-rule
K.apply -> scale -> K.adjoint -> AddRule chain (two passes over K plus element-wise launches).

This is the operator ADMM hands to CG for its x-update: ``QuadraticFunc.prox`` builds
``Q + HomothetyOp(1 / tau)`` (reference abc/operator.py:1273-1291) with ``Q = K.T * Q1 * K`` from
``ChainRule._quad_spec`` (reference abc/arithmetic.py:1255-1264) and ``Q1 = c * I`` from
``SquaredL2Norm._quad_spec`` scaled by the loss weight (reference operator/func/norm.py:111-112).

The walk reads only the structure the arithmetic rules record (the bound ``apply`` of each node and
its operands); it never evaluates anything.  A node it does not know ends the match (None), and the
caller keeps the generic ``A.apply``: results are the same operator, rounded in a different order.
"""
import pyxu_amd.abc.arithmetic as _ar

__all__ = ["normal_form", "normal_form_ex"]


def _mul(t1, t2):
    out = {}
    for c1, k1 in t1.items():
        for c2, k2 in t2.items():
            key = c1 + c2
            out[key] = out.get(key, 0.0) + k1 * k2
    return out


def _add(t1, t2):
    out = dict(t1)
    for c, k in t2.items():
        out[c] = out.get(c, 0.0) + k
    return out


def _terms(op, mats, depth):
    """op -> {chain: coefficient}: op = sum coef * (atom_0 o atom_1 o ...), atoms ('K', i) / ('KT', i)
    over the dense matrices collected in `mats`; None when a node is not a linear rule / known leaf."""
    if depth > 64:
        return None
    from pyxu_amd.operator.linop.base import IdentityOp

    f = getattr(op, "apply", None)
    fn = getattr(f, "__func__", None)
    node = getattr(f, "__self__", op)  # an asop() shell forwards to its core's bound methods
    if fn is _ar.ScaleRule.apply:
        t = _terms(node._op, mats, depth + 1)
        return None if t is None else {c: k * float(node._cst) for c, k in t.items()}
    if fn is _ar.AddRule.apply:
        if tuple(node._lhs.shape) != tuple(node._rhs.shape):
            return None  # range broadcasting: not a plain sum of square operators
        a, b = _terms(node._lhs, mats, depth + 1), _terms(node._rhs, mats, depth + 1)
        return None if a is None or b is None else _add(a, b)
    if fn is _ar.ChainRule.apply:
        a, b = _terms(node._lhs, mats, depth + 1), _terms(node._rhs, mats, depth + 1)
        return None if a is None or b is None else _mul(a, b)
    if fn is _ar.TransposeRule.apply:
        t = _terms(node._op, mats, depth + 1)
        if t is None:
            return None
        flip = {"K": "KT", "KT": "K"}
        return {tuple((flip[k], i) for k, i in reversed(c)): v for c, v in t.items()}
    if isinstance(node, IdentityOp):
        return {(): 1.0}
    name = getattr(node, "_name", None)
    if name == "HomothetyOp":
        return {(): float(node._cst)}
    group = None
    if name == "RowShardedLinOp" and getattr(node, "_local", None) is not None:
        # this rank's row block K_r of a row-sharded K (pyxu_amd.distributed): sum_r K_r^T K_r = K^T K
        group, node, name = getattr(node, "_group", None), node._local, "_ExplicitLinOp"
        sharded = True
    else:
        sharded = False
    if name == "_ExplicitLinOp" and getattr(node, "_mat", None) is not None:
        mat = node._mat
        for i, (m, _, _) in enumerate(mats):
            if m is mat:
                return {(("K", i),): 1.0}
        mats.append((mat, sharded, group))
        return {(("K", len(mats) - 1),): 1.0}
    return None


def normal_form_ex(op):
    """(K_matrix, s, d, sharded, group) with op = s * K^T K + d * I, or None.  sharded: K is this rank's
    row block of a row-sharded operator, and s * K^T K p is the all-reduce (sum over `group`) of the
    ranks' s * K_r^T K_r p."""
    mats = []
    try:
        t = _terms(op, mats, 0)
    except Exception:  # an unexpected node layout: no match, the generic path runs
        return None
    if t is None or len(mats) != 1:
        return None
    s = d = 0.0
    for chain, k in t.items():
        if chain == ():
            d += k
        elif chain == (("KT", 0), ("K", 0)):
            s += k
        elif k != 0.0:
            return None
    if s == 0.0:
        return None
    mat, sharded, group = mats[0]
    return mat, s, d, sharded, group


def normal_form(op):
    """(K_matrix, s, d) with op = s * K^T K + d * I for one (unsharded) dense K, or None."""
    r = normal_form_ex(op)
    if r is None or r[3]:
        return None
    return r[0], r[1], r[2]
