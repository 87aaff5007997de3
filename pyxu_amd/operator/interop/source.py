"""``from_source``: define operators from raw callables (reference operator/interop/source.py:15-262).

This is the reference's generic plugin entry point; the callables receive MI355X device tensors.
"""
import types

import pyxu_amd.abc.operator as pxo
import pyxu_amd.runtime as pxrt

__all__ = ["from_source"]

_EKWARGS = dict(
    apply=dict(i="arr"),
    prox=dict(i=("arr", "tau")),
    grad=dict(i="arr"),
    adjoint=dict(i="arr"),
    pinv=dict(i=("arr", "damp")),
    svdvals=dict(),
    trace=dict(),
)


def from_source(cls, shape, embed=None, vectorize=frozenset(), vmethod=None, enforce_precision=frozenset(), **kwargs):
    assert cls in pxo._core_operators(), f"Unknown Operator type: {cls}."
    op = cls(shape)
    meth = frozenset.union(*[p.arithmetic_methods() for p in pxo.Property])
    if not (set(kwargs) <= meth):
        unknown = ", ".join(f"{name}()" for name in set(kwargs) - meth)
        raise ValueError(f"Unknown arithmetic methods: {unknown}")
    if isinstance(enforce_precision, str):
        enforce_precision = frozenset([enforce_precision])
    if not (frozenset(enforce_precision) <= set(_EKWARGS)):
        raise ValueError("Can only enforce precision on arithmetic methods " + ", ".join(_EKWARGS))
    if vectorize:
        # stacking dimensions are native to every device kernel here; nothing to vectorize
        pass
    for p in op.properties():
        for name in p.arithmetic_methods():
            func = kwargs.get(name, False)
            if func:
                if name in enforce_precision:
                    func = pxrt.enforce_precision(**_EKWARGS[name])(func)
                setattr(op, name, types.MethodType(func, op))
    for name, attr in (embed or {}).items():
        setattr(op, name, attr)
    return op
