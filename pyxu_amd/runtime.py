"""
Runtime floating-point precision state (mirrors reference ``pyxu.runtime``,
src/pyxu/runtime/_runtime.py:25-263): ``Width``, ``Precision``, ``EnforcePrecision``,
``enforce_precision``, ``coerce``, ``getPrecision``.

Default precision is DOUBLE, like the reference.  Device arrays are torch-ROCm tensors; numpy
arrays and Python scalars are coerced with numpy semantics.
"""
import contextlib
import enum
import functools
import inspect
import numbers

import numpy as np

__all__ = [
    "Width",
    "CWidth",
    "Precision",
    "EnforcePrecision",
    "enforce_precision",
    "coerce",
    "getPrecision",
    "getCoerceState",
]


@enum.unique
class Width(enum.Enum):
    """Machine-dependent floating-point types (_runtime.py:25-44)."""

    SINGLE = np.dtype(np.single)
    DOUBLE = np.dtype(np.double)

    def eps(self) -> float:
        return float(np.finfo(self.value).eps)

    @property
    def complex(self) -> "CWidth":
        return CWidth[self.name]

    @property
    def torch(self):
        import torch

        return {Width.SINGLE: torch.float32, Width.DOUBLE: torch.float64}[self]


@enum.unique
class CWidth(enum.Enum):
    SINGLE = np.dtype(np.csingle)
    DOUBLE = np.dtype(np.cdouble)

    @property
    def real(self) -> Width:
        return Width[self.name]


_state = {"width": Width.DOUBLE, "coerce": True}


def getPrecision() -> Width:
    return _state["width"]


def getCoerceState() -> bool:
    return _state["coerce"]


class Precision(contextlib.AbstractContextManager):
    """Locally redefine the runtime FP precision (_runtime.py:67-99)."""

    def __init__(self, width: Width):
        self._width = Width(width)
        self._prev = None

    def __enter__(self):
        self._prev = _state["width"]
        _state["width"] = self._width
        return self

    def __exit__(self, *exc):
        _state["width"] = self._prev
        return False


class EnforcePrecision(contextlib.AbstractContextManager):
    """Locally disable :py:func:`enforce_precision` (_runtime.py:102-136)."""

    def __init__(self, state: bool):
        self._s = bool(state)
        self._prev = None

    def __enter__(self):
        self._prev = _state["coerce"]
        _state["coerce"] = self._s
        return self

    def __exit__(self, *exc):
        _state["coerce"] = self._prev
        return False


def _is_tensor(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def _torch_float_types():
    import torch

    return (torch.float32, torch.float64)


def _carrier(tdt, device):
    import torch

    return torch.empty((1,), dtype=tdt, device=device)


def coerce(x):
    """Cast a scalar / NDArray to the runtime precision (_runtime.py:213-245).

    Complex or otherwise unsafe casts raise TypeError, as in the reference.
    """
    if not _state["coerce"]:
        return x
    width = _state["width"]
    t = type(x)
    if t is float or t is int:  # (the common case, without the ABC instance checks below: same value)
        return np.dtype(width.value).type(x)
    if isinstance(x, (numbers.Real, np.number)) and not isinstance(x, (np.complexfloating, complex)):
        return np.array(x, dtype=width.value)[()]
    if _is_tensor(x):
        if x.is_complex():
            raise TypeError(f"Cannot coerce {x.dtype} tensor to precision {width.value}.")
        tdt = width.torch
        if x.dtype == tdt:
            return x
        if x.is_cuda and x.dtype in (_torch_float_types()):
            from pyxu_amd import _dev

            return _dev.cast(x, _carrier(tdt, x.device))  # HIP cast kernel
        return x.to(tdt)  # host tensors (construction-time data, e.g. a shift vector before upload)
    try:
        dt = x.dtype
    except AttributeError:
        raise TypeError(f"Cannot coerce {type(x)} to scalar/array of precision {width.value}.")
    if np.can_cast(dt, width.value, casting="same_kind"):
        return x.astype(width.value, copy=False)
    raise TypeError(f"Cannot coerce {type(x)} to scalar/array of precision {width.value}.")


def enforce_precision(i=frozenset(), o: bool = True, allow_None: bool = True):
    """Decorator coercing parameters `i` (and the output if `o`) to the runtime precision
    (_runtime.py:139-200).

    The parameter lookup is resolved once at decoration time (positional index + name), so the
    per-call cost is a few tuple operations instead of a signature bind.
    """
    names = (i,) if isinstance(i, str) else tuple(i)

    def decorator(func):
        sig = inspect.signature(func)
        params = list(sig.parameters)
        for k in names:
            if k not in params:
                raise ValueError(f"Parameter[{k}] not part of {func.__qualname__}() parameter list.")
        pos = {k: params.index(k) for k in names}

        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            if _state["coerce"] and names:
                args = list(args)
                for k, p in pos.items():
                    if p < len(args):
                        v = args[p]
                        if v is None:
                            if not allow_None:
                                raise ValueError(f"Parameter[{k}] cannot be None-valued.")
                        else:
                            args[p] = coerce(v)
                    elif k in kwargs:
                        v = kwargs[k]
                        if v is None:
                            if not allow_None:
                                raise ValueError(f"Parameter[{k}] cannot be None-valued.")
                        else:
                            kwargs[k] = coerce(v)
            out = func(*args, **kwargs)
            if o and out is not None and _state["coerce"]:
                out = coerce(out)
            return out

        return wrapper

    return decorator
