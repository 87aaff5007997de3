"""NumPy restatement of `numba.stencil` (constant mode) + identity JIT decorators.

Only what the reference's generated stencil source (`_stencil.py:232-261`) touches.
"""
import sys
import types

import numpy as np


class _OffsetRecorder:
    def __init__(self):
        self.offsets = []

    def __getitem__(self, idx):
        self.offsets.append(tuple(int(i) for i in idx))
        return 0.0


class _ShiftedView:
    def __init__(self, arr, lo, hi):
        self._arr, self._lo, self._hi = arr, lo, hi

    def __getitem__(self, idx):
        sl = tuple(
            slice(l + o, n - h + o)
            for (o, l, h, n) in zip(idx, self._lo, self._hi, self._arr.shape)
        )
        return self._arr[sl]


def stencil(func_or_mode="constant", cval=0, **kwargs):
    assert func_or_mode == "constant"

    def decorate(kernel):
        def run(a, out):
            rec = _OffsetRecorder()
            kernel(rec)
            offs = np.array(rec.offsets, dtype=int).reshape(-1, a.ndim)
            lo = np.maximum(0, -offs.min(axis=0))
            hi = np.maximum(0, offs.max(axis=0))
            out[...] = cval
            core = tuple(slice(l, n - h) for (l, h, n) in zip(lo, hi, a.shape))
            if all(c.start < c.stop for c in core):
                out[core] = kernel(_ShiftedView(a, lo, hi))
            return out

        return run

    return decorate


def jit(*args, **kwargs):
    if args and callable(args[0]):
        return args[0]
    return lambda f: f


njit = jit
prange = range

cuda = types.ModuleType("numba.cuda")
cuda.jit = jit
cuda.grid = lambda n: 0
sys.modules["numba.cuda"] = cuda

core = types.ModuleType("numba.core")
errors = types.ModuleType("numba.core.errors")


class NumbaPerformanceWarning(Warning):
    pass


errors.NumbaPerformanceWarning = NumbaPerformanceWarning
core.errors = errors
sys.modules["numba.core"] = core
sys.modules["numba.core.errors"] = errors
