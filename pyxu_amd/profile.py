"""Tracing hooks around the solver iteration (the reference has none).

* ``PXA_PROFILE=1``: every ``m_step`` runs inside a roctx range named ``<Solver>.m_step[<k>]`` (and every
  ``fit`` inside ``<Solver>.fit``), so a ``rocprofv3 --marker-trace --kernel-trace`` timeline groups each
  iteration's kernels under its step.  roctx is ``libroctx64.so`` from ``/opt/rocm/lib``; without it the flag
  raises at the first instrumented call rather than silently doing nothing.
* ``PXA_DEBUG_SYNC=1``: after every ``m_step`` the device is synchronised and checked -- an asynchronous HIP
  error (a faulting kernel) is raised from inside the step that launched it, where ``Solver._step`` catches
  and logs it like any other failure (``solver.py:653-663``), instead of surfacing steps later.

Both are read once, when a solver's ``fit`` starts; neither changes any result.
"""
import ctypes as ct
import os

__all__ = ["enabled", "debug_sync", "instrument", "range_push", "range_pop"]

_ROCTX = None


def enabled() -> bool:
    return os.environ.get("PXA_PROFILE", "0") not in ("", "0")


def debug_sync() -> bool:
    return os.environ.get("PXA_DEBUG_SYNC", "0") not in ("", "0")


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        last = None
        for name in ("libroctx64.so", "libroctx64.so.4", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"),
                                                                      "lib", "libroctx64.so")):
            try:
                lib = ct.CDLL(name)
                break
            except OSError as e:
                last = e
        else:
            raise RuntimeError(f"PXA_PROFILE is set but libroctx64.so cannot be loaded: {last}")
        lib.roctxRangePushA.argtypes = [ct.c_char_p]
        lib.roctxRangePushA.restype = ct.c_int
        lib.roctxRangePop.argtypes = []
        lib.roctxRangePop.restype = ct.c_int
        _ROCTX = lib
    return _ROCTX


def range_push(name: str) -> None:
    _roctx().roctxRangePushA(name.encode())


def range_pop() -> None:
    _roctx().roctxRangePop()


def _check_device():
    import torch

    torch.cuda.synchronize()  # raises the pending asynchronous error of any kernel launched so far


def instrument(solver) -> None:
    """Wrap ``solver.m_step`` (instance attribute) for the flags above; a no-op when neither is set.
    Idempotent: a solver fitted twice is wrapped once."""
    prof, dbg = enabled(), debug_sync()
    if not (prof or dbg):
        saved = solver.__dict__.pop("_pxa_m_step_orig", None)
        if saved is not None:  # flags cleared since the last fit: restore what m_step was before wrapping
            orig, was_instance_attr = saved
            if was_instance_attr:
                solver.m_step = orig  # an instance-level override the solver had of its own
            else:
                solver.__dict__.pop("m_step", None)  # the class method again
        return
    saved = solver.__dict__.get("_pxa_m_step_orig")
    if saved is None:
        saved = (solver.m_step, "m_step" in solver.__dict__)
        solver._pxa_m_step_orig = saved
    orig = saved[0]
    name = type(solver).__name__

    def m_step():
        if prof:
            range_push(f"{name}.m_step[{solver._astate.get('idx', 0)}]")
        try:
            orig()
            if dbg:
                _check_device()
        finally:
            if prof:
                range_pop()

    solver.m_step = m_step
