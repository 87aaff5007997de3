"""
Stopping criteria (mirrors reference ``pyxu.opt.stop``, src/pyxu/opt/stop.py).

Norms are evaluated on the device (``pxa_row_reduce``, double accumulation) and only the per-row
scalars cross to the host — the single device->host sync of a stop check (stop.py:381).
"""
import datetime as dt
import math
import numbers
import os

import numpy as np

import pyxu_amd.abc as pxa
from pyxu_amd import _dev

__all__ = ["MaxIter", "ManualStop", "MaxDuration", "Memorize", "AbsError", "RelError"]


_RED = {2: "RED_SUMSQ", 1: "RED_ABS", np.inf: "RED_MAXABS"}


def _rowstat(x, norm, y=None, out=None):
    """(..., N) device tensor(s) -> float64 DEVICE (rows,) row statistic of (x - y) for the Ln norm:
    sum of squares (2), sum of |.| (1) or max |.| (inf).  Stays on the device so that sharded
    criteria can all-reduce it before the single host sync (pyxu_amd.distributed)."""
    x2 = x.reshape(-1, x.shape[-1])
    if norm not in _RED:  # any other Ln, norm >= 0 (stop.py:258, numpy ord=p): sum |x - y|^p or nnz count
        y2 = y.reshape(-1, y.shape[-1]) if y is not None else None
        return _dev.row_reduce_pow(float(norm), x2, y2, out=out)
    if y is not None:
        y2 = y.reshape(-1, y.shape[-1])
        if norm == 2:
            return _dev.row_reduce(_dev.RED_DIFFSQ, x2, y2, out=out)
        x2 = _dev.axpby(1.0, x2, -1.0, y2)
    return _dev.row_reduce(getattr(_dev, _RED[norm]), x2, out=out)


def _finish(stat, norm):
    """host row statistic -> Ln norm (numpy.linalg.norm(ord=norm) semantics)."""
    if norm == 2:
        return stat**0.5
    if norm in (1, np.inf, 0):
        return stat
    return stat ** (1.0 / norm)


def _rownorm(x, norm, reduce=None):
    """(..., N) device tensor -> numpy (..., 1) Ln norm over the last axis."""
    st = _rowstat(x, norm)
    if reduce is not None:
        st = reduce(st, "max" if norm == np.inf else "sum")
    return _finish(st.cpu().numpy(), norm).reshape(*x.shape[:-1], 1)


def _identity(x):
    return x


def _as_vec(x):
    if isinstance(x, numbers.Real):
        return None
    return x


class MaxIter(pxa.StoppingCriterion):
    """Stop after `n` stop-checks (stop.py:29-68)."""

    def __init__(self, n):
        try:
            assert int(n) > 0
            self._n = int(n)
        except Exception:
            raise ValueError(f"n: expected positive integer, got {n}.")
        self._i = 0

    def stop(self, state) -> bool:
        self._i += 1
        return self._i > self._n

    def info(self):
        return dict(N_iter=self._i)

    def clear(self):
        self._i = 0


class ManualStop(pxa.StoppingCriterion):
    def stop(self, state) -> bool:
        return False

    def info(self):
        return dict()


class MaxDuration(pxa.StoppingCriterion):
    def __init__(self, t: dt.timedelta):
        try:
            assert t > dt.timedelta()
            self._t_max = t
        except Exception:
            raise ValueError(f"t: expected positive duration, got {t}.")
        self._t_start = dt.datetime.now()
        self._t_now = self._t_start

    def stop(self, state) -> bool:
        self._t_now = dt.datetime.now()
        return (self._t_now - self._t_start) > self._t_max

    def info(self):
        return dict(duration=(self._t_now - self._t_start).total_seconds())

    def clear(self):
        self._t_start = dt.datetime.now()
        self._t_now = self._t_start


class Memorize(pxa.StoppingCriterion):
    """Record min / max of a state variable (stop.py:181-210) without stalling the solver loop.

    For a device variable, stop() reduces it on the device (pxa_row_reduce MIN / MAX) and starts an
    asynchronous copy of the two doubles into pinned host memory; info() waits only for that copy
    (an event recorded before the solver enqueues its next m_step), so the host never blocks the
    device queue to log an objective value."""

    def __init__(self, var):
        self._var = var
        self._val = np.r_[0]
        self._pending = None  # (event, pinned (2,) float64, size)

    def stop(self, state) -> bool:
        x = state[self._var]
        if isinstance(x, numbers.Real):
            x = np.r_[x]
        if hasattr(x, "device") and getattr(x.device, "type", "cpu") != "cpu":
            import torch

            assert x.ndim == 1
            flat = x.reshape(1, -1)
            mm = torch.empty((2,), dtype=torch.float64, device=x.device)
            _dev.row_reduce(_dev.RED_MIN, flat, out=mm[0:1])
            _dev.row_reduce(_dev.RED_MAX, flat, out=mm[1:2])
            host = torch.empty((2,), dtype=torch.float64, pin_memory=True)
            host.copy_(mm, non_blocking=True)  # D2H into pinned memory (ordered on the stream)
            ev = torch.cuda.Event()
            _dev.record_event(ev)
            self._pending = (ev, host, x.numel(), mm)
            return False
        x = x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)
        assert x.ndim == 1
        self._pending = None
        self._val = x
        return False

    def _resolve(self):
        if self._pending is not None:
            ev, host, size, _ = self._pending
            ev.synchronize()
            mn, mx = float(host[0]), float(host[1])
            self._val = np.r_[mx] if size == 1 else np.r_[mn, mx]
            self._pending = None

    def info(self):
        self._resolve()
        if self._val.size == 1:
            return {f"Memorize[{self._var}]": float(self._val.max())}
        return {f"Memorize[{self._var}]_min": float(self._val.min()), f"Memorize[{self._var}]_max": float(self._val.max())}

    def clear(self):
        self._val = np.r_[0]
        self._pending = None


class AbsError(pxa.StoppingCriterion):
    """Stop when ||f(x)|| <= eps (stop.py:222-297)."""

    def __init__(self, eps, var="x", f=None, norm=2, satisfy_all=True):
        try:
            assert eps > 0
            self._eps = eps
        except Exception:
            raise ValueError(f"eps: expected positive threshold, got {eps}.")
        self._var = var
        self._f = f if (f is not None) else _identity
        try:
            assert norm >= 0
            self._norm = norm
        except Exception:
            raise ValueError(f"norm: expected non-negative, got {norm}.")
        self._satisfy_all = satisfy_all
        self._val = np.r_[0]

    def stop(self, state) -> bool:
        x = state[self._var]
        # a row statistic the solver step already computed for this very array (CG publishes
        # ||r||^2 of its residual: the same pxa_row_reduce, hence the same bits) saves a reduction and
        # a host sync on the whole device queue
        pre = state.get("__rowstat__", {}).get(self._var) if hasattr(state, "get") else None
        if pre is not None and pre[0] is x and pre[1] == self._norm and self._f is _identity and self._reduce is None:
            st = np.asarray(pre[2].host(), dtype=np.float64)
            self._val = _finish(st, self._norm).reshape(*x.shape[:-1], 1)
        else:
            fx = self._f(x)
            if isinstance(fx, numbers.Real):
                self._val = np.abs(np.r_[fx])
            else:
                self._val = _rownorm(fx, self._norm, reduce=self._reduce)
        rule = np.all if self._satisfy_all else np.any
        return bool(rule(self._val <= self._eps))

    # hook: combine a device row statistic across shards (identity on one process)
    _reduce = None

    def info(self):
        if self._val.size == 1:
            return {f"AbsError[{self._var}]": float(self._val.max())}
        return {f"AbsError[{self._var}]_min": float(self._val.min()), f"AbsError[{self._var}]_max": float(self._val.max())}

    def clear(self):
        self._val = np.r_[0]


class RelError(pxa.StoppingCriterion):
    """Stop when ||f(x) - f(x_prev)|| <= eps ||f(x_prev)|| (stop.py:300-396)."""

    def __init__(self, eps, var="x", f=None, norm=2, satisfy_all=True):
        try:
            assert eps > 0
            self._eps = eps
        except Exception:
            raise ValueError(f"eps: expected positive threshold, got {eps}.")
        self._var = var
        self._f = f if (f is not None) else _identity
        try:
            assert norm >= 0
            self._norm = norm
        except Exception:
            raise ValueError(f"norm: expected non-negative, got {norm}.")
        self._satisfy_all = satisfy_all
        self._val = np.r_[0]
        self._x_prev = None

    def _keep(self, state, x):
        """What the criterion keeps of x for its next check: a reference when the solver promises never
        to write a tensor it has published under this name (state["__immutable__"]), else a copy."""
        if hasattr(state, "get") and self._var in state.get("__immutable__", ()):
            return x
        return _dev.copy(x)

    def _fused(self, state, x):
        """The solver step's own statistics for this check, or None: the fused PGD step publishes
        (var, x_new, x, per-tile partials, rows, tiles per row) when its launch computed
        sum (x_new - x)^2 and sum x^2 per tile; they are this check's statistics iff x_new is the state
        x and x is the very tensor this criterion kept at its previous check (stop_rate 1, or any rate
        whose previous check saw the launch's input)."""
        h = state.get("__relerr__") if hasattr(state, "get") else None
        if (h is None or h[0] != self._var or h[1] is not x or self._x_prev is not h[2] or self._f is not _identity
                or self._norm != 2):
            return None
        return h

    def _decide1(self, n, d, shape):
        """_decide for one row from the two finished statistics as host floats."""
        decision = n <= self._eps * d
        v = n / d if d != 0 else (np.inf if n > 0 else 0.0)
        v = np.array([0.0 if v != v else v])
        self._val = v if len(shape) == 0 else v.reshape(*shape, 1)
        return bool(decision)

    def _decide(self, st, shape):
        if st.shape[-1] == 1:  # one row: the same decision and value in host floats (no numpy temporaries)
            return self._decide1(float(st[0, 0]), float(st[1, 0]), shape)
        num = st[0].reshape(*shape, 1)
        den = st[1].reshape(*shape, 1)
        rule = np.all if self._satisfy_all else np.any
        decision = bool(rule(num <= self._eps * den))
        with np.errstate(divide="ignore", invalid="ignore"):  # 0/0 -> nan -> 0 below (stop.py:375-379)
            self._val = num / den
            self._val[np.isnan(self._val)] = 0
        return decision

    def stop(self, state) -> bool:
        x = state[self._var]
        if isinstance(x, numbers.Real):
            raise NotImplementedError("pyxu_amd: RelError on scalar state variables is not supported.")
        if self._x_prev is None:
            self._x_prev = self._keep(state, x)
            self._val = np.zeros(shape=(1,) if (x.ndim == 1) else tuple(x.shape[:-1]))
            return False
        h = self._fused(state, x)
        if h is not None:
            st = _dev.empty_f64((2, max(h[4], 1)), x)
            _dev.tile_partials_fold(h[3], h[4], h[5], st)
            if self._reduce is not None:
                st = self._reduce(st, "sum")
            self._x_prev = x
            return self._decide(_finish(st.cpu().numpy(), 2), x.shape[:-1])
        fx_prev = self._f(self._x_prev)
        fx = self._f(x)
        # numerator and denominator row statistics in one device tensor -> one host sync
        rows = fx.numel() // fx.shape[-1]
        st = _dev.empty_f64((2, max(rows, 1)), fx)
        # the reference copies x after the decision (stop.py:381); the copy is decision-independent, so it
        # is made here, before the host sync.  Identity f and the 2-norm (the default): both statistics
        # and the copy in one pass over x and x_prev (pxa_relerr_stats).
        borrow = hasattr(state, "get") and self._var in state.get("__immutable__", ())
        if self._f is _identity and self._norm == 2 and 0 < rows <= 65535 and fx.dtype == fx_prev.dtype:
            x_copy = _dev.relerr_stats(fx, fx_prev, st, copy=not borrow)
        else:
            _rowstat(fx, self._norm, fx_prev, out=st[0])
            _rowstat(fx_prev, self._norm, out=st[1])
            x_copy = None if borrow else _dev.copy(x)
        if self._reduce is not None:
            st = self._reduce(st, "max" if self._norm == np.inf else "sum")
        decision = self._decide(_finish(st.cpu().numpy(), self._norm), fx.shape[:-1])
        self._x_prev = x if borrow else x_copy
        return decision

    # hook: combine a device row statistic across shards (identity on one process)
    _reduce = None
    # Offer the fused PGD step a host buffer to fold its statistics into ("__relerr_sink__" of the solver state):
    # the step then launches the fold right behind its own launch, instead of this criterion launching it at the
    # next check, after the host's decision on the previous one -- at stop_rate 1 that put a host hop between
    # every step and its fold (r05q: 36 us per step, the device idle ~9 us of it).  PXA_RELERR_SINK=1 folds in
    # the step's last workgroup instead (pxa_pgd_tv2d_plan_step's rel_values; same bits, but its flags reached
    # the host ~200 us late on MI355X, r05e).
    _offer_sink = True
    _in_kernel_fold = os.environ.get("PXA_RELERR_SINK", "0") == "1"

    def stop_async(self, state):
        """stop() in two phases: the statistics (written by the device into pinned host memory) and the
        copy of x are enqueued now; the returned callable waits for them only and decides.  Same
        kernels, same bits, same decision, same info() as stop()."""
        x = state[self._var]
        self._last_async = ("sync", None)  # (kind, readiness probe) of this check's statistics: the lagged engine
        if (isinstance(x, numbers.Real) or self._x_prev is None or self._reduce is not None
                or self._f is not _identity or self._norm != 2):
            return super().stop_async(state)
        import torch

        rows = x.numel() // x.shape[-1]
        if not (0 < rows <= 65535 and x.dtype == self._x_prev.dtype):
            return super().stop_async(state)
        if (getattr(self, "_window_stats", False) and hasattr(state, "__setitem__") and state.get("__window_ok__")
                and state.get("x_prev") is self._x_prev):
            # (the solver's lagged engine) the NEXT step computes this check's statistics from the (x, x_prev) pair
            # it reads anyway and folds them into a ring buffer: this check is resolved after that step has run
            nb = max(2, int(getattr(self, "_nbufs", 2)))
            bufs = getattr(self, "_flag_bufs", None)
            if bufs is None or bufs[0].rows != rows or len(bufs) != nb:
                bufs = self._flag_bufs = tuple(_dev.HostFlagBuffer(rows) for _ in range(nb))
            self._win_i = (getattr(self, "_win_i", -1) + 1) % nb
            fb = bufs[self._win_i]
            seq = fb.next_seq()
            state["__relerr_window__"] = (fb, seq)
            state.pop("__relerr_sink__", None)
            self._x_prev = x
            shape = x.shape[:-1]

            if rows == 1:  # (the statistics as host floats: sqrt is _finish's numpy power 0.5, exactly rounded)
                vals = fb.values

                def resolve_window():
                    fb.wait(seq)
                    return self._decide1(math.sqrt(vals[0]), math.sqrt(vals[1]), shape)
            else:
                def resolve_window():
                    fb.wait(seq)
                    return self._decide(_finish(fb.stats.copy(), self._norm), shape)

            self._last_async = ("fused", lambda: fb.landed(seq))
            return resolve_window
        h = self._fused(state, x)
        if h is not None:
            # the step's own per-tile partials, folded straight into coherent host memory with a completion flag
            # per statistic: no pass over x / x_prev, no copy, no stream event.  x is kept (a reference) now, so
            # that the solver's next step, enqueued before the decision is read, may recycle the previous
            # iterate's buffer.  Two buffers, alternately: this check reads one while the launch behind it
            # (enqueued before the decision) may fold into the other -- the solver finds that one as the
            # "__relerr_sink__" of its state, and then the fold is part of its launch (h[6] = (buffer, seq))
            # a ring of _nbufs buffers (2: this check's and the next launch's; the solver's lagged engine keeps
            # several checks unresolved and asks for more, abc/solver.py _lag_loop)
            nb = max(2, int(getattr(self, "_nbufs", 2)))
            bufs = getattr(self, "_flag_bufs", None)
            if bufs is None or bufs[0].rows != rows or len(bufs) != nb:
                bufs = self._flag_bufs = tuple(_dev.HostFlagBuffer(rows) for _ in range(nb))
            folded = h[6] if len(h) > 6 else None
            if folded is not None and any(folded[0] is b for b in bufs):
                fb, seq = folded
            else:
                fb = bufs[0]
                seq = fb.fold(h[3], h[5])
            if self._offer_sink and hasattr(state, "__setitem__"):
                nxt = bufs[(next(i for i, b in enumerate(bufs) if b is fb) + 1) % nb]
                state["__relerr_sink__"] = (self._var, nxt, self._in_kernel_fold)
            self._x_prev = x
            shape = x.shape[:-1]

            def resolve_flags():
                fb.wait(seq)
                return self._decide(_finish(fb.stats.copy(), self._norm), shape)  # (2, rows) view

            self._last_async = ("fused", lambda: fb.landed(seq))
            return resolve_flags
        # one device / pinned-host statistics pair and one event per criterion, reused: a check is
        # resolved before the next one is issued
        buf = getattr(self, "_async_buf", None)
        if buf is None or buf[0].shape[1] != rows:
            buf = (torch.empty((2, rows), dtype=torch.float64, pin_memory=True), torch.cuda.Event())
            self._async_buf = buf
        host, ev = buf
        # the final fold writes the statistics straight into the pinned host buffer (device-mapped): no device ->
        # host copy launch between the statistics and the event
        borrow = self._var in state.get("__immutable__", ()) if hasattr(state, "get") else False
        x_copy = _dev.relerr_stats(x, self._x_prev, host, copy=not borrow)
        if borrow:
            x_copy = x
        _dev.record_event(ev)
        shape = x.shape[:-1]
        self._last_async = ("event", ev.query)  # (one buffer: resolved before the next check is issued)

        def resolve():
            _dev.wait_event(ev)
            decision = self._decide(_finish(host.numpy().copy(), self._norm), shape)
            self._x_prev = x_copy
            return decision

        return resolve

    def info(self):
        if self._val.size == 1:
            return {f"RelError[{self._var}]": float(self._val.item())}
        return {f"RelError[{self._var}]_min": float(self._val.min()), f"RelError[{self._var}]_max": float(self._val.max())}

    def clear(self):
        self._val = np.r_[0]
        self._x_prev = None
