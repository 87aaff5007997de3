"""Proximal Gradient Descent (mirrors reference opt/solver/pgd.py:14-219)."""
import itertools
import os
import sys
import math
import warnings

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.opt.solver._fused import match_pgd_deblur
from pyxu_amd.util import copy_if_unsafe

__all__ = ["PGD"]

# PXA_NO_SPEC=1: synchronous stop checks (A/B measurements of the speculative ones)
_NO_SPEC = os.environ.get("PXA_NO_SPEC", "0") == "1"


class AutoInferenceWarning(UserWarning):
    pass


class _Momentum:
    """The momentum sequence a_k (pgd.py:164-171) with `push`, which returns a consumed value (rollback of a
    speculative step) without nesting one more itertools.chain per rollback."""

    def __init__(self, it):
        self._it = iter(it)
        self._buf = []

    def __iter__(self):
        return self

    def __next__(self):
        return self._buf.pop() if self._buf else next(self._it)

    def push(self, v):
        self._buf.append(v)


class PGD(pxa.Solver):
    r"""Accelerated proximal gradient descent (Chambolle--Dossal momentum).

    ``fit(x0, tau=None, acceleration=True, d=75, fused=True)``.  With ``fused=True`` (default) a
    deblurring objective ``1/2||H.-y||^2 [+ lam env_mu(L21) o Grad]`` with ``g`` in
    {None, PositiveOrthant, lam*L1Norm} runs each iteration as ONE HIP launch; anything else runs the
    generic rule-by-rule path (also HIP).
    """

    def __init__(self, f=None, g=None, **kwargs):
        kwargs.update(log_var=kwargs.get("log_var", ("x",)))
        super().__init__(**kwargs)
        if (f is None) and (g is None):
            raise ValueError("Cannot minimize always-0 functional. At least one of Parameter[f, g] must be specified.")
        self._f = f
        self._g = g

    @pxrt.enforce_precision(i=("x0", "tau"))
    def m_init(self, x0, tau=None, acceleration: bool = True, d=75, fused: bool = True):
        from pyxu_amd.operator.linop import NullFunc

        mst = self._mstate
        x0 = _dev.require(x0, "x0")
        mst["x"] = mst["x_prev"] = x0
        if self._f is None:
            self._f = NullFunc(dim=x0.shape[-1])
        if self._g is None:
            self._g = NullFunc(dim=x0.shape[-1])
        if tau is None:
            mst["tau"] = pxrt.coerce(1 / self._f.diff_lipschitz)
            if math.isinf(mst["tau"]):
                mst["tau"] = pxrt.coerce(1)
                warnings.warn(rf"The gradient/proximal step size \tau is auto-set to {mst['tau']}.", AutoInferenceWarning)
        else:
            try:
                assert tau > 0
                mst["tau"] = tau
            except Exception:
                raise ValueError(f"tau must be positive, got {tau}.")
        if acceleration:
            try:
                assert d > 2
                mst["a"] = _Momentum(pxrt.coerce(k / (k + 1 + d)) for k in itertools.count(start=0))
            except Exception:
                raise ValueError(f"Expected d > 2, got {d}.")
        else:
            mst["a"] = _Momentum(itertools.repeat(pxrt.coerce(0)))
        self._plan = match_pgd_deblur(self._f, self._g, x0) if fused else None
        if self._plan is not None:
            p = self._plan
            y = _dev.axpby(-1.0, pxrt.coerce(p["shift"]))  # data y = -shift
            # the fused kernel evaluates H^T (H yk - y) as (H^T H) yk - H^T y: H^T y is iteration-invariant
            p["hty"] = _dev.copy(p["H"].adjoint(y))
            p["stack"] = p["rows"] * p["B"]
            p["plan"] = _dev.PgdPlan(x0, p["stack"], p["B"], p["n0"], p["n1"], p["taps0"], p["taps1"], p["h0"], p["h1"],
                                     p["lam"], p["mu"], p["prox"])
            # per-tile RelError partials of the launch that precedes a stop check (pxa_tile_partials_fold)
            ntiles = int(_dev.lib.pxa_pgd_tv2d_partials_count(p["stack"], p["n0"], p["n1"]))
            p["parts"] = _dev.empty_f64((2 * ntiles,), x0)
            p["tiles_per_row"] = ntiles // max(p["rows"], 1)
            self._spare = None
            self._x_check = None  # the x of the last stop check (RelError partials against it)
            # the solver never writes a tensor it has published as x (outputs go to fresh or recycled
            # buffers nobody else references), so stop criteria may keep references instead of copies
            mst["__immutable__"] = frozenset({"x"})
            # the step can compute the RelError statistics of the (x, x_prev) pair it reads (pxa_pgd_tv2d_plan_step_wfold):
            # offered to the criterion under the lagged engine, which resolves a check after the next step ran
            mst["__window_ok__"] = True

    # publish the fused step's per-tile RelError partials to the stop criteria (False: A/B and parity tests)
    _fused_relerr = True

    # speculative stop checks (abc/solver.py _step_speculative): the fused step writes a buffer that is
    # neither x nor x_prev, so undoing it is restoring (x, x_prev) and the momentum value it consumed
    def _spec_supported(self):
        return self._plan is not None and not _NO_SPEC

    def _spec_begin(self):
        mst = self._mstate
        self._spec_refs = 1  # the token below holds one more reference to x_prev
        return (mst["x"], mst["x_prev"])

    def _spec_rollback(self, token):
        mst = self._mstate
        mst["x"], mst["x_prev"] = token
        mst["a"].push(self._last_a)
        mst.pop("__relerr__", None)
        self._spare = None
        self._spec_refs = 0

    # lagged stop checks (abc/solver.py _lag_loop): a check's state is (x, x_prev); dropping the steps launched after
    # it means restoring that pair and returning their momentum values (the fused path only: its steps write a
    # buffer that is neither x nor x_prev, and one the solver holds no other reference to)
    _LAG_PUB = os.environ.get("PXA_LAG_PUB", "1") == "1"

    def _lag_supported(self):
        return self._plan is not None and self._fused_relerr and not _NO_SPEC

    def _lag_flush(self):
        """Publish the window statistics still waiting for the next launch's extra workgroup (the run will not
        launch again): one fold launch."""
        pend = getattr(self, "_wpub_pending", None)
        self._wpub_pending = None
        if pend is not None:
            p = self._plan
            _dev.tile_partials_publish(pend[0], p["rows"], p["tiles_per_row"], pend[1], pend[2])

    def _lag_snapshot(self):
        mst = self._mstate
        return (mst["x"], mst["x_prev"])

    def _lag_restore(self, snap, undone):
        mst = self._mstate
        mst["x"], mst["x_prev"] = snap
        hist = list(getattr(self, "_a_hist", ()))
        for v in reversed(hist[len(hist) - undone:] if undone > 0 else []):  # next() returns the earliest first
            mst["a"].push(v)
        mst.pop("__relerr__", None)
        mst.pop("__relerr_sink__", None)
        mst.pop("__relerr_window__", None)
        self._wpub_pending = None
        self._spare = None
        self._x_check = None
        self.__dict__.pop("_pool", None)

    # Output buffers under the lagged engine: the held check states keep the old x_prev referenced, so the refcount
    # recycling below never finds it free and every step would allocate (torch.empty_like: several us of host time
    # per step at stop_rate 1, where the host sets the pace).  Retired iterates wait in a small pool instead and are
    # reused once nothing references them (the same refcount + storage test: a held state, a steps() item or a user
    # view keeps a buffer out of reuse).
    _POOL_MAX = 16

    def _pool_take(self, x, xp):
        pool = self.__dict__.get("_pool")
        if pool:
            for i in range(len(pool)):
                b = pool[i]
                # references: the pool's, b, getrefcount's argument
                if (sys.getrefcount(b) == 3 and b is not x and b is not xp and b.shape == x.shape and b.dtype == x.dtype
                        and _dev.storage_exclusive(b)):
                    del pool[i]
                    return b
        return _dev.empty_like(x)

    def _pool_put(self, b):
        if self._astate.get("lag") is None:  # (only while the lagged engine runs; emptied when it ends)
            self.__dict__.pop("_pool", None)
            return
        pool = self.__dict__.setdefault("_pool", [])
        pool.append(b)
        if len(pool) > self._POOL_MAX:
            del pool[0]

    def _rel_on_x(self):
        """Whether the run's stop criterion holds a RelError on x (the statistics the fused step's partials feed):
        without one, the check steps skip the partials (an extra read of x per launch)."""
        crit = self._astate.get("stop_crit")
        key = id(crit)
        cached = self.__dict__.get("_rel_on_x_cache")
        if cached is not None and cached[0] == key and cached[1] is crit:
            return cached[2]
        from pyxu_amd.abc.solver import _StoppingCriteriaComposition
        from pyxu_amd.opt.stop import RelError

        todo, found = [crit], False
        while todo:
            c = todo.pop()
            if isinstance(c, _StoppingCriteriaComposition):
                todo += [c._lhs, c._rhs]
            elif isinstance(c, RelError) and c._var == "x":
                found = True
        self._rel_on_x_cache = (key, crit, found)
        return found

    def m_step(self):
        mst = self._mstate
        a = next(mst["a"])
        self._last_a = a
        ah = self.__dict__.get("_a_hist")
        if ah is None:
            import collections

            ah = self._a_hist = collections.deque(maxlen=256)
        ah.append(a)
        if self._plan is not None:
            p = self._plan
            mst.pop("__relerr__", None)  # (holds x_prev: drop it before the buffer-recycling refcount below)
            x, xp = mst["x"], mst["x_prev"]
            out = self._spare
            if out is None or out is x or out is xp:
                out = self._pool_take(x, xp)
            tau = mst["tau"]
            wnd = mst.pop("__relerr_window__", None)
            if wnd is not None:
                # (lagged engine) this launch computes the statistics of the check before it from its window loads,
                # and an extra workgroup of it publishes those of the check before that (two partials buffers,
                # alternately): no fold launch (PXA_LAG_PUB=0: a fold launch behind the step instead)
                if self._LAG_PUB:
                    wp = p.get("wparts")
                    if wp is None:
                        wp = p["wparts"] = (p["parts"], _dev.empty_f64(p["parts"].shape, x))
                    self._wpar_i = getattr(self, "_wpar_i", 0) ^ 1
                    cur = wp[self._wpar_i]
                    p["plan"].step_wpub(x, xp, p["hty"], out, a, tau, tau * p["prox_scale"], cur,
                                        getattr(self, "_wpub_pending", None))
                    self._wpub_pending = (cur, wnd[0], wnd[1])
                else:
                    p["plan"].step_window(x, xp, p["hty"], out, a, tau, tau * p["prox_scale"], p["parts"], wnd[0], wnd[1])
                mst["x_prev"], mst["x"] = x, out
                refs = 2 + getattr(self, "_spec_refs", 0)
                self._spec_refs = 0
                self._spare = xp if (sys.getrefcount(xp) == refs and xp.data_ptr() != x.data_ptr()
                                     and _dev.storage_exclusive(xp)) else None
                if self._spare is None:
                    self._pool_put(xp)
                return
            # RelError partials only for the launch right before a stop check (the engine advances idx
            # before m_step: the next check runs at idx when idx % stop_rate == 0).  RelError compares with
            # the iterate of the PREVIOUS check (opt/stop.py:353-382), which the criterion keeps: x itself at
            # stop_rate 1, else the x this solver saw at that check (self._x_check, the same tensor object)
            ast = self._astate
            sr = ast.get("stop_rate")
            if sr is not None and (ast["idx"] - 1) % sr == 0:
                self._x_check = x  # a check ran right before this step, on this x
            want = self._fused_relerr and sr is not None and ast["idx"] % sr == 0 and self._rel_on_x()
            parts = p["parts"] if want else None
            xref = self._x_check if want else None
            if xref is None:
                xref = x
            # the stop criterion's host buffer for this launch's folded statistics, if it offered one
            sink = mst.pop("__relerr_sink__", None) if want else None
            in_kernel = sink is not None and sink[0] == "x" and len(sink) > 2 and bool(sink[2])
            sink = sink[1] if sink is not None and sink[0] == "x" else None
            # the fold: in the launch's last workgroup (PXA_RELERR_SINK=1), else a fold launch right behind it,
            # enqueued by the same C call (a side stream for it, so that it ran beside the next launch, cost more
            # host time in the event record / wait than it saved: r05s)
            seq = sink.next_seq() if sink is not None else 0
            p["plan"].step(x, xp, p["hty"], out, a, tau, tau * p["prox_scale"], partials=parts,
                           x_ref=None if xref is x else xref, sink=sink, seq=seq,
                           fold_launch=sink is not None and not in_kernel)
            if want:  # (var, x_new, the x the statistics are relative to, partials, rows, tiles per row, folded)
                mst["__relerr__"] = ("x", out, xref, parts, p["rows"], p["tiles_per_row"],
                                     (sink, seq) if sink is not None else None)
            else:
                mst.pop("__relerr__", None)
            mst["x_prev"], mst["x"] = x, out
            # recycle the old x_prev as the next output buffer iff nobody else holds it (the reference
            # allocates fresh arrays, so user-held results must never be overwritten)
            refs = 2 + getattr(self, "_spec_refs", 0)
            self._spec_refs = 0
            self._spare = xp if (sys.getrefcount(xp) == refs and xp.data_ptr() != x.data_ptr()
                                 and _dev.storage_exclusive(xp)) else None
            return
        # generic path: y = (x - x_prev) * a + x ; z = y - tau * grad(y) ; x+ = prox_g(z, tau)
        y = _dev.extrapolate(a, mst["x"], mst["x_prev"])
        z = copy_if_unsafe(self._f.grad(y))
        z = _dev.axpby(-mst["tau"], z, 1.0, y, out=z)
        mst["x_prev"], mst["x"] = mst["x"], self._g.prox(z, mst["tau"])

    def default_stop_crit(self):
        from pyxu_amd.opt.stop import RelError

        return RelError(eps=1e-4, var="x", f=None, norm=2, satisfy_all=True)

    def objective_func(self):
        x = self._mstate["x"]
        return _dev.axpby(1.0, self._f.apply(x), 1.0, self._g.apply(x))

    def solution(self):
        data, _ = self.stats()
        return data.get("x")
