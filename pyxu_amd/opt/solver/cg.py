"""Conjugate Gradient (mirrors reference opt/solver/cg.py:14-187)."""
import os

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.opt.solver._normal import normal_form_ex

__all__ = ["CG"]

# m_state key of row statistics a step has already computed for a state variable:
# {var: (tensor, norm, host-readable row statistic)}, read by pyxu_amd.opt.stop.AbsError
_ROWSTAT = "__rowstat__"


# A p and the CG's <p, A p> partials from one set of launches when the operator can produce them
# (pxa_dense_normal_pdot -> pxa_cg_update_tail; same bits either way).  Tests switch it off for the A/B.
_FUSED_DOT = True
# ... and the p update of a CG step formed inside the next step's operator pass (pxa_dense_normal_pdot_pfold), when
# that pass is launched ahead of the stop check: one launch and one pass over r / p fewer per step, same bits
_FOLD_P = os.environ.get("PXA_CG_FOLD_P", "1") == "1"  # (PXA_CG_FOLD_P=0: the separate p launch, for A/B)


def _rows2d(x):
    return x.reshape(-1, x.shape[-1])


class _HostRows:
    """Device float64 row vector plus its host copy, fetched with a non-blocking copy into pinned memory
    behind an event: the host waits for it only where it branches on the value (the ||r||^2 <= eps test
    of the next step), by which time that step's A p, <p, A p> and x update are already queued."""

    def __init__(self, dev, pool=None):
        """pool: a solver's list of reusable [pinned buffer, event, generation] slots, taken round robin (a pinned
        allocation and an event per statistic cost ~10 us of host time at every CG set-up and explicit-residual
        step).  A slot is re-taken only after len(pool) newer statistics; host() checks the slot's generation,
        so an object whose slot was re-taken before it was read raises instead of returning the newer value."""
        import torch

        self.dev = dev
        slot = None
        if pool is not None:
            pool[1] = (pool[1] + 1) % len(pool[0])
            slot = pool[0][pool[1]]
            if slot is None or slot[0].shape != dev.shape or slot[0].dtype != dev.dtype:
                slot = pool[0][pool[1]] = [torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True),
                                           torch.cuda.Event(), 0]
            slot[2] += 1
        else:
            slot = [torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True), torch.cuda.Event(), 1]
        self._slot, self._gen = slot, slot[2]
        self._h, self._ev = slot[0], slot[1]
        self._h.copy_(dev, non_blocking=True)
        _dev.record_event(self._ev)

    def host(self):
        if self._slot[2] != self._gen:
            raise RuntimeError("CG row statistic read after its pinned slot was reused by a newer one")
        _dev.wait_event(self._ev)
        return self._h.numpy().copy()  # (the pinned slot is reused later)


class _KernelRows(_HostRows):
    """A row statistic that a kernel writes into a device buffer AND straight into coherent host memory with a
    completion flag (pxa_cg_update into a HostFlagBuffer): no copy launch, no stream event -- the host polls
    the flag, and the next kernel (A p', launched ahead of the stop check) follows without a gap."""

    def __init__(self, dev, fb, seq):
        self.dev, self._fb, self._seq = dev, fb, seq

    def host(self):
        self._fb.wait(self._seq)
        return self._fb.values.copy()


class CG(pxa.Solver):
    """Solve ``A x = b`` for positive-definite ``A`` (cg.py:14-187)."""

    steps_taken = 0  # process-wide count of CG iterations (diagnostic: inner iterations of ADMM / prox)
    _pap_ready = None  # A p whose <p, A p> partials the tail workspace holds (see _apply_p)

    def __init__(self, A, **kwargs):
        kwargs.update(log_var=kwargs.get("log_var", ("x",)))
        super().__init__(**kwargs)
        self._A = A

    @pxrt.enforce_precision(i=("b", "x0"))
    def m_init(self, b, x0=None, restart_rate=None, _preset=None):
        mst = self._mstate
        b = _dev.require(b, "b")
        if restart_rate is not None:
            assert restart_rate >= 1
            mst["restart_rate"] = int(restart_rate)
        else:
            mst["restart_rate"] = self._A.dim
        if _preset is not None:
            # (x0 = 0, r0 = b, p0 = b) already written by the caller's kernel (pxa_admm_l1_update): the start
            # from zero below, without the fill and the two copies
            assert x0 is None and all(t.shape == b.shape and t.dtype == b.dtype for t in _preset[:3])
            mst["b"], mst["x"] = b, _preset[0]
        elif x0 is None:
            mst["b"] = b
            mst["x"] = _dev.zeros(b.shape, b)
        elif b.shape == x0.shape:
            mst["b"] = b
            mst["x"] = _dev.copy(x0)
        else:
            # broadcast the single right-hand side or initial point over the other's stack (pxa_copy2d
            # with a zero source stride)
            x0 = _dev.require(x0, "x0")
            big = b if b.numel() >= x0.numel() else x0
            n = big.shape[-1]
            rows = big.numel() // n

            def bcast(t):
                if t.numel() == big.numel():
                    return _dev.copy(t) if t is x0 else t
                return _dev.copy2d(t, _dev.empty(big.shape, t), rows, n, 0, n)

            mst["b"], mst["x"] = bcast(b), bcast(x0)
        key = (tuple(mst["x"].shape), mst["x"].dtype, str(mst["x"].device))
        if getattr(self, "_apply_key", None) != key:  # (the operator is fixed per solver: reuse across fits)
            self._apply, self._apply_key = self._make_apply(mst["x"]), key
        if _preset is not None:
            mst["residual"], mst["conjugate_dir"] = _preset[1], _preset[2]
        else:
            if x0 is None:
                # x = 0: A x = 0 exactly, so r = b - A x = b bit for bit -- skip the product (one full pass over
                # the operator per solve; QuadraticFunc.prox, i.e. every ADMM x-update, starts from zero)
                mst["residual"] = _dev.copy(mst["b"])
            else:
                mst["residual"] = _dev.axpby(1.0, mst["b"], -1.0, self._apply(mst["x"]))
            mst["conjugate_dir"] = _dev.copy(mst["residual"])
        self._rr_hist = []  # host ||r||^2 (max over rows) of the last steps: convergence-rate estimate
        self._abs_eps = self._stop_eps()
        # ||r0||^2 with an async host copy, published for the first stop check (AbsError on the residual:
        # the same reduction, so the same bits) and reused by the first step's alpha; a sub-solver then
        # launches A p0 before that check, so the device works while the host decides
        r = mst["residual"]
        ahead = _preset[3:] if _preset is not None and len(_preset) == 5 else None
        hr0 = ahead[0] if ahead else _HostRows(_dev.row_reduce(_dev.RED_SUMSQ, _rows2d(r)), self._hr_pool())
        self._rr = (hr0, r)  # ||r||^2 of the current residual (then carried from the previous step's beta)
        mst[_ROWSTAT] = {"residual": (r, 2, hr0)}
        self._Ap_next = None  # A p of the current p, launched ahead of the stop check (see m_step)
        if self._astate.get("internal"):
            self._Ap_next = ahead[1] if ahead else self._apply_p(mst["conjugate_dir"])

    def _launch_start(self, r0, p0):
        """||r0||^2 (with its async host copy) and A p0 of a solve about to start from (x0 = 0, r0, p0 = r0),
        launched by the caller right after it wrote r0 / p0 (ADMM._m_step_l1), so that the device starts the
        first operator pass while the host sets the solve up; m_init takes them as _preset[3:].  The same
        launches m_init would make, hence the same bits.  None if the operator for these vectors is not set
        up yet (the first solve)."""
        if getattr(self, "_apply_key", None) != (tuple(p0.shape), p0.dtype, str(p0.device)):
            return None
        return _HostRows(_dev.row_reduce(_dev.RED_SUMSQ, _rows2d(r0)), self._hr_pool()), self._apply_p(p0)

    def _make_apply(self, like):
        """A.apply, or -- when A = s K^T K + d I for one dense K (ADMM's QuadraticFunc.prox operator,
        opt/solver/_normal.py) and the vectors fit pxa_dense_normal -- the one-pass normal operator.  A
        row-sharded K (pyxu_amd.distributed.RowShardedLinOp): each rank applies s K_r^T K_r in one pass
        over its rows, one all-reduce sums them (the exchange K.adjoint makes anyway), then + d p."""
        nf = normal_form_ex(self._A)
        if nf is None:
            return self._A.apply
        mat, s, d, sharded, group = nf
        if not _dev.dense_normal_supported(mat, like):
            return self._A.apply
        work = [None]

        def workspace(v):
            if work[0] is None:
                import torch

                wsz = int(_dev.lib.pxa_dense_normal_workspace_bytes(_dev.dtcode(v), mat.shape[0], mat.shape[1], 1))
                work[0] = torch.empty((wsz,), dtype=torch.uint8, device=v.device)
            return work[0]

        def apply(v):
            if not _dev.dense_normal_supported(mat, v):
                return self._A.apply(v)
            if not sharded:
                return _dev.dense_normal(mat, v, s, d, work=workspace(v))
            from pyxu_amd.distributed import allreduce

            y = allreduce(_dev.dense_normal(mat, v, s, 0.0, work=workspace(v)), "sum", group)
            return _dev.axpby(1.0, y, d, v, out=y)

        def apply_pdot(v, pdot):
            if sharded or not _dev.dense_normal_supported(mat, v):
                return None
            return _dev.dense_normal(mat, v, s, d, work=workspace(v), pdot=pdot)

        def apply_pfold(r, p, p_new, rr, rr_out, fb, seq, pdot):
            return _dev.dense_normal_pfold(mat, r, p, p_new, rr, rr_out, fb, seq, s, d, workspace(p), pdot)

        apply.fused = True
        apply.pdot = apply_pdot
        apply.mat = mat
        if not sharded:
            apply.pfold = apply_pfold
        return apply

    def _apply_p(self, p):
        """A p for a CG step; when the operator can produce them in the same launches (one dense normal
        operator, one row), also the step's <p, A p> partials into the tail workspace, marked by
        self._pap_ready = A p for m_step's pxa_cg_update_tail."""
        pd = getattr(self._apply, "pdot", None)
        if pd is not None and _FUSED_DOT and p.dim() == 1:
            Ap = pd(p, self._cg_workspace(1))
            if Ap is not None:
                self._pap_ready = Ap
                return Ap
        return self._apply(p)

    def _hr_pool(self):
        """Four (pinned buffer, event) slots for _HostRows, round robin: a statistic is read by the stop check
        and the step after it, long before its slot comes round again."""
        pool = self.__dict__.get("_hr_slots")
        if pool is None:
            pool = self._hr_slots = [[None] * 4, 0]
        return pool

    def _cg_workspace(self, rows):
        import torch

        w = getattr(self, "_cg_work", None)
        need = max(int(_dev.lib.pxa_cg_update_workspace_bytes(rows)) // 8, 1)
        if w is None or w.numel() < need or w.device != self._mstate["x"].device:
            w = self._cg_work = torch.empty((need,), dtype=torch.float64, device=self._mstate["x"].device)
        return w

    def m_step(self):
        """cg.py:125-153.  alpha = ||r||^2 / <p, A p> and beta = ||r'||^2 / ||r||^2 are formed on the
        device (pxa_row_ratio, float64 division then the cast the host path would do) and applied per
        row (pxa_axpy_rows), so a step has ONE host read: ||r||^2 for the eps test, issued as an async
        copy at the end of the previous step.

        Sub-solver runs (QuadraticFunc.prox -> CG, whose stop criterion is the default AbsError on the
        residual): the new residual's ||r'||^2 is published for that criterion (the same row statistic
        it would compute, so the same bits), and A p' of the next direction is launched at the end of
        the step, before the stop check: the check then waits only for ||r'||^2, and the device works on
        A p' while the host decides.  A p' of the last step is computed and dropped (no state changes)."""
        mst = self._mstate
        CG.steps_taken += 1
        mst[_ROWSTAT] = {}
        x, r, p = mst["x"], mst["residual"], mst["conjugate_dir"]
        Ap, self._Ap_next = self._Ap_next, None
        if Ap is None:
            Ap = self._apply_p(p)
        have_pap, self._pap_ready = self._pap_ready is Ap, None
        if self._rr is not None and self._rr[1] is r:
            rr = self._rr[0]  # ||r||^2 of this r: the previous step's beta numerator (identical bits)
        else:
            rr = _HostRows(_dev.row_reduce(_dev.RED_SUMSQ, _rows2d(r)), self._hr_pool())
        self._rr = None
        eps = pxrt.Width(np.dtype(str(x.dtype).replace("torch.", ""))).eps()
        rr_host = rr.host()  # already waited for by the stop check of this iteration (same value)
        fast = (not np.any(rr_host <= eps) and self._astate["idx"] % mst["restart_rate"] != 0
                and 0 < _rows2d(x).shape[0] <= 65535)
        internal = self._astate.get("internal")
        if (fast and internal and have_pap and _FOLD_P and _FUSED_DOT and p.dim() == 1
                and getattr(self._apply, "pfold", None) is not None and _dev.dense_normal_supported(self._apply.mat, p)
                and _dev.tuning(_dev.TUNE_NORMAL_KERNEL) & 15 != 1 and not self._predict_stop(rr_host)):
            # x, r and the ||r'||^2 partials now (pxa_cg_update_xr); p' = r' + beta p, ||r'||^2's publication and
            # A p' with its <p', A p'> partials in the next operator pass, launched ahead of the stop check
            hr = self._rows_buffers(1)
            _dev.cg_update_xr(_rows2d(x), _rows2d(r), _rows2d(p), _rows2d(Ap), rr.dev, self._cg_work)
            pn = _dev.empty_like(p)
            seq = hr[1].next_seq()
            self._Ap_next = self._apply.pfold(r, p, pn, rr.dev, hr[0], hr[1], seq, self._cg_workspace(1))
            self._pap_ready = self._Ap_next
            hr = _KernelRows(hr[0], hr[1], seq)
            self._rr = (hr, r)
            mst[_ROWSTAT] = {"residual": (r, 2, hr)}
            mst["x"], mst["residual"], mst["conjugate_dir"] = x, r, pn
            return
        if fast:
            # the whole tail in three launches (pxa_cg_update): alpha, x, r, ||r'||^2, beta, p; ||r'||^2 is
            # written straight into pinned host memory for the next stop check
            hr = self._rows_buffers(_rows2d(x).shape[0])
            seq = _dev.cg_update(_rows2d(x), _rows2d(r), _rows2d(p), _rows2d(Ap), rr.dev, hr[0], hr[1], self._cg_work,
                                 have_pap=have_pap)
            hr = _KernelRows(hr[0], hr[1], seq)
            self._rr = (hr, r)
            if internal:
                mst[_ROWSTAT] = {"residual": (r, 2, hr)}
                if not self._predicted_stop(rr_host):
                    self._Ap_next = self._apply_p(p)
            mst["x"], mst["residual"], mst["conjugate_dir"] = x, r, p
            return
        pAp = _dev.row_reduce(_dev.RED_DOT, _rows2d(p), _rows2d(Ap))
        alpha = _dev.row_ratio(rr.dev, pAp, x)
        _dev.axpy_rows(alpha, 1.0, _rows2d(p), _rows2d(x), out=_rows2d(x))  # x += alpha p
        if np.any(rr_host <= eps):
            _dev.axpby(1.0, mst["b"], -1.0, self._apply(x), out=r)
        else:
            _dev.axpy_rows(alpha, -1.0, _rows2d(Ap), _rows2d(r), out=_rows2d(r))  # r -= alpha A p
        if self._astate["idx"] % mst["restart_rate"] == 0:
            _dev.axpby(1.0, mst["b"], -1.0, self._apply(x), out=r)
            _dev.axpby(0.0, p, 1.0, r, out=p)  # beta = 0
        else:
            rr_new = _dev.row_reduce(_dev.RED_SUMSQ, _rows2d(r))
            hr = _HostRows(rr_new, self._hr_pool())  # async copy of ||r'||^2, event recorded before beta / p / A p'
            beta = _dev.row_ratio(rr_new, rr.dev, p)
            _dev.axpy_rows(beta, 1.0, _rows2d(p), _rows2d(r), out=_rows2d(p))  # p = r + beta p
            self._rr = (hr, r)
            if self._astate.get("internal"):
                mst[_ROWSTAT] = {"residual": (r, 2, hr)}
                if not self._predict_stop(rr_host):
                    self._Ap_next = self._apply_p(p)
        mst["x"], mst["residual"], mst["conjugate_dir"] = x, r, p

    def _rows_buffers(self, rows):
        """(device float64 (rows,), host HostFlagBuffer) buffers for ||r'||^2, two sets used alternately (a step
        reads the previous step's device value while its kernel writes the other), plus the update workspace."""
        import torch

        bufs = getattr(self, "_rr_bufs", None)
        if bufs is None or bufs[0][0].numel() != rows:
            dev = self._mstate["x"].device
            bufs = [(torch.empty((rows,), dtype=torch.float64, device=dev),
                     _dev.HostFlagBuffer(rows, rows, rows)) for _ in range(2)]
            self._rr_bufs, self._rr_flip = bufs, 0
        self._cg_workspace(rows)
        self._rr_flip ^= 1
        return bufs[self._rr_flip]

    def _stop_eps(self):
        """eps of the AbsError(var="residual", norm=2) in this run's stop criterion (None if absent)."""
        from pyxu_amd.abc.solver import _StoppingCriteriaComposition
        from pyxu_amd.opt.stop import AbsError

        todo, found = [self._astate.get("stop_crit")], None
        while todo:
            c = todo.pop()
            if isinstance(c, _StoppingCriteriaComposition):
                todo += [c._lhs, c._rhs]
            elif isinstance(c, AbsError) and c._var == "residual" and c._norm == 2 and c._reduce is None:
                found = float(c._eps)
        return found

    def _predicted_stop(self, rr_host):
        """_predict_stop of this step, evaluated at most once per step (the fold test above may have asked it)."""
        got = self.__dict__.get("_pred_cache")
        if got is not None and got[0] is rr_host:
            return got[1]
        return self._predict_stop(rr_host)

    def _predict_stop(self, rr_host):
        """Whether the NEXT stop check will probably end the solve, from the geometric rate of the last two
        ||r||^2: then A p' is not launched ahead (it would be dropped).  A wrong guess either way only
        moves where A p' is computed; the iterates are the same."""
        self._rr_hist = (self._rr_hist + [float(np.max(rr_host))])[-2:]
        if self._abs_eps is None or len(self._rr_hist) < 2 or self._rr_hist[0] <= 0:
            out = False
        else:
            r0, r1 = self._rr_hist
            pred = r1 * (r1 / r0)  # ||r_next||^2 at the current contraction rate
            out = pred <= self._abs_eps**2
        self._pred_cache = (rr_host, out)
        return out

    def default_stop_crit(self):
        from pyxu_amd.opt.stop import AbsError

        return AbsError(eps=1e-4, var="residual", f=None, norm=2, satisfy_all=True)

    def objective_func(self):
        x, b = self._mstate["x"], self._mstate["b"]
        f = _dev.axpby(0.5, self._apply(x), -1.0, b)
        r = _dev.row_reduce(_dev.RED_DOT, f.reshape(-1, f.shape[-1]), x.reshape(-1, x.shape[-1]))
        return _dev.cast(r, x).reshape(*x.shape[:-1], 1)

    def solution(self):
        data, _ = self.stats()
        return data.get("x")
