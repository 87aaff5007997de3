"""Conjugate Gradient (mirrors reference opt/solver/cg.py:14-187)."""
import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["CG"]


def _rowsq(x):
    """||x||^2 per row -> host float64 (..., 1)."""
    r = _dev.row_reduce(_dev.RED_SUMSQ, x.reshape(-1, x.shape[-1]))
    return r.cpu().numpy().reshape(*x.shape[:-1], 1)


def _rowdot(x, y):
    r = _dev.row_reduce(_dev.RED_DOT, x.reshape(-1, x.shape[-1]), y.reshape(-1, y.shape[-1]))
    return r.cpu().numpy().reshape(*x.shape[:-1], 1)


def _rowsq_rowdot(r, p, Ap):
    """(||r||^2, <p, Ap>) per row with ONE host synchronisation (two reductions into one buffer)."""
    rows = r.numel() // r.shape[-1]
    buf = _dev.empty_f64((2, rows), r)
    _dev.row_reduce(_dev.RED_SUMSQ, r.reshape(-1, r.shape[-1]), out=buf[0])
    _dev.row_reduce(_dev.RED_DOT, p.reshape(-1, p.shape[-1]), Ap.reshape(-1, Ap.shape[-1]), out=buf[1])
    h = buf.cpu().numpy()
    sh = (*r.shape[:-1], 1)
    return h[0].reshape(sh), h[1].reshape(sh)


class CG(pxa.Solver):
    """Solve ``A x = b`` for positive-definite ``A`` (cg.py:14-187)."""

    def __init__(self, A, **kwargs):
        kwargs.update(log_var=kwargs.get("log_var", ("x",)))
        super().__init__(**kwargs)
        self._A = A

    @pxrt.enforce_precision(i=("b", "x0"))
    def m_init(self, b, x0=None, restart_rate=None):
        mst = self._mstate
        b = _dev.require(b, "b")
        if restart_rate is not None:
            assert restart_rate >= 1
            mst["restart_rate"] = int(restart_rate)
        else:
            mst["restart_rate"] = self._A.dim
        if x0 is None:
            mst["b"] = b
            mst["x"] = _dev.zeros(b.shape, b)
        elif b.shape == x0.shape:
            mst["b"] = b
            mst["x"] = _dev.copy(x0)
        else:
            import torch

            bb, xx = torch.broadcast_tensors(b, x0)
            mst["b"], mst["x"] = bb.contiguous(), xx.contiguous()
        mst["residual"] = _dev.axpby(1.0, mst["b"], -1.0, self._A.apply(mst["x"]))
        mst["conjugate_dir"] = _dev.copy(mst["residual"])
        self._rr = None  # ||r||^2 of the current residual, carried from the previous step's beta

    def _scale_rows(self, coef, v):
        """coef (..., 1) host numpy -> device tensor broadcast multiplier."""
        import torch

        c = torch.from_numpy(np.ascontiguousarray(coef, dtype=np.float64)).to(device=v.device, dtype=v.dtype)
        return c

    def m_step(self):
        mst = self._mstate
        x, r, p = mst["x"], mst["residual"], mst["conjugate_dir"]
        Ap = self._A.apply(p)
        # ||r||^2 is the previous step's beta numerator (same reduction of the same r: identical bits);
        # otherwise it is computed together with <p, A p> behind one host synchronisation
        if self._rr is not None and self._rr[1] is r:
            rr, pAp = self._rr[0], _rowdot(p, Ap)
        else:
            rr, pAp = _rowsq_rowdot(r, p, Ap)
        self._rr = None
        alpha = rr / pAp
        eps = pxrt.Width(np.dtype(str(x.dtype).replace("torch.", ""))).eps()
        if x.ndim <= 1 or x.numel() == x.shape[-1]:
            a = float(np.asarray(alpha).reshape(-1)[0])
            _dev.axpby(1.0, x, a, p, out=x)
            if np.any(rr <= eps):
                _dev.axpby(1.0, mst["b"], -1.0, self._A.apply(x), out=r)
            else:
                _dev.axpby(1.0, r, -a, Ap, out=r)
            if self._astate["idx"] % mst["restart_rate"] == 0:
                beta = 0.0
                _dev.axpby(1.0, mst["b"], -1.0, self._A.apply(x), out=r)
            else:
                rr_new = _rowsq(r)
                self._rr = (rr_new, r)
                beta = float((rr_new / rr).reshape(-1)[0])
            _dev.axpby(beta, p, 1.0, r, out=p)
        else:
            # stacked right-hand sides: per-row coefficients
            A_ = self._scale_rows(alpha, x).reshape(-1)
            _dev.axpy_rows(A_, 1.0, p, x, out=x)  # x += alpha p (per row)
            if np.any(rr <= eps):
                _dev.axpby(1.0, mst["b"], -1.0, self._A.apply(x), out=r)
            else:
                _dev.axpy_rows(A_, -1.0, Ap, r, out=r)  # r -= alpha A p
            if self._astate["idx"] % mst["restart_rate"] == 0:
                _dev.axpby(1.0, mst["b"], -1.0, self._A.apply(x), out=r)
                _dev.axpby(0.0, p, 1.0, r, out=p)
            else:
                rr_new = _rowsq(r)
                self._rr = (rr_new, r)
                B_ = self._scale_rows(rr_new / rr, p).reshape(-1)
                _dev.axpy_rows(B_, 1.0, p, r, out=p)  # p = r + beta p (per row)
        mst["x"], mst["residual"], mst["conjugate_dir"] = x, r, p

    def default_stop_crit(self):
        from pyxu_amd.opt.stop import AbsError

        return AbsError(eps=1e-4, var="residual", f=None, norm=2, satisfy_all=True)

    def objective_func(self):
        x, b = self._mstate["x"], self._mstate["b"]
        f = _dev.axpby(0.5, self._A.apply(x), -1.0, b)
        r = _dev.row_reduce(_dev.RED_DOT, f.reshape(-1, f.shape[-1]), x.reshape(-1, x.shape[-1]))
        return r.to(x.dtype).reshape(*x.shape[:-1], 1)

    def solution(self):
        data, _ = self.stats()
        return data.get("x")
