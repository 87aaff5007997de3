"""
Primal-dual splitting solvers (mirrors reference opt/solver/pds.py): CondatVu (CV), PD3O,
ChambollePock (CP), LorisVerhoeven (LV), DavisYin (DY), DouglasRachford (DR), ADMM,
ForwardBackward (FB), ProximalPoint (PP).

Step-size rules, momentum and initialisation follow the reference line by line (pds.py:131-204,
444-517, 763-864, 1604-1687); the iterates live on the MI355X and every update is a HIP kernel.
"""
import math
import sys
import types
import warnings

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = [
    *("CondatVu", "CV"),
    "PD3O",
    *("ChambollePock", "CP"),
    *("LorisVerhoeven", "LV"),
    *("DavisYin", "DY"),
    *("DouglasRachford", "DR"),
    "ADMM",
    *("ForwardBackward", "FB"),
    *("ProximalPoint", "PP"),
]


def _is_null(op) -> bool:
    return getattr(op, "_name", None) == "NullFunc"


class _PrimalDualSplitting(pxa.Solver):
    """Base class of PDS solvers (pds.py:26-204)."""

    def __init__(self, f=None, g=None, h=None, K=None, beta=None, **kwargs):
        from pyxu_amd.operator.linop import IdentityOp, NullFunc, NullOp

        kwargs.update(log_var=kwargs.get("log_var", ("x", "z")))
        super().__init__(**kwargs)
        if (f is None) and (g is None) and (h is None):
            raise ValueError("Cannot minimize always-0 functional. At least one of Parameter[f, g, h] must be specified.")
        primal_dim = f.dim if f is not None else (g.dim if g is not None else h.dim)
        if h is not None:
            dual_dim = h.dim
        elif K is not None:
            dual_dim = K.shape[0]
        else:
            dual_dim = primal_dim
        self._f = NullFunc(dim=primal_dim) if f is None else f
        self._g = NullFunc(dim=primal_dim) if g is None else g
        self._h = NullFunc(dim=dual_dim) if h is None else h
        self._beta = self._set_beta(beta)
        if h is not None:
            self._K = IdentityOp(dim=h.dim) if K is None else K
        else:
            if K is None:
                K_dim = f.dim if f is not None else g.dim
                self._K = NullOp(shape=(K_dim, K_dim))
            else:
                raise ValueError("Optional argument ``h`` mut be specified if ``K`` is not None.")
        self._objective_func_cache = None  # f + g + h o K, built on first use (construction stays compute-free)

    @pxrt.enforce_precision(i=("x0", "z0", "tau", "sigma", "rho"), allow_None=True)
    def m_init(self, x0, z0=None, tau=None, sigma=None, rho=None, tuning_strategy=1, fused=True):
        mst = self._mstate
        mst["x"] = _dev.require(x0, "x0")
        mst["z"] = self._set_dual_variable(z0)
        self._tuning_strategy = int(tuning_strategy)
        gamma = self._set_gamma(tuning_strategy)
        mst["tau"], mst["sigma"], delta = self._set_step_sizes(tau, sigma, gamma)
        mst["rho"] = self._set_momentum_term(rho, delta)
        self._spare = None
        self._la = None  # look-ahead step: (state arrays it was computed for, x of the next iteration)
        self._zspare = None
        self._plan = self._fused_plan(mst["x"]) if fused else None
        if self._plan is not None:
            # the fused steps never write a tensor they have published as x while anything else references it (new
            # or recycled buffers, reuse guarded by the reference count): stop criteria may keep references instead
            # of copies (RelError: no 4-byte-per-voxel copy of x at every check)
            mst["__immutable__"] = frozenset({"x"})

    _FUSED_ALGO = None  # pxa_pds_step algo code of the subclass (0 PD3O, 1 CondatVu), None: no fused step

    def _fused_plan(self, x0):
        """Parameters of the fused pxa_pds_step iteration, or None (generic rule-by-rule path)."""
        from pyxu_amd.opt.solver._fused import match_pds_deblur

        if self._FUSED_ALGO is None or _is_null(self._h) or x0.dtype != self._mstate["z"].dtype:
            return None
        p = match_pds_deblur(self._f, self._g, self._h, self._K, x0)
        if p is None:
            return None
        mst = self._mstate
        y = _dev.axpby(-1.0, pxrt.coerce(p["shift"]))  # data y = -shift
        p["hty"] = _dev.copy(p["H"].adjoint(y))  # S^T y: iteration-invariant (G x - S^T y = grad f(x))
        stack = p["rows"]
        p["pre"] = _dev.pds_args(stack, 1, p["n0"], p["n1"], p["n2"], p["D"], p["taps"], p["c0"], p["c1"], mst["tau"],
                                 mst["sigma"], mst["rho"], p["lam"], p["prox"], mst["tau"] * p["prox_scale"], p["h_kind"])
        x = mst["x"]
        p["w"] = _dev.empty_like(x)
        p["q"] = None if p["taps"][0] == ([0], [1.0]) else _dev.empty_like(x)
        p["nseg"] = 0  # axis-0 march segments (0: one per column; tuning knob of pxa_pds_step)
        p["la"] = bool(self._LOOKAHEAD)
        p["kt"] = _dev.empty_like(x) if p["la"] and self._FUSED_ALGO == 1 else None
        return p

    # Two launches per iteration (pxa_pds_step_la: kernel B + the dual update fused with the next
    # iteration's axis-0 march) instead of three (pxa_pds_step); False selects the three-launch step.
    _LOOKAHEAD = True

    def _primed(self, *state):
        """True iff the previous look-ahead step left the march of this iteration done for exactly
        these state arrays, unmodified since (any restart or state replacement re-primes).  An array
        edited in place through torch bumps its version counter, which is recorded with it; an edit that
        bypasses torch (raw pointers) must call ``reset_lookahead()``."""
        la = self._la
        return (la is not None and len(la[0]) == len(state)
                and all(a is b and v == getattr(b, "_version", v) for (a, v), b in zip(la[0], state)))

    @staticmethod
    def _la_key(*state):
        return tuple((t, getattr(t, "_version", None)) for t in state)

    def reset_lookahead(self):
        """Forget the look-ahead march of the next iteration: the next m_step re-primes from the current
        state.  Call after writing the solver state (``_mstate`` x / u / z) in place outside torch."""
        self._la = None

    def _take_zspare(self, z):
        zs = self._zspare
        self._zspare = None
        return zs if zs is not None and zs is not z else _dev.empty_like(z)

    @staticmethod
    def _owned(t, extra=0):
        """True iff `t` is referenced only by the solver state (+ `extra` caller locals): it may be
        overwritten in place.  The reference allocates fresh arrays each step, so arrays a user holds
        (z0, logged iterates, and views of user arrays such as ``batch[i]``) are never modified."""
        return sys.getrefcount(t) <= 3 + extra and _dev.storage_exclusive(t)

    def m_step(self):
        raise NotImplementedError

    def default_stop_crit(self):
        from pyxu_amd.opt.stop import RelError

        sx = RelError(eps=1e-4, var="x", f=None, norm=2, satisfy_all=True)
        sz = RelError(eps=1e-4, var="z", f=None, norm=2, satisfy_all=True)
        return sx & sz if not _is_null(self._h) else sx

    def solution(self, which="primal"):
        data, _ = self.stats()
        if which == "primal":
            assert "x" in data, "Primal variable x was not logged (declare it in log_var to log it)."
            return data.get("x")
        if which == "dual":
            assert "z" in data, "Dual variable z was not logged (declare it in log_var to log it)."
            return data.get("z")
        raise ValueError(f"Parameter which must be one of ['primal', 'dual'] got: {which}.")

    @property
    def _objective_func(self):
        if self._objective_func_cache is None:
            self._objective_func_cache = self._f + self._g + (self._h * self._K)
        return self._objective_func_cache

    def objective_func(self):
        return self._objective_func(self._mstate["x"])

    @pxrt.enforce_precision(i="beta", allow_None=True)
    def _set_beta(self, beta):
        if beta is None:
            dl = self._f.diff_lipschitz
            if math.isfinite(dl):
                return pxrt.coerce(dl)
            raise ValueError("beta: automatic inference not supported for operators with unbounded Lipschitz gradients.")
        return beta

    def _set_dual_variable(self, z):
        if z is None:
            return self._K(_dev.copy(self._mstate["x"]))
        return _dev.require(z, "z0")

    def _set_gamma(self, tuning_strategy):
        return pxrt.coerce(self._beta) if tuning_strategy != 2 else pxrt.coerce(self._beta / 1.9)

    def _set_step_sizes(self, tau, sigma, gamma):
        raise NotImplementedError

    def _set_momentum_term(self, rho, delta):
        if rho is None:
            rho = 1.0 if self._tuning_strategy != 3 else delta - 0.1
        else:
            assert rho <= delta, f"Parameter rho must be smaller than delta: {rho} > {delta}."
        return pxrt.coerce(rho)

    def _K_lipschitz(self):
        return self._K.lipschitz


_PDS = _PrimalDualSplitting


def _knorm_msg():
    return "Please compute the Lipschitz constant of the linear operator K by calling its method 'estimate_lipschitz()'"


class CondatVu(_PrimalDualSplitting):
    """Condat-Vu primal-dual splitting (pds.py:207-520)."""

    _FUSED_ALGO = 1

    def m_step(self):
        mst = self._mstate
        if self._plan is not None:
            p = self._plan
            x, z = mst["x"], mst["z"]
            if p["la"]:
                primed = self._primed(x, z)
                self._la = None
                out = self._spare
                if out is None or out is x:
                    out = _dev.empty_like(x)
                z_out = self._take_zspare(z)
                _dev.pds_step_la(1, p["pre"], primed, x, None, z, p["hty"], out, None, z_out, p["q"], p["kt"], p["w"],
                                 nseg=p["nseg"])
                mst["x"], mst["z"] = out, z_out
                self._la = (self._la_key(out, z_out), None)
                self._spare = x if (sys.getrefcount(x) == 2 and _dev.storage_exclusive(x)) else None
                self._zspare = z if (sys.getrefcount(z) == 2 and _dev.storage_exclusive(z)) else None
                return
            out = self._spare
            if out is None or out is x:
                out = _dev.empty_like(x)
            z_out = z if self._owned(z, extra=1) else _dev.empty_like(z)
            _dev.pds_step(1, p["pre"], x, None, z, p["hty"], out, None, z_out, p["q"], p["w"], nseg=p["nseg"])
            mst["x"], mst["z"] = out, z_out
            self._spare = x if (sys.getrefcount(x) == 2 and _dev.storage_exclusive(x)) else None
            return
        x = mst["x"]
        tau = mst["tau"]
        # x - tau*grad_f(x) - tau*K^T z
        t = _dev.axpby(1.0, x, -tau, self._f.grad(x))
        t = _dev.axpby(1.0, t, -tau, self._K.jacobian(x).adjoint(mst["z"]), out=t)
        x_temp = self._g.prox(t, tau=tau)
        if not _is_null(self._h):
            u = _dev.axpby(2.0, x_temp, -1.0, x)
            z_in = _dev.axpby(1.0, mst["z"], mst["sigma"], self._K(u))
            z_temp = self._h.fenchel_prox(z_in, sigma=mst["sigma"])
            mst["z"] = _dev.axpby(mst["rho"], z_temp, 1 - mst["rho"], mst["z"])
        mst["x"] = _dev.axpby(mst["rho"], x_temp, 1 - mst["rho"], x)

    def _set_step_sizes(self, tau, sigma, gamma):
        if not isinstance(self._K, pxa.LinOp):
            raise ValueError("Automatic selection of parameters is only supported in the case in which K is a linear operator. "
                             f"Got operator of type {self._K.__class__}.")
        tau = None if tau == 0 else tau
        sigma = None if sigma == 0 else sigma
        L = self._K_lipschitz
        if (tau is not None) and (sigma is None):
            assert tau > 0, f"Parameter tau must be positive, got {tau}."
            if _is_null(self._h):
                assert tau <= 1 / gamma, f"Parameter tau must be smaller than 1/gamma: {tau} > {1 / gamma}."
                sigma = 0
            else:
                if math.isfinite(L()):
                    sigma = ((1 / tau) - gamma) * (1 / L() ** 2)
                else:
                    raise ValueError(_knorm_msg())
        elif (tau is None) and (sigma is not None):
            assert sigma > 0
            if _is_null(self._h):
                tau = 1 / gamma
            else:
                if math.isfinite(L()):
                    tau = 1 / (gamma + (sigma * L() ** 2))
                else:
                    raise ValueError(_knorm_msg())
        elif (tau is None) and (sigma is None):
            if self._beta > 0:
                if _is_null(self._h):
                    tau, sigma = 1 / gamma, 0
                else:
                    if math.isfinite(L()):
                        tau = sigma = (1 / L() ** 2) * ((-gamma / 2) + math.sqrt((gamma**2 / 4) + L() ** 2))
                    else:
                        raise ValueError(_knorm_msg())
            else:
                if _is_null(self._h):
                    tau, sigma = 1, 0
                else:
                    if math.isfinite(L()):
                        tau = sigma = 1 / L()
                    else:
                        raise ValueError(_knorm_msg())
        delta = (
            2
            if (self._beta == 0 or (isinstance(self._f, pxa.QuadraticFunc) and gamma <= self._beta))
            else 2 - self._beta / (2 * gamma)
        )
        return pxrt.coerce(tau), pxrt.coerce(sigma), pxrt.coerce(delta)


CV = CondatVu


class PD3O(_PrimalDualSplitting):
    """Primal-Dual Three-Operator splitting (pds.py:523-864)."""

    _FUSED_ALGO = 0

    @pxrt.enforce_precision(i=("x0", "z0", "tau", "sigma", "rho"), allow_None=True)
    def m_init(self, x0, z0=None, tau=None, sigma=None, rho=None, tuning_strategy=1, fused=True):
        super().m_init(x0=x0, z0=z0, tau=tau, sigma=sigma, rho=rho, tuning_strategy=tuning_strategy, fused=fused)
        if _is_null(self._g) and _is_null(self._h):
            self._mstate["u"] = _dev.axpby(1.01, self._mstate["x"])
        else:
            self._mstate["u"] = _dev.copy(self._mstate["x"])

    def m_step(self):
        mst = self._mstate
        if self._plan is not None:
            p = self._plan
            x, u, z = mst["x"], mst["u"], mst["z"]
            if p["la"]:
                # this iteration's x is the previous call's look-ahead x (primed) or computed here
                primed = self._primed(x, u, z)
                x_cur = self._la[1] if primed else None
                self._la = None  # drop its references before the ownership checks
                if x_cur is None:
                    x_cur = x if self._owned(x, extra=1) else _dev.empty_like(x)
                x_next = self._spare
                if x_next is None or x_next is x_cur:
                    x_next = _dev.empty_like(x)
                u_out = u if self._owned(u, extra=1) else _dev.empty_like(u)
                z_out = self._take_zspare(z)
                _dev.pds_step_la(0, p["pre"], primed, x_cur, u, z, p["hty"], x_next, u_out, z_out, p["q"], None,
                                 p["w"], nseg=p["nseg"])
                mst["x"], mst["u"], mst["z"] = x_cur, u_out, z_out
                self._la = (self._la_key(x_cur, u_out, z_out), x_next)
                del x_next, u_out
                # the previous iterate's arrays are reused when nothing else holds them
                self._spare = x if (x is not x_cur and sys.getrefcount(x) == 2 and _dev.storage_exclusive(x)) else None
                self._zspare = z if (sys.getrefcount(z) == 2 and _dev.storage_exclusive(z)) else None
                return
            x_out = x if self._owned(x, extra=1) else _dev.empty_like(x)
            u_out = u if self._owned(u, extra=1) else _dev.empty_like(u)
            z_out = z if self._owned(z, extra=1) else _dev.empty_like(z)
            _dev.pds_step(0, p["pre"], None, u, z, p["hty"], x_out, u_out, z_out, p["q"], p["w"], nseg=p["nseg"])
            mst["x"], mst["u"], mst["z"] = x_out, u_out, z_out
            return
        tau, rho = mst["tau"], mst["rho"]
        t = _dev.axpby(1.0, mst["u"], -tau, self._K.jacobian(mst["u"]).adjoint(mst["z"]))
        mst["x"] = self._g.prox(t, tau=tau)
        u_temp = _dev.axpby(1.0, mst["x"], -tau, self._f.grad(mst["x"]))
        if not _is_null(self._h):
            w = _dev.lincomb3(1.0, mst["x"], 1.0, u_temp, -1.0, mst["u"])
            z_in = _dev.axpby(1.0, mst["z"], mst["sigma"], self._K(w))
            z_temp = self._h.fenchel_prox(z_in, sigma=mst["sigma"])
            mst["z"] = _dev.axpby(1 - rho, mst["z"], rho, z_temp)
        mst["u"] = _dev.axpby(1 - rho, mst["u"], rho, u_temp)

    def _set_step_sizes(self, tau, sigma, gamma):
        if not isinstance(self._K, pxa.LinOp):
            raise ValueError("Automatic selection of parameters is only supported in the case in which K is a linear operator. "
                             f"Got operator of type {self._K.__class__}.")
        tau = None if tau == 0 else tau
        sigma = None if sigma == 0 else sigma
        L = self._K_lipschitz
        if (tau is not None) and (sigma is None):
            assert 0 < tau <= 1 / gamma, "tau must be positive and smaller than 1/gamma."
            if _is_null(self._h):
                sigma = 0
            else:
                if math.isfinite(L()):
                    sigma = 1 / (tau * L() ** 2)
                else:
                    raise ValueError(_knorm_msg())
        elif (tau is None) and (sigma is not None):
            assert sigma > 0, f"sigma must be positive, got {sigma}."
            if _is_null(self._h):
                tau = 1 / gamma
            else:
                if math.isfinite(L()):
                    tau = min(1 / (sigma * L() ** 2), 1 / gamma)
                else:
                    raise ValueError(_knorm_msg())
        elif (tau is None) and (sigma is None):
            if self._beta > 0:
                if _is_null(self._h):
                    tau, sigma = 1 / gamma, 0
                else:
                    if math.isfinite(L()):
                        tau, sigma = self._optimize_step_sizes(gamma)
                    else:
                        raise ValueError(_knorm_msg())
            else:
                if _is_null(self._h):
                    tau, sigma = 1, 0
                else:
                    if math.isfinite(L()):
                        tau = sigma = 1 / L()
                    else:
                        raise ValueError(_knorm_msg())
        delta = 2 if self._beta == 0 else 2 - self._beta * tau / 2
        return pxrt.coerce(tau), pxrt.coerce(sigma), pxrt.coerce(delta)

    @pxrt.enforce_precision()
    def _optimize_step_sizes(self, gamma):
        """Same 2-variable LP as the reference (pds.py:831-864), solved with scipy.optimize.linprog."""
        from scipy.optimize import linprog

        c = np.array([-1, -1])
        A_ub = np.array([[1, 1], [1, 0]])
        b_ub = np.array([np.log(0.99) - 2 * np.log(self._K_lipschitz()), np.log(1 / gamma)])
        A_eq = np.array([[1, -1]])
        b_eq = np.array([0])
        result = linprog(c=c, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=b_eq, bounds=(None, None))
        if not result.success:
            warnings.warn("Automatic parameter selection has not converged.", UserWarning)
        return np.exp(result.x)


def ChambollePock(g=None, h=None, K=None, base=CondatVu, **kwargs):
    """Chambolle-Pock = base with f=None, beta=0 (pds.py:867-967)."""
    kwargs.update(log_var=kwargs.get("log_var", ("x", "z")))
    obj = base(f=None, g=g, h=h, K=K, beta=0, **kwargs)
    obj.__repr__ = lambda _: "ChambollePock"
    return obj


CP = ChambollePock


class LorisVerhoeven(PD3O):
    """PD3O with g=None (pds.py:970-1099)."""

    def __init__(self, f=None, h=None, K=None, beta=None, **kwargs):
        kwargs.update(log_var=kwargs.get("log_var", ("x", "z")))
        super().__init__(f=f, g=None, h=h, K=K, beta=beta, **kwargs)

    def _set_step_sizes(self, tau, sigma, gamma):
        tau, sigma, _ = super()._set_step_sizes(tau=tau, sigma=sigma, gamma=gamma)
        delta = 2 if (self._beta == 0 or isinstance(self._f, pxa.QuadraticFunc)) else 2 - self._beta / (2 * gamma)
        return pxrt.coerce(tau), pxrt.coerce(sigma), pxrt.coerce(delta)


LV = LorisVerhoeven


class DavisYin(PD3O):
    """PD3O with K = Identity and tau = 1/sigma (pds.py:1102-1226)."""

    def __init__(self, f, g=None, h=None, beta=None, **kwargs):
        kwargs.update(log_var=kwargs.get("log_var", ("x", "z")))
        super().__init__(f=f, g=g, h=h, K=None, beta=beta, **kwargs)

    def _set_step_sizes(self, tau, sigma, gamma):
        if tau is not None:
            assert 0 < tau <= 1 / gamma, "tau must be positive and smaller than 1/gamma."
        else:
            tau = 1.0 if self._beta == 0 else 1 / gamma
        delta = 2.0 if self._beta == 0 else 2 - self._beta * tau / 2
        return pxrt.coerce(tau), pxrt.coerce(1 / tau), pxrt.coerce(delta)


DY = DavisYin


def DouglasRachford(g=None, h=None, base=CondatVu, **kwargs):
    """Douglas-Rachford (pds.py:1229-1310)."""
    kwargs.update(log_var=kwargs.get("log_var", ("x", "z")))
    obj = base(f=None, g=g, h=h, K=None, beta=0, **kwargs)
    obj.__repr__ = lambda _: "DouglasRachford"

    def _set_step_sizes_custom(_, tau, sigma, gamma):
        tau = 1.0 if tau is None else tau
        return pxrt.coerce(tau), pxrt.coerce(1 / tau), pxrt.coerce(2.0)

    obj._set_step_sizes = types.MethodType(_set_step_sizes_custom, obj)
    return obj


DR = DouglasRachford


class ADMM(_PDS):
    """ADMM (pds.py:1313-1687): "prox" x-update when f is proximable and K is None, "cg" for a
    QuadraticFunc f with K given, or a user `solver` callable ("custom")."""

    def __init__(self, f=None, h=None, K=None, solver=None, solver_kwargs=None, **kwargs):
        from pyxu_amd.operator.linop import NullFunc, NullOp

        kwargs.update(log_var=kwargs.get("log_var", ("x", "u", "z")))
        x_update_solver = "custom"
        g = None
        if solver is None:
            if f is None:
                if h is None:
                    raise ValueError("Cannot minimize always-0 functional. At least one of Parameter[f, h] must be specified.")
                if K is None:
                    f = NullFunc(h.dim)
                else:
                    f = pxa.QuadraticFunc(shape=(1, h.dim), Q=NullOp(shape=(h.dim, h.dim)), c=NullFunc(dim=h.dim))
            if f.has(pxa.Property.PROXIMABLE) and K is None:
                x_update_solver = "prox"
                g = f
                f = None
            elif isinstance(f, pxa.QuadraticFunc):
                x_update_solver = "cg"
                self._K_gram = K.gram()
                warnings.warn("A sub-iterative conjugate gradient algorithm is used for the x-minimization step of ADMM. "
                              "This might be computationally expensive.", UserWarning)
            else:
                raise TypeError("Unsupported scenario: f must either be a ProxFunc (in which case K must be None), a "
                                "QuadraticFunc, or a solver must be provided for the x-minimization step of ADMM.")
        self._solver = solver
        self._x_update_solver = x_update_solver
        self._init_kwargs = solver_kwargs if solver_kwargs is not None else dict(show_progress=False)
        super().__init__(f=f, g=g, h=h, K=K, **kwargs)

    @pxrt.enforce_precision(i=("x0", "z0", "tau", "rho"), allow_None=True)
    def m_init(self, x0, z0=None, tau=None, rho=None, tuning_strategy=1, solver_kwargs=None, **kwargs):
        super().m_init(x0=x0, z0=z0, tau=tau, sigma=None, rho=rho, tuning_strategy=tuning_strategy)
        self._mstate["u"] = self._K(_dev.require(x0, "x0"))
        self._fit_kwargs = dict() if solver_kwargs is None else solver_kwargs

    def m_step(self):
        mst = self._mstate
        tau, rho = mst["tau"], mst["rho"]
        fast = self._l1_fast_path()
        if fast is not None:
            return self._m_step_l1(fast, tau, rho)
        mst["x"] = self._x_update(_dev.axpby(1.0, mst["u"], -1.0, mst["z"]), tau=tau)
        Kx = self._K(mst["x"])
        z_temp = _dev.lincomb3(1.0, mst["z"], 1.0, Kx, -1.0, mst["u"])
        if not _is_null(self._h):
            mst["u"] = self._h.prox(_dev.axpby(1.0, Kx, 1.0, z_temp), tau=tau)
        mst["z"] = _dev.lincomb3(1.0, z_temp, rho - 1, Kx, -(rho - 1), mst["u"])

    def _l1_fast_path(self):
        """(QuadraticFunc q, L1 scale or None) when the outer update can run as one kernel: the x-update is
        q.prox (CG on Q + I/tau), K = Id and h = lam ||.||_1 (lam = None: h = ||.||_1); else None."""
        if "_l1_fast" in self.__dict__:
            return self._l1_fast
        from pyxu_amd.abc.arithmetic import quadratic_prox_target
        from pyxu_amd.operator.func.norm import L1Norm
        from pyxu_amd.operator.linop import IdentityOp

        fast, h = None, self._h
        if self._x_update_solver == "prox" and type(self._K) is IdentityOp and not _is_null(h):
            qf = quadratic_prox_target(self._g)
            if type(h) is L1Norm:
                fast = None if qf is None else (qf, None)
            elif (qf is not None and h.has(pxa.Property.CAN_EVAL) and h._expr()[0] == "scale"
                  and type(h._op) is L1Norm):
                fast = (qf, h._cst)
        self._l1_fast = fast
        return fast

    def _m_step_l1(self, fast, tau, rho):
        """m_step for h = lam L1, K = Id and a CG x-update (pds.py:1606-1620): the outer update and the next
        x-update's right-hand side in one launch (pxa_admm_l1_update, same roundings as the chain of map
        launches of the general m_step), whose b / r0 / p0 / x0 planes the next CG solve starts from.  The
        first step (or one after the state was replaced) forms b the general way."""
        mst = self._mstate
        qf, cst = fast
        pre = self.__dict__.get("_l1_pre")
        if pre is not None and pre[0] is mst["u"] and pre[1] is mst["z"] and pre[2] == float(tau):
            x = qf._prox_solve(pre[3], tau, preset=pre[4:])
        else:
            x = self._x_update(_dev.axpby(1.0, mst["u"], -1.0, mst["z"]), tau=tau)
        _, c, _ = qf._quad_spec()
        thr = pxrt.coerce(tau) if cst is None else pxrt.coerce(pxrt.coerce(tau) * cst)  # ScaleRule -> L1Norm.prox
        u, z, b, r0, p0, x0 = _dev.admm_l1_update(x, mst["z"], mst["u"], qf._c_grad(c, x), rho - 1, thr, tau)
        # the next solve's ||r0||^2 and first operator pass go to the device now, ahead of the host's
        # bookkeeping between the two x-updates
        ahead = qf._prox_cg(tau)[0]._launch_start(r0, p0)
        mst["x"], mst["u"], mst["z"] = x, u, z
        self._l1_pre = (u, z, float(tau), b, x0, r0, p0) + (ahead if ahead is not None else ())

    def _x_update(self, arr, tau):
        if self._x_update_solver == "custom":
            return self._solver(arr, tau)
        if self._x_update_solver == "prox":
            return self._g.prox(arr, tau=tau)
        from pyxu_amd.opt.solver import CG

        # "cg": reads f._Q / f._c directly, as the reference does (pds.py:1645-1653)
        b = _dev.axpby(1 / tau, self._K.adjoint(arr), -1.0, self._f._c.grad(arr))
        A = self._f._Q + (1 / tau) * self._K_gram
        slvr = CG(A=A, **self._init_kwargs)
        slvr.fit(b=b, x0=_dev.copy(self._mstate["x"]), **self._fit_kwargs)
        return slvr.solution()

    def solution(self, which="primal"):
        data, _ = self.stats()
        if which == "primal":
            return data.get("x")
        if which == "primal_h":
            return data.get("u")
        if which == "dual":
            return _dev.div(data.get("z"), self._mstate["tau"])
        raise ValueError(f"Parameter which must be one of ['primal', 'primal_h', 'dual'] got: {which}.")

    def _set_step_sizes(self, tau, sigma, gamma):
        if tau is not None:
            assert tau > 0, f"Parameter tau must be positive, got {tau}."
        else:
            tau = 1.0
        return pxrt.coerce(tau), pxrt.coerce(1 / tau), pxrt.coerce(2.0)


class ForwardBackward(CondatVu):
    """Forward-backward splitting = CondatVu with h=None (pds.py:1690-1786)."""

    def __init__(self, f=None, g=None, beta=None, **kwargs):
        kwargs.update(log_var=kwargs.get("log_var", ("x",)))
        super().__init__(f=f, g=g, h=None, K=None, beta=beta, **kwargs)


FB = ForwardBackward


def ProximalPoint(g=None, base=CondatVu, **kwargs):
    """Proximal point = base with f=h=None (pds.py:1789-1862)."""
    kwargs.update(log_var=kwargs.get("log_var", ("x",)))
    obj = base(f=None, g=g, h=None, K=None, beta=None, **kwargs)
    obj.__repr__ = lambda _: "ProximalPoint"
    return obj


PP = ProximalPoint
