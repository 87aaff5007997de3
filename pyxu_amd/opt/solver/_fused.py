"""
Pattern matcher: recognise the proximal-splitting problems that have a fused one-launch m_step.

The reference evaluates ``f.grad`` / ``g.prox`` by walking the arithmetic-rule tree
(abc/arithmetic.py) one NumPy pass per node.  For the deblurring objectives of BASELINE.json the
whole PGD iteration is a single HIP kernel (pxa_pgd_tv2d_step); this module extracts its
parameters from the operator tree (introspection fields ``_op/_cst/_lhs/_rhs`` set by the rules,
exactly the reference's embedding convention) and returns None when the tree does not match, in
which case the solver runs the generic (still all-HIP) rule-by-rule path.
"""
import warnings

import numpy as np

import pyxu_amd.abc as pxa
from pyxu_amd.operator.func.indicator import PositiveOrthant
from pyxu_amd.operator.func.norm import L1Norm, L21Norm, SquaredL2Norm
from pyxu_amd.operator.linop.diff import _DiffStack
from pyxu_amd.operator.linop.stencil import Stencil
from pyxu_amd.util import is_device_array

__all__ = ["match_pgd_deblur", "match_pds_deblur"]

MAX_R = 8


class FusedPathWarning(UserWarning):
    """The problem has the fused kernel's structure but a parameter outside its envelope: the solver
    runs the generic rule-by-rule HIP path (2-3x slower) instead."""


def _radius_ok(o):
    r = max(abs(v) for v in o)
    if r > MAX_R:
        warnings.warn(f"blur radius {r} > {MAX_R}: the fused one-launch step is not used; running the generic "
                      f"per-operator HIP path.", FusedPathWarning, stacklevel=4)
        return False
    return True


def _unscale(op):
    """Peel ScaleRule layers: returns (inner, total_scale)."""
    s = 1.0
    while hasattr(op, "_op") and hasattr(op, "_cst") and isinstance(getattr(op, "_cst"), float) and \
            op._expr()[0] == "scale":
        s *= op._cst
        op = op._op
    return op, s


def _core(op):
    """Undo asop()/squeeze() re-wrapping (a 1x1 operator is squeezed to a LinFunc shell)."""
    while hasattr(op, "_core"):
        op = op._core
    return op


def _data_term(f):
    """f = c * SquaredL2Norm.argshift(-y) o H  ->  (H, y, c) ; the reference's 1/2||H.-y||^2 has c=1/2."""
    if not (hasattr(f, "_lhs") and f._expr()[0] == "compose"):
        return None
    lhs, H = f._lhs, f._rhs
    lhs, c = _unscale(lhs)
    if not (hasattr(lhs, "_op") and lhs._expr()[0] == "argshift"):
        return None
    if not isinstance(lhs._op, SquaredL2Norm) or not hasattr(lhs._cst, "data_ptr"):
        return None
    if not np.isclose(c, 0.5):
        return None
    return _core(H), lhs._cst  # shift = -y


def _tv_term(t):
    """t = lam * env_mu(L21Norm((2, *sh))) o Grad  (or (lam*env) o Grad)  ->  (G, lam, mu, l21)."""
    t, s_out = _unscale(t)
    if not (hasattr(t, "_lhs") and t._expr()[0] == "compose"):
        return None
    env, G = t._lhs, _core(t._rhs)
    env, s_in = _unscale(env)
    if getattr(env, "_name", None) != "moreau_envelope" or not hasattr(env, "_inner"):
        return None
    inner = env._inner
    if not isinstance(inner, L21Norm) or tuple(inner._l2_axis.tolist()) != (0,):
        return None
    if not isinstance(G, _DiffStack) or G._fused is None:
        return None
    return G, s_out * s_in, float(env._mu), inner


def _stencil_axes(H, sh):
    """Separable constant-mode stencil on the trailing 2 axes (leading axes identity)."""
    if not isinstance(H, Stencil) or not H._separable:
        return None
    if any(m != "constant" for m in H._mode):
        return None
    D = len(sh)
    specs = H._st_fw
    for d in range(D - 2):
        if not specs[d].identity:
            return None
    taps = []
    for d in (D - 2, D - 1):
        st = specs[d]
        if st.identity:
            o, c = [0], [1.0]
        else:
            o, c = st.axis_taps()
        if not _radius_ok(o):
            return None
        taps.append((list(o), list(c)))
    return taps


def match_pgd_deblur(f, g, x0):
    """Return a dict of fused-kernel parameters or None."""
    if f is None:
        return None
    data, tv = f, None
    if hasattr(f, "_lhs") and f._expr()[0] == "add":
        data, tv = f._lhs, f._rhs
        if _data_term(data) is None:
            data, tv = tv, data
    dt = _data_term(data)
    if dt is None:
        return None
    H, shift = dt
    sh = getattr(H, "_arg_shape", None)
    if sh is None or len(sh) < 2:
        return None
    taps = _stencil_axes(H, sh)
    if taps is None:
        return None
    n0, n1 = sh[-2], sh[-1]
    B = int(np.prod(sh[:-2])) if len(sh) > 2 else 1
    lam, mu, h0, h1 = 0.0, 1.0, 1.0, 1.0
    if tv is not None:
        tvm = _tv_term(tv)
        if tvm is None:
            return None
        G, lam, mu, l21 = tvm
        if tuple(G.arg_shape) != tuple(sh):
            return None
        D = len(sh)
        if tuple(G._directions) != (D - 2, D - 1) or tuple(l21._arg_shape) != (2, *sh):
            return None
        hs = []
        for (d, o0, c0, o1, c1) in G._fused:
            if (o0, o1) != (0, 1) or not np.isclose(c0, -c1):
                return None
            hs.append(1.0 / c1)
        h0, h1 = hs
    # g
    if g is None or getattr(g, "_name", "") == "NullFunc":
        prox, pw = 0, 0.0
    else:
        gi, gs = _unscale(g)
        if isinstance(gi, PositiveOrthant) and gs > 0:
            prox, pw = 1, 0.0
        elif isinstance(gi, L1Norm) and gs > 0:
            prox, pw = 2, gs
        else:
            return None
    N = int(np.prod(sh))
    if x0.shape[-1] != N:
        return None
    rows = int(np.prod(x0.shape[:-1])) if x0.ndim > 1 else 1
    return dict(shift=shift, H=H, taps0=taps[0], taps1=taps[1], n0=n0, n1=n1, B=B, rows=rows, lam=lam, mu=mu, h0=h0,
                h1=h1, prox=prox, prox_scale=pw)


def _all_axis_taps(H, sh):
    """Per-axis taps of a separable constant-mode Stencil over ALL axes of sh (identity -> [1] at 0)."""
    if not isinstance(H, Stencil) or not H._separable or any(m != "constant" for m in H._mode):
        return None
    taps = []
    for st in H._st_fw:
        if st.identity:
            taps.append(([0], [1.0]))
            continue
        o, c = st.axis_taps()
        if not _radius_ok(o):
            return None
        taps.append((list(o), list(c)))
    return taps


def _g_prox(g):
    if g is None or getattr(g, "_name", "") == "NullFunc":
        return 0, 0.0
    gi, gs = _unscale(g)
    if isinstance(gi, PositiveOrthant) and gs > 0:
        return 1, 0.0
    if isinstance(gi, L1Norm) and gs > 0:
        return 2, gs
    return None


def match_pds_deblur(f, g, h, K, x0):
    """PD3O / CondatVu fused step (pxa_pds_step): f = 1/2||S.-y||^2 (S separable zero-boundary
    stencil, 2-D or 3-D), K = Gradient (all axes, or the trailing two of a batch-as-axis volume),
    h = lam L1 (anisotropic TV) or lam L21 over the directions (isotropic TV), g in {None,
    PositiveOrthant, lam L1}.  Returns the kernel parameters or None."""
    if f is None or h is None or K is None:
        return None
    dt = _data_term(f)
    if dt is None:
        return None
    H, shift = dt
    sh = tuple(getattr(H, "_arg_shape", ()) or ())
    if len(sh) not in (2, 3) or shift.ndim != 1:
        return None
    taps = _all_axis_taps(H, sh)
    if taps is None:
        return None
    G = _core(K)
    if not isinstance(G, _DiffStack) or G._fused is None or tuple(G.arg_shape) != sh:
        return None
    dirs = tuple(G._directions)
    if len(sh) == 2:
        if dirs != (0, 1):
            return None
        n0, (n1, n2), D = 1, sh, 2
        taps = [([0], [1.0])] + taps
        axes = (1, 2)
    else:
        if dirs == (0, 1, 2):
            D = 3
        elif dirs == (1, 2):
            D = 2
        else:
            return None
        n0, n1, n2 = sh
        axes = dirs
    c0, c1 = [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]
    for ax, (d, o0, a0, o1, a1) in zip(axes, G._fused):
        if (o0, o1) != (0, 1):
            return None
        c0[ax], c1[ax] = float(a0), float(a1)
    hi, lam = _unscale(h)
    if lam <= 0:
        return None
    N = int(np.prod(sh))
    if isinstance(hi, L1Norm) and hi.dim == D * N:
        h_kind = 0
    elif isinstance(hi, L21Norm) and tuple(hi._l2_axis.tolist()) == (0,) and tuple(hi._arg_shape) == (D, *sh):
        h_kind = 1
    else:
        return None
    gp = _g_prox(g)
    if gp is None:
        return None
    if x0.shape[-1] != N:
        return None
    rows = int(np.prod(x0.shape[:-1])) if x0.ndim > 1 else 1
    return dict(shift=shift, H=H, taps=taps, n0=n0, n1=n1, n2=n2, D=D, c0=c0, c1=c1, lam=float(lam), h_kind=h_kind,
                prox=gp[0], prox_scale=gp[1], rows=rows)
