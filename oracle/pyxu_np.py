"""
NumPy restatement of Pyxu's proximal-splitting hot path (reference snapshot 2025-01-24).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Every function cites the reference
file:line it restates; paths are relative to ``/root/reference/src/pyxu``.  Arithmetic order
follows the reference's NumPy path term-for-term so that, in the same precision, results agree
bit-for-bit with the goldens recorded from the reference itself.
"""
import itertools
import math

import numpy as np

__all__ = [
    "gaussian_taps",
    "fd_taps",
    "canonical_stencil",
    "pad_apply",
    "pad_adjoint",
    "stencil_apply",
    "stencil_adjoint",
    "gradient_kernels",
    "gradient_apply",
    "gradient_adjoint",
    "diff_kernels",
    "divergence_apply",
    "divergence_adjoint",
    "hessian_components",
    "hessian_apply",
    "hessian_adjoint",
    "gaussian_kernel1d",
    "gd_kernels",
    "stack_apply",
    "stack_adjoint",
    "gd_gradient_comps",
    "gd_hessian_comps",
    "fd_hessian_comps",
    "unit_direction",
    "outer_triu",
    "contract_apply",
    "contract_adjoint",
    "laplacian_apply",
    "l1_prox",
    "l21_apply",
    "l21_prox",
    "fenchel_prox",
    "moreau_grad",
    "positive_orthant_prox",
    "relerror",
    "deblur_tv_grad",
    "pgd",
    "pd3o",
    "condat_vu",
    "pd3o_step_sizes",
    "condat_vu_step_sizes",
    "cg",
    "admm_dense_l1",
]


# ----------------------------------------------------------------------------- taps
def gaussian_taps(sigma: float, truncate: float = 3.0, dtype=np.float64):
    """Gaussian filter taps as built by ``Gaussian`` (operator/linop/filter.py:294-309).

    ``radius = int(truncate*sigma + 0.5)``; taps = ``flip(scipy.ndimage._filters._gaussian_kernel1d
    (sigma, 0, radius))`` (third-party, scipy>=1.11,<2, setup.cfg:32): ``phi = exp(-0.5/sigma^2 x^2)``
    on ``x in [-r, r]`` in float64, normalised by its sum; then cast to the runtime precision.
    Returns ``(taps, center)`` with ``center = radius``.  ``sigma == 0`` gives ``([1], 0)``.
    """
    if not sigma:
        return np.array([1], dtype=dtype), 0
    radius = int(truncate * float(sigma) + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x**2)
    phi = phi / phi.sum()
    return np.asarray(np.flip(phi), dtype=dtype), radius


def fd_taps(order: int = 1, scheme: str = "forward", accuracy: int = 1, sampling: float = 1.0, dtype=np.float64):
    """Finite-difference taps of ``_FiniteDifference`` (operator/linop/diff.py:213-258).

    Returns ``(ids, coefs, center)``; ``coefs`` computed in ``dtype`` exactly as the reference
    (vander system solved in the runtime precision, then ``/= sampling**order``).
    """
    if scheme == "central":
        n = 2 * ((order + 1) // 2) - 1 + accuracy
        ids = list(range(-(n // 2), n // 2 + 1))
    else:
        n = order + accuracy
        if scheme == "forward":
            ids = list(range(0, n))
        elif scheme == "backward":
            ids = list(range(-n + 1, 1))
        else:
            raise ValueError(scheme)
    mat = np.vander(np.array(ids), increasing=True).T.astype(dtype)
    vec = np.zeros(len(ids), dtype=dtype)
    vec[order] = math.factorial(order)
    coefs = np.linalg.solve(mat, vec)
    coefs /= sampling**order
    return ids, coefs, ids.index(0)


# ----------------------------------------------------------------------------- stencil
def canonical_stencil(arg_shape, kernel, center, dtype):
    """``Stencil._canonical_repr`` (operator/linop/stencil/stencil.py:497-538).

    Returns ``(kernels, centers)``: a list of rank-D arrays (one per separable axis, shape 1 on the
    other axes; or a single N-D kernel) and the matching list of rank-D centers.
    """
    D = len(arg_shape)
    if isinstance(kernel, np.ndarray):  # array input -> non-separable filter
        assert kernel.ndim == D
        return [np.asarray(kernel, dtype=dtype)], [np.array(center, dtype=int)]
    kernels, centers = [], []
    for i in range(D):
        sh = [1] * D
        sh[i] = -1
        kernels.append(np.asarray(kernel[i], dtype=dtype).reshape(sh))
        c = np.zeros(D, dtype=int)
        c[i] = center[i]
        centers.append(c)
    return kernels, centers


def _pad_width(kernels, centers, modes):
    """``Stencil._compute_pad_width`` (stencil.py:540-561)."""
    D = kernels[0].ndim
    out = []
    for i in range(D):
        if len(kernels) == 1:
            c, n = centers[0][i], kernels[0].shape[i]
        else:
            c, n = centers[i][i], kernels[i].size
        p = max(c, n - c - 1) if modes[i] == "constant" else n - 1
        out.append((int(p), int(p)))
    return tuple(out)


def pad_apply(x, arg_shape, pad_width, modes):
    """``Pad.apply`` (operator/linop/pad.py:235-306).  ``x``: (..., prod(arg_shape))."""
    sh = x.shape[:-1]
    D = len(arg_shape)
    a = x.reshape(*sh, *arg_shape)
    out = np.pad(a, ((0, 0),) * len(sh) + tuple(pad_width), mode="constant", constant_values=0)
    pad_shape = out.shape[len(sh):]
    for i in range(D, 0, -1):
        mode = modes[-i]
        lhs, rhs = pad_width[-i]
        N = pad_shape[-i]
        r = [slice(None)] * (len(sh) + D)
        w = [slice(None)] * (len(sh) + D)
        if mode == "constant":
            continue
        if mode == "wrap":
            r[-i], w[-i] = slice(N - rhs - lhs, N - rhs), slice(0, lhs)
            out[tuple(w)] = out[tuple(r)]
            r[-i], w[-i] = slice(lhs, lhs + rhs), slice(N - rhs, N)
            out[tuple(w)] = out[tuple(r)]
        elif mode == "reflect":
            r[-i], w[-i] = slice(2 * lhs, lhs, -1), slice(0, lhs)
            out[tuple(w)] = out[tuple(r)]
            r[-i], w[-i] = slice(N - rhs - 2, N - 2 * rhs - 2, -1), slice(N - rhs, N)
            out[tuple(w)] = out[tuple(r)]
        elif mode == "symmetric":
            r[-i], w[-i] = slice(2 * lhs - 1, lhs - 1, -1), slice(0, lhs)
            out[tuple(w)] = out[tuple(r)]
            r[-i], w[-i] = slice(N - rhs - 1, N - 2 * rhs - 1, -1), slice(N - rhs, N)
            out[tuple(w)] = out[tuple(r)]
        elif mode == "edge":
            if lhs > 0:
                r[-i], w[-i] = slice(lhs, lhs + 1), slice(0, lhs)
                out[tuple(w)] = out[tuple(r)]
            if rhs > 0:
                r[-i], w[-i] = slice(N - rhs - 1, N - rhs), slice(N - rhs, N)
                out[tuple(w)] = out[tuple(r)]
        else:
            raise ValueError(mode)
    return out.reshape(*sh, -1), pad_shape


def pad_adjoint(y, arg_shape, pad_width, modes):
    """``Pad.adjoint`` (operator/linop/pad.py:307-372).  ``y``: (..., prod(pad_shape))."""
    sh = y.shape[:-1]
    D = len(arg_shape)
    pad_shape = tuple(n + l + r for n, (l, r) in zip(arg_shape, pad_width))
    out = y.reshape(*sh, *pad_shape).copy()
    for i in range(1, D + 1):
        mode = modes[-i]
        lhs, rhs = pad_width[-i]
        N = pad_shape[-i]
        r = [slice(None)] * (len(sh) + D)
        w = [slice(None)] * (len(sh) + D)
        if mode == "constant":
            continue
        if mode == "wrap":
            r[-i], w[-i] = slice(0, lhs), slice(N - rhs - lhs, N - rhs)
            out[tuple(w)] += out[tuple(r)]
            r[-i], w[-i] = slice(N - rhs, N), slice(lhs, lhs + rhs)
            out[tuple(w)] += out[tuple(r)]
        elif mode == "reflect":
            if lhs > 0:
                r[-i], w[-i] = slice(lhs - 1, None, -1), slice(lhs + 1, 2 * lhs + 1)
                out[tuple(w)] += out[tuple(r)]
            r[-i], w[-i] = slice(N - 1, N - rhs - 1, -1), slice(N - 2 * rhs - 1, N - rhs - 1)
            out[tuple(w)] += out[tuple(r)]
        elif mode == "symmetric":
            if lhs > 0:
                r[-i], w[-i] = slice(lhs - 1, None, -1), slice(lhs, 2 * lhs)
                out[tuple(w)] += out[tuple(r)]
            r[-i], w[-i] = slice(N - 1, N - rhs - 1, -1), slice(N - 2 * rhs, N - rhs)
            out[tuple(w)] += out[tuple(r)]
        elif mode == "edge":
            if lhs > 0:
                r[-i], w[-i] = slice(0, lhs), slice(lhs, lhs + 1)
                out[tuple(w)] += out[tuple(r)].sum(axis=-i, keepdims=True)
            if rhs > 0:
                r[-i], w[-i] = slice(N - rhs, N), slice(N - rhs - 1, N - rhs)
                out[tuple(w)] += out[tuple(r)].sum(axis=-i, keepdims=True)
        else:
            raise ValueError(mode)
    sel = [slice(None)] * len(sh) + [slice(l, n - r) for n, (l, r) in zip(pad_shape, pad_width)]
    return out[tuple(sel)].reshape(*sh, -1)


def _correlate_zeroed(a, kernel, center):
    """One generated Numba stencil (operator/linop/stencil/_stencil.py:232-305) on a (S, *shape) array.

    ``out[s, i] = sum_q k[q] * a[s, i - c + q]`` on fully-supported indices, 0 elsewhere (numba
    ``@stencil`` constant mode, cval=0).  Taps with ``isclose(k, 0)`` are dropped, taps with
    ``isclose(k, 1)`` are applied without a multiply; terms are summed left-to-right in kernel
    ``itertools.product`` order (``_stencil.py:284-305``).
    """
    terms = []
    for idx in itertools.product(*map(range, kernel.shape)):
        cst = kernel[idx]
        if np.isclose(cst, 0):
            continue
        off = tuple(i - c for i, c in zip(idx, center))
        terms.append((off, None if np.isclose(cst, 1) else kernel.dtype.type(cst)))
    out = np.zeros_like(a)
    if not terms:
        return out
    offs = np.array([t[0] for t in terms]).reshape(len(terms), -1)
    lo = np.maximum(0, -offs.min(axis=0))
    hi = np.maximum(0, offs.max(axis=0))
    spatial = a.shape[1:]
    if not all(l < n - h for l, h, n in zip(lo, hi, spatial)):
        return out
    core = (slice(None),) + tuple(slice(l, n - h) for l, h, n in zip(lo, hi, spatial))
    acc = None
    for off, cst in terms:
        sl = (slice(None),) + tuple(slice(l + o, n - h + o) for o, l, h, n in zip(off, lo, hi, spatial))
        t = a[sl] if cst is None else cst * a[sl]
        acc = t.copy() if acc is None else acc + t
    out[core] = acc
    return out


def _chain(x, kernels, centers):
    """``Stencil._stencil_chain`` (stencil.py:608-627): apply stencils in sequence."""
    for k, c in zip(kernels, centers):
        x = _correlate_zeroed(x, k, c)
    return x


def _bw_equivalent(kernels, centers):
    """``Stencil._bw_equivalent`` (stencil.py:563-576): flipped kernels, centers ``k - c - 1``."""
    k_bw = [np.flip(k) for k in kernels]
    if len(kernels) == 1:
        c_bw = [np.array(kernels[0].shape) - centers[0] - 1]
    else:
        D = kernels[0].ndim
        c_bw = []
        for i in range(D):
            c = np.zeros(D, dtype=int)
            c[i] = kernels[i].shape[i] - centers[i][i] - 1
            c_bw.append(c)
    return k_bw, c_bw


def _canon_modes(mode, D):
    if isinstance(mode, str):
        mode = (mode,) * D
    return tuple(m.strip().lower() for m in mode)


def stencil_apply(x, arg_shape, kernel, center, mode="constant"):
    """``Stencil.apply`` = Trim o chain(st_fw) o Pad (stencil.py:441-450)."""
    arg_shape = tuple(arg_shape)
    kernels, centers = canonical_stencil(arg_shape, kernel, center, x.dtype)
    modes = _canon_modes(mode, len(arg_shape))
    pw = _pad_width(kernels, centers, modes)
    xp, pad_shape = pad_apply(x, arg_shape, pw, modes)
    y = _chain(xp.reshape(-1, *pad_shape), kernels, centers)
    core = (slice(None),) + tuple(slice(l, n - r) for n, (l, r) in zip(pad_shape, pw))
    return y[core].reshape(*x.shape[:-1], -1)


def stencil_adjoint(x, arg_shape, kernel, center, mode="constant"):
    """``Stencil.adjoint`` = Pad^T o chain(st_bw) o Trim^T (stencil.py:452-461)."""
    arg_shape = tuple(arg_shape)
    kernels, centers = canonical_stencil(arg_shape, kernel, center, x.dtype)
    modes = _canon_modes(mode, len(arg_shape))
    pw = _pad_width(kernels, centers, modes)
    pad_shape = tuple(n + l + r for n, (l, r) in zip(arg_shape, pw))
    S = int(np.prod(x.shape[:-1], dtype=int))
    z = np.zeros((S, *pad_shape), dtype=x.dtype)
    core = (slice(None),) + tuple(slice(l, n - r) for n, (l, r) in zip(pad_shape, pw))
    z[core] = x.reshape(S, *arg_shape)
    k_bw, c_bw = _bw_equivalent(kernels, centers)
    y = _chain(z, k_bw, c_bw)
    return pad_adjoint(y.reshape(*x.shape[:-1], -1), arg_shape, pw, modes)


# ----------------------------------------------------------------------------- gradient
def gradient_kernels(arg_shape, direction, scheme="forward", accuracy=1, sampling=1.0, dtype=np.float64):
    """Per-direction separable kernels of ``PartialDerivative.finite_difference``
    (diff.py:140-155 ``_create_kernel`` + :213-258): FD taps on ``direction``, ``[1]`` elsewhere."""
    D = len(arg_shape)
    samp = sampling if isinstance(sampling, (list, tuple)) else (sampling,) * D
    kernels = [np.array([1.0], dtype=dtype)] * D
    center = [0] * D
    _, coefs, c = fd_taps(1, scheme, accuracy, samp[direction], dtype)
    kernels = list(kernels)
    kernels[direction] = coefs
    center[direction] = c
    return kernels, center


def gradient_apply(x, arg_shape, directions=None, scheme="forward", accuracy=1, sampling=1.0, mode="constant"):
    """``Gradient.apply`` = vstack of PartialDerivatives (diff.py:1113-1265; blocks.py:660-679).

    Output (..., len(directions)*N), direction-major."""
    directions = tuple(range(len(arg_shape))) if directions is None else tuple(directions)
    parts = []
    for d in directions:
        k, c = gradient_kernels(arg_shape, d, scheme, accuracy, sampling, x.dtype)
        parts.append(stencil_apply(x, arg_shape, k, c, mode))
    return np.concatenate(parts, axis=-1)


def gradient_adjoint(z, arg_shape, directions=None, scheme="forward", accuracy=1, sampling=1.0, mode="constant"):
    """``Gradient.adjoint``: ``sum_d D_d^T z_d`` summed left-to-right (blocks.py:838-860)."""
    directions = tuple(range(len(arg_shape))) if directions is None else tuple(directions)
    N = int(np.prod(arg_shape))
    out = 0
    for j, d in enumerate(directions):
        k, c = gradient_kernels(arg_shape, d, scheme, accuracy, sampling, z.dtype)
        out = out + stencil_adjoint(z[..., j * N:(j + 1) * N], arg_shape, k, c, mode)
    return out


# ----------------------------------------------------------------------------- divergence / hessian / laplacian
def diff_kernels(arg_shape, order, scheme, accuracy=1, sampling=1.0, dtype=np.float64):
    """Separable kernels of ``PartialDerivative.finite_difference`` for a full per-axis ``order`` tuple
    (diff.py:140-155, 501-741): FD taps of ``order[a]`` on every axis with ``order[a] > 0``."""
    D = len(arg_shape)
    kernels, center = [np.array([1.0], dtype=dtype)] * D, [0] * D
    kernels = list(kernels)
    for a in range(D):
        if order[a] > 0:
            _, coefs, c = fd_taps(order[a], scheme, accuracy, sampling, dtype)
            kernels[a], center[a] = coefs, c
    return kernels, center


def divergence_apply(z, arg_shape, directions=None, scheme="central"):
    """``Divergence.apply`` = Sum(axis=0) o block_diag(Gradient(direction d)) with the scheme reversed
    (diff.py:1540-1589): forward <-> backward, central unchanged."""
    scheme = {"central": "central", "forward": "backward", "backward": "forward"}[scheme]
    directions = tuple(range(len(arg_shape))) if directions is None else tuple(directions)
    N = int(np.prod(arg_shape))
    out = 0
    for j, d in enumerate(directions):
        order = [0] * len(arg_shape)
        order[d] = 1
        k, c = diff_kernels(arg_shape, order, scheme, dtype=z.dtype)
        out = out + stencil_apply(z[..., j * N:(j + 1) * N], arg_shape, k, c)
    return out


def divergence_adjoint(x, arg_shape, directions=None, scheme="central"):
    scheme = {"central": "central", "forward": "backward", "backward": "forward"}[scheme]
    directions = tuple(range(len(arg_shape))) if directions is None else tuple(directions)
    parts = []
    for d in directions:
        order = [0] * len(arg_shape)
        order[d] = 1
        k, c = diff_kernels(arg_shape, order, scheme, dtype=x.dtype)
        parts.append(stencil_adjoint(x, arg_shape, k, c))
    return np.concatenate(parts, axis=-1)


def hessian_components(arg_shape, directions="all"):
    """(axes, order) pairs of ``_StackDiffHelper._check_directions_and_order`` (diff.py:1060-1111)."""
    import itertools

    D = len(arg_shape)
    if isinstance(directions, (int, np.integer)):
        directions = [[int(directions)] * 2]
    elif isinstance(directions, str):
        directions = [list(c) for c in itertools.combinations_with_replacement(range(D), 2)]
    elif not isinstance(directions[0], (list, tuple, np.ndarray)):
        directions = [list(directions)]
    comps = []
    for ds in directions:
        axes = sorted(set(int(v) for v in ds))
        o = 3 - len(axes)
        order = [0] * D
        for a in axes:
            order[a] = o
        comps.append((order, "central" if o == 2 else "forward"))
    return comps


def hessian_apply(x, arg_shape, directions="all"):
    """``Hessian.apply``: vstack of the second-order partial derivatives (diff.py:1591-1797)."""
    parts = []
    for order, scheme in hessian_components(arg_shape, directions):
        k, c = diff_kernels(arg_shape, order, scheme, dtype=x.dtype)
        parts.append(stencil_apply(x, arg_shape, k, c))
    return np.concatenate(parts, axis=-1)


def hessian_adjoint(z, arg_shape, directions="all"):
    N = int(np.prod(arg_shape))
    out = 0
    for j, (order, scheme) in enumerate(hessian_components(arg_shape, directions)):
        k, c = diff_kernels(arg_shape, order, scheme, dtype=z.dtype)
        out = out + stencil_adjoint(z[..., j * N:(j + 1) * N], arg_shape, k, c)
    return out


def laplacian_apply(x, arg_shape):
    """``Laplacian.apply`` = Sum(axis=0) o Hessian(diagonal directions) (diff.py:1923-1936)."""
    N = int(np.prod(arg_shape))
    h = hessian_apply(x, arg_shape, [[i, i] for i in range(len(arg_shape))])
    out = 0
    for j in range(len(arg_shape)):
        out = out + h[..., j * N:(j + 1) * N]
    return out


# ----------------------------------------------------------------------------- Gaussian derivatives, stacks
def gaussian_kernel1d(sigma, order, radius):
    """scipy.ndimage._filters._gaussian_kernel1d (scipy>=1.11,<2, called at diff.py:343 and filter.py:305):
    the float64 Gaussian on [-radius, radius] normalised by its sum; order n via the polynomial recursion."""
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x**2)
    phi = phi / phi.sum()
    if order == 0:
        return phi
    rng = np.arange(order + 1)
    q = np.zeros(order + 1)
    q[0] = 1
    Q = np.diag(rng[1:], 1) + np.diag(np.ones(order) / -(sigma * sigma), -1)
    for _ in range(order):
        q = Q.dot(q)
    return (x[:, None] ** rng).dot(q) * phi


def gd_kernels(arg_shape, order, sigma=1.0, truncate=3.0, sampling=1.0, dtype=np.float64):
    """``PartialDerivative.gaussian_derivative`` kernels (diff.py:885-919 -> _GaussianDerivative
    :264-350): on EVERY axis the flipped order-``order[a]`` Gaussian derivative of sigma / sampling pixels,
    radius int(truncate * sigma_pix + 0.5), divided by sampling**order[a]."""
    D = len(arg_shape)
    t = lambda v: tuple(v) if isinstance(v, (list, tuple)) else (v,) * D  # noqa: E731
    sigma, truncate, sampling = t(sigma), t(truncate), t(sampling)
    kernels, centers = [], []
    for a in range(D):
        s_pix = sigma[a] / sampling[a]
        r = int(truncate[a] * float(s_pix) + 0.5)
        k = np.flip(gaussian_kernel1d(s_pix, order[a], r)) / sampling[a] ** order[a]
        kernels.append(k.astype(dtype))
        centers.append(r)
    return kernels, centers


def stack_apply(x, arg_shape, comps):
    """vstack of stencils (blocks.py:660-679): comps = [(kernels, centers)], direction-major output."""
    return np.concatenate([stencil_apply(x, arg_shape, k, c) for k, c in comps], axis=-1)


def stack_adjoint(z, arg_shape, comps):
    """vstack adjoint: sum_j S_j^T z_j, left to right (blocks.py:838-860)."""
    N = int(np.prod(arg_shape))
    out = 0
    for j, (k, c) in enumerate(comps):
        out = out + stencil_adjoint(z[..., j * N:(j + 1) * N], arg_shape, k, c)
    return out


def gd_gradient_comps(arg_shape, dtype, directions=None, **gd):
    directions = tuple(range(len(arg_shape))) if directions is None else tuple(directions)
    comps = []
    for d in directions:
        order = [0] * len(arg_shape)
        order[d] = 1
        comps.append(gd_kernels(arg_shape, order, dtype=dtype, **gd))
    return comps


def gd_hessian_comps(arg_shape, dtype, directions="all", **gd):
    """Hessian(diff_method="gd") (diff.py:1591-1797): components of hessian_components(), Gaussian derivatives."""
    return [gd_kernels(arg_shape, order, dtype=dtype, **gd) for order, _ in hessian_components(arg_shape, directions)]


def fd_hessian_comps(arg_shape, dtype, directions="all"):
    return [diff_kernels(arg_shape, order, scheme, dtype=dtype) for order, scheme in hessian_components(arg_shape, directions)]


def unit_direction(d, dtype):
    """direction / ||direction||_2 over axis 0, in the direction dtype (diff.py:2012)."""
    d = np.asarray(d)
    return (d / np.linalg.norm(d, axis=0, keepdims=True)).astype(dtype)


def outer_triu(n1, n2):
    """Upper-triangular outer product, off-diagonal terms doubled, Hessian component order
    (diff.py:2020-2033)."""
    ndim = n1.shape[0]
    o = n1[:, None, ...] * n2[None, ...]
    if ndim == 1:
        return o.reshape(1, *o.shape[2:])
    o = o.reshape(ndim**2, *o.shape[2:])
    dummy = np.arange(ndim**2).reshape(ndim, ndim)
    o[dummy[np.triu_indices(ndim, k=1)].ravel()] *= 2
    return o[dummy[np.triu_indices(ndim, k=0)].ravel()]


def contract_apply(w, d, N):
    """Sum o DiagonalOp of the directional operators (diff.py:2049-2060): y_g = sum_j w[g, j] * d_{j mod K},
    each product rounded, summed left to right.  w: (G, J) or (G, J, N); d: (..., K*N)."""
    G, J = w.shape[:2]
    K = d.shape[-1] // N
    dd = d.reshape(*d.shape[:-1], K, N)
    out = []
    for g in range(G):
        acc = None
        for j in range(J):
            wj = w[g, j] if w.ndim == 2 else w[g, j].reshape(-1)
            t = wj * dd[..., j % K, :]
            acc = t if acc is None else acc + t
        out.append(acc)
    return np.concatenate(out, axis=-1)


def contract_adjoint(w, z, N, K):
    """Adjoint of contract_apply: t_k = sum_g sum_{j mod K = k} w[g, j] * z_g."""
    G, J = w.shape[:2]
    zz = z.reshape(*z.shape[:-1], G, N)
    out = []
    for k in range(K):
        acc = None
        for g in range(G):
            for j in range(k, J, K):
                wj = w[g, j] if w.ndim == 2 else w[g, j].reshape(-1)
                t = wj * zz[..., g, :]
                acc = t if acc is None else acc + t
        out.append(acc)
    return np.concatenate(out, axis=-1)


# ----------------------------------------------------------------------------- proxes
def l1_prox(x, tau):
    """``L1Norm.prox`` (operator/func/norm.py:47-52): ``fmax(0, |x| - tau) * sign(x)``."""
    tau = x.dtype.type(tau)
    y = np.fmax(0, np.fabs(x) - tau)
    y *= np.sign(x)
    return y


def l21_apply(x, arg_shape, l2_axis=(0,)):
    """``L21Norm.apply`` (norm.py:338-350)."""
    sh = x.shape[:-1]
    a = x.reshape(sh + tuple(arg_shape))
    l2 = tuple(len(sh) + np.array(l2_axis))
    n = np.sqrt((a**2).sum(axis=l2, keepdims=True))
    l1 = tuple(len(sh) + np.setdiff1d(np.arange(len(arg_shape)), l2_axis))
    return n.sum(axis=l1, keepdims=True).reshape(*sh, -1)


def l21_prox(x, tau, arg_shape, l2_axis=(0,)):
    """``L21Norm.prox`` (norm.py:352-364): ``x * (1 - tau / fmax(||x||_2, tau))``."""
    tau = x.dtype.type(tau)
    sh = x.shape[:-1]
    a = x.reshape(sh + tuple(arg_shape))
    l2 = tuple(len(sh) + np.array(l2_axis))
    n = (a**2).sum(axis=l2, keepdims=True)
    np.sqrt(n, out=n)
    out = a.copy()
    out *= 1 - tau / np.fmax(n, tau)
    return out.reshape(*sh, -1)


def fenchel_prox(prox, x, sigma):
    """``ProxFunc.fenchel_prox`` Moreau form (operator.py:940-944): ``x - sigma prox(x/sigma, 1/sigma)``."""
    sigma = x.dtype.type(sigma)
    out = prox(x / sigma, x.dtype.type(1 / sigma))
    out *= -sigma
    out += x
    return out


def moreau_grad(prox, x, mu):
    """``moreau_envelope`` gradient (operator.py:1053-1058): ``(x - prox(x, mu)) / mu``."""
    out = x.copy()
    out -= prox(x, mu)
    out /= mu
    return out


def positive_orthant_prox(x, tau=None):
    """``PositiveOrthant.prox`` (operator/func/indicator.py:204-206): ``clip(0, None)``."""
    return x.clip(0, None)


def relerror(x, x_prev):
    """``RelError`` value (opt/stop.py:365-378): per-row ``||x - x_prev|| / ||x_prev||``."""
    num = np.linalg.norm(x - x_prev, axis=-1, keepdims=True)
    den = np.linalg.norm(x_prev, axis=-1, keepdims=True)
    with np.errstate(all="ignore"):
        v = num / den
    v[np.isnan(v)] = 0
    return v


# ----------------------------------------------------------------------------- objective pieces
def deblur_tv_grad(x, blur, y, lam, mu, grad_kw, tv="l21"):
    """Gradient of ``F = 1/2||H . - y||^2 + lam * env_mu(L21 or L1) o Grad`` as the reference's rule
    stack computes it (arithmetic.py AddRule.grad :940-943, ChainRule.grad :1288-1316,
    ScaleRule.grad :209-213, ArgShiftRule.grad :648-652; norm.py:96-98; operator.py:1053-1058).

    ``blur``: dict(arg_shape, kernel, center, mode, convolve) for H.  ``lam == 0`` drops the TV term.
    """
    dt = x.dtype.type
    sh = blur["arg_shape"]
    fw, bw = (stencil_adjoint, stencil_apply) if blur.get("convolve") else (stencil_apply, stencil_adjoint)
    # data term: H^T( 0.5 * (2 * (Hx + (-y))) )
    t = fw(x, sh, blur["kernel"], blur["center"], blur.get("mode", "constant"))
    t = t.copy()
    t += -y
    g = 2 * t
    g *= 0.5
    out = bw(g, sh, blur["kernel"], blur["center"], blur.get("mode", "constant"))
    if lam:
        v = gradient_apply(x, **grad_kw)
        D = len(grad_kw.get("directions") or grad_kw["arg_shape"])
        if tv == "l21":
            prox = lambda a, t_: l21_prox(a, t_, (D, *grad_kw["arg_shape"]))
        else:
            prox = l1_prox
        q = moreau_grad(prox, v, mu)
        q *= lam
        out = out.copy()
        out += gradient_adjoint(q, **grad_kw)
    return out


# ----------------------------------------------------------------------------- solvers
def pgd(x0, grad, prox, tau, n_iter, d=75, acceleration=True, history=False, snap=None):
    """``PGD.m_init``/``m_step`` (opt/solver/pgd.py:129-191); returns ``(x, x_prev[, hist])``.

    ``grad(y)`` and ``prox(z, tau)`` are the composite callables; ``tau`` the (fp-coerced) step.
    ``snap``: optional dict whose keys are iteration counts k; snap[k] receives a copy of x after k steps.
    """
    dt = x0.dtype.type
    tau = dt(tau)
    x = x_prev = x0
    hist = []
    for k in range(n_iter):
        a = dt(k / (k + 1 + d)) if acceleration else dt(0)
        y = x - x_prev
        y *= a
        y += x
        z = grad(y).copy()
        z *= -tau
        z += y
        x_prev, x = x, prox(z, tau)
        if history:
            hist.append(relerror(x, x_prev))
        if snap is not None and (k + 1) in snap:
            snap[k + 1] = x.copy()
    return (x, x_prev, hist) if history else (x, x_prev)


def pd3o_step_sizes(beta, K_lipschitz, dtype):
    """``PD3O._set_step_sizes`` + ``_optimize_step_sizes`` for tau=sigma=None, beta>0, h given
    (pds.py:763-864).  The reference solves a 2-variable LP with scipy ``linprog``; we call the same
    LP so the step sizes are identical.  Returns ``(tau, sigma, delta, rho)`` coerced to ``dtype``."""
    from scipy.optimize import linprog

    dt = np.dtype(dtype).type
    gamma = dt(beta)
    L = dt(K_lipschitz)
    res = linprog(
        c=np.array([-1, -1]),
        A_ub=np.array([[1, 1], [1, 0]]),
        b_ub=np.array([np.log(0.99) - 2 * np.log(L), np.log(1 / gamma)]),
        A_eq=np.array([[1, -1]]),
        b_eq=np.array([0]),
        bounds=(None, None),
    )
    tau, sigma = np.exp(res.x).astype(dtype)
    delta = 2 if beta == 0 else 2 - dt(beta) * tau / 2
    return dt(tau), dt(sigma), dt(delta), dt(1.0)


def condat_vu_step_sizes(beta, K_lipschitz, dtype, quadratic_f=True):
    """``CondatVu._set_step_sizes`` for tau=sigma=None, beta>0, h given (pds.py:444-517)."""
    dt = np.dtype(dtype).type
    gamma = dt(beta)
    L = dt(K_lipschitz)
    tau = sigma = (1 / L**2) * ((-gamma / 2) + math.sqrt((gamma**2 / 4) + L**2))
    beta = dt(beta)
    delta = 2 if (beta == 0 or (quadratic_f and gamma <= beta)) else 2 - beta / (2 * gamma)
    return dt(tau), dt(sigma), dt(delta), dt(1.0)


def pd3o(x0, grad_f, prox_g, K, KT, fprox_h, tau, sigma, rho, n_iter, z0=None, u0=None, history=False, snap=None):
    """``PD3O.m_init``/``m_step`` (pds.py:722-761).  ``prox_g=None`` means NullFunc (identity prox).
    ``snap``: optional dict of iteration counts k -> (x, z) copies after k steps."""
    dt = x0.dtype.type
    tau, sigma, rho = dt(tau), dt(sigma), dt(rho)
    x = x0
    z = K(x0.copy()) if z0 is None else z0
    u = x0.copy() if u0 is None else u0
    hist = []
    for _ in range(n_iter):
        x_prev, z_prev = x, z
        t = u - tau * KT(z)
        x = t if prox_g is None else prox_g(t, tau)
        u_temp = x - tau * grad_f(x)
        z_temp = fprox_h(z + sigma * K(x + u_temp - u), sigma)
        z = (1 - rho) * z + rho * z_temp
        u = (1 - rho) * u + rho * u_temp
        if history:
            hist.append((relerror(x, x_prev), relerror(z, z_prev)))
        if snap is not None and (_ + 1) in snap:
            snap[_ + 1] = (x.copy(), z.copy())
    return (x, z, u, hist) if history else (x, z, u)


def condat_vu(x0, grad_f, prox_g, K, KT, fprox_h, tau, sigma, rho, n_iter, z0=None, history=False, snap=None):
    """``CondatVu.m_step`` (pds.py:429-442).  ``snap``: as in pd3o()."""
    dt = x0.dtype.type
    tau, sigma, rho = dt(tau), dt(sigma), dt(rho)
    x = x0
    z = K(x0.copy()) if z0 is None else z0
    hist = []
    for _ in range(n_iter):
        x_prev, z_prev = x, z
        t = x - tau * grad_f(x) - tau * KT(z)
        x_temp = t if prox_g is None else prox_g(t, tau)
        u = 2 * x_temp - x
        z_temp = fprox_h(z + sigma * K(u), sigma)
        z = rho * z_temp + (1 - rho) * z
        x = rho * x_temp + (1 - rho) * x
        if history:
            hist.append((relerror(x, x_prev), relerror(z, z_prev)))
        if snap is not None and (_ + 1) in snap:
            snap[_ + 1] = (x.copy(), z.copy())
    return (x, z, hist) if history else (x, z)


def cg(A, b, x0=None, eps=1e-4, max_iter=None, restart_rate=None):
    """``CG`` (opt/solver/cg.py:72-165) under its default stop ``AbsError(residual, 1e-4)``
    OR-ed with ``MaxIter`` (stop checked before each step, solver.py:588-652).  Returns ``(x, n_steps)``."""
    dt = b.dtype
    dim = b.shape[-1]
    restart_rate = dim if restart_rate is None else restart_rate
    x = np.zeros_like(b) if x0 is None else x0.copy()
    r = b.copy()
    r -= A(x)
    p = r.copy()
    max_iter = 2 * dim if max_iter is None else max_iter
    idx, n_stop = 0, 0
    eps_w = np.finfo(dt).eps
    while True:
        # stop criterion evaluated first (AbsError | MaxIter)
        n_stop += 1
        res = np.linalg.norm(r, axis=-1, keepdims=True)
        if np.all(res <= eps) or n_stop > max_iter:
            return x, idx
        idx += 1
        Ap = A(p)
        rr = np.linalg.norm(r, ord=2, axis=-1, keepdims=True) ** 2
        alpha = rr / (p * Ap).sum(axis=-1, keepdims=True)
        x += alpha * p
        if np.any(rr <= eps_w):
            r[:] = b
            r -= A(x)
        else:
            r -= alpha * Ap
        if idx % restart_rate == 0:
            beta = 0
            r[:] = b
            r -= A(x)
        else:
            beta = np.linalg.norm(r, ord=2, axis=-1, keepdims=True) ** 2 / rr
        p *= beta
        p += r


def admm_dense_l1(Kmat, y, lam, x0, tau, n_iter, rho=1.0, history=False):
    """ADMM "prox" x-update path (pds.py:1537-1660) for ``f = 1/2||K . - y||^2`` (QuadraticFunc
    through ChainRule, operator.py:1273-1291), ``h = lam*L1Norm``, ADMM's own K = Identity.

    x-update = QuadraticFunc.prox: CG on ``(K^T K + I/tau) x = arr/tau + K^T y``."""
    dt = x0.dtype.type
    tau, rho = dt(tau), dt(rho)
    KT_y = (Kmat.T @ y).astype(x0.dtype)

    def A(p):
        return (Kmat.T @ (Kmat @ p.T)).T.astype(p.dtype) + (1 / tau) * p

    x = x0
    u = x0.copy()
    z = np.zeros_like(x0)
    # m_init: z0 = K(x0) with ADMM-internal K = IdentityOp; u = K(x0)
    z = x0.copy()
    u = x0.copy()
    inner = []
    for _ in range(n_iter):
        arr = u - z
        b = arr.copy()
        b /= tau
        b -= -KT_y
        x, n = cg(A, b)
        inner.append(n)
        z_temp = z + x - u
        u = l1_prox(x + z_temp, tau * dt(lam))
        z = z_temp + (rho - 1) * (x - u)
    return (x, u, z, inner)
