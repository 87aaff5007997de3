"""
Differential operators (mirrors reference operator/linop/diff.py): PartialDerivative (finite and
Gaussian-derivative differences), Gradient, Jacobian, Divergence, Hessian, Laplacian and the directional
family (DirectionalDerivative / Gradient / Laplacian / Hessian).

``Gradient`` (diff.py:1113-1265) is a vstack of per-direction separable Stencils, output
direction-major ``(..., D*N)`` (diff.py:923-935, blocks.py:674-679).  When every direction is a
2-tap difference with zero boundary (the default forward scheme, and backward / accuracy-1 forms)
the whole stack runs as ONE kernel (pxa_gradient2 / pxa_gradient2_adjoint); otherwise each
direction runs its own Stencil writing straight into its output slice.
"""
import math

import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.operator.linop.stencil import Stencil

__all__ = ["PartialDerivative", "Gradient", "Jacobian", "Hessian", "Laplacian", "Divergence", "DirectionalDerivative",
           "DirectionalGradient", "DirectionalLaplacian", "DirectionalHessian", "fd_coefficients", "gd_coefficients"]


def fd_coefficients(order, scheme, accuracy, sampling, dtype):
    """_FiniteDifference._compute_ids/_compute_coefficients (diff.py:213-245), in `dtype`."""
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
            raise ValueError(f"Incorrect value for variable 'type'. 'type' should be ['forward', 'backward', 'central'], but got {scheme}.")
    mat = np.vander(np.array(ids), increasing=True).T.astype(dtype)
    vec = np.zeros(len(ids), dtype=dtype)
    vec[order] = math.factorial(order)
    coefs = np.linalg.solve(mat, vec)
    coefs /= sampling**order
    return ids, coefs, ids.index(0)


def gd_coefficients(order, sigma, truncate, sampling):
    """_GaussianDerivative._fill_coefs (diff.py:330-349): the order-`order` derivative of a Gaussian of
    standard deviation sigma / sampling pixels, truncated at `truncate` deviations, flipped for correlation,
    divided by sampling**order (float64; cast to the runtime precision by Stencil)."""
    from pyxu_amd.operator.linop.filter import gaussian_kernel1d

    sigma_pix = sigma / sampling
    radius = int(truncate * float(sigma_pix) + 0.5)
    coefs = np.flip(gaussian_kernel1d(sigma_pix, order, radius)) / sampling**order
    return list(range(-radius, radius + 1)), coefs, radius


def _tuple(v, n):
    if isinstance(v, (list, tuple)):
        return tuple(v) if len(v) == n else tuple(v) * (n // len(v) if len(v) == 1 else 1)
    return (v,) * n


class PartialDerivative:
    """Factory namespace (diff.py:446-899)."""

    @staticmethod
    def finite_difference(arg_shape, order, scheme="forward", axes=None, accuracy=1, mode="constant", gpu=True,
                          dtype=None, sampling=1):
        arg_shape = tuple(arg_shape)
        D = len(arg_shape)
        dtype = pxrt.getPrecision().value if dtype is None else dtype
        order = _tuple(order, 1) if not isinstance(order, (list, tuple)) else tuple(order)
        if len(order) != D:
            assert axes is not None, "If `order` is not a tuple with size of arg_shape, then `axes` must be specified."
            axes = _tuple(axes, len(order))
            full = [0] * D
            for o, a in zip(order, axes):
                full[a] = o
            order = tuple(full)
        scheme, accuracy, sampling = _tuple(scheme, D), _tuple(accuracy, D), _tuple(sampling, D)
        kernel = [np.array([1.0], dtype=dtype) for _ in range(D)]
        center = [0] * D
        for ax in range(D):
            if order[ax] > 0:
                _, coefs, c = fd_coefficients(order[ax], scheme[ax], accuracy[ax], sampling[ax], dtype)
                kernel[ax] = np.asarray(coefs, dtype=dtype)
                center[ax] = c
        op = Stencil(arg_shape=arg_shape, kernel=kernel, center=center, mode=mode)
        op._name = "PartialDerivative"
        op.meta = dict(sampling=sampling, scheme=scheme, accuracy=accuracy)
        return op

    @staticmethod
    def gaussian_derivative(arg_shape, order, sigma=1.0, truncate=3.0, mode="constant", gpu=True, dtype=None,
                            sampling=1):
        """Gaussian-derivative partial derivative (diff.py:762-919): EVERY axis is filtered by the
        derivative of a Gaussian of its order (order 0 = Gaussian smoothing), as one separable Stencil."""
        arg_shape = tuple(arg_shape)
        D = len(arg_shape)
        dtype = pxrt.getPrecision().value if dtype is None else dtype
        order = tuple(order)
        assert len(order) == D, "`order` must have one entry per axis of `arg_shape`"
        assert all(o >= 0 for o in order), "Order must be positive"
        sigma, truncate, sampling = _tuple(sigma, D), _tuple(truncate, D), _tuple(sampling, D)
        assert all(v >= 0 for v in sigma), "Sigma must be strictly positive"
        assert all(v > 0 for v in truncate), "Truncate must be strictly positive"
        assert all(v > 0 for v in sampling), "Sampling must be strictly positive"
        kernel, center = [], []
        for ax in range(D):
            _, coefs, c = gd_coefficients(order[ax], sigma[ax], truncate[ax], sampling[ax])
            kernel.append(np.asarray(coefs, dtype=dtype))
            center.append(c)
        op = Stencil(arg_shape=arg_shape, kernel=kernel, center=center, mode=mode)
        op._name = "PartialDerivative"
        op.meta = dict(sampling=sampling, sigma=sigma, truncate=truncate)
        return op


class _DiffStack(pxa.LinOp):
    """vstack of per-direction PartialDerivative Stencils (blocks.py vstack semantics)."""

    def __init__(self, arg_shape, stencils, directions):
        N = int(np.prod(arg_shape))
        super().__init__(shape=(len(stencils) * N, N))
        self.arg_shape = tuple(arg_shape)
        self._stencils = stencils
        self._directions = tuple(directions)
        self._N = N
        # 2-tap zero-boundary form for the fused kernel, per direction
        self._fused = None
        if all(all(m == "constant" for m in st._mode) for st in stencils):
            spec = []
            for d, st in zip(directions, stencils):
                if not st._separable:
                    spec = None
                    break
                fw = st._st_fw[d]
                others_identity = all(s.identity for i, s in enumerate(st._st_fw) if i != d)
                if not others_identity or len(fw.taps) != 2:
                    spec = None
                    break
                (o0, c0), (o1, c1) = [(t[0][d], t[1]) for t in fw.taps]
                spec.append((d, o0, c0, o1, c1))
            self._fused = spec
        L2 = sum(float(st.lipschitz) ** 2 for st in stencils)
        self.lipschitz = np.sqrt(L2)

    def unravel(self, arr):
        return arr.reshape(*arr.shape[:-1], -1, *self.arg_shape)

    def ravel(self, arr):
        return arr.reshape(*arr.shape[: -1 - len(self.arg_shape)], -1)

    def _stack(self, arr):
        sh = arr.shape[:-1]
        return sh, (int(np.prod(sh)) if len(sh) else 1)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        sh, S = self._stack(x)
        N, K = self._N, len(self._stencils)
        if self._fused is not None:
            d, o0, c0, o1, c1 = zip(*self._fused)
            g = _dev.gradient2(x, S, self.arg_shape, d, o0, c0, o1, c1, adjoint=False)
            return g.reshape(*sh, K * N)
        out = _dev.empty((S, K * N), x)
        for k, st in enumerate(self._stencils):
            out[:, k * N:(k + 1) * N] = st.apply(x.reshape(S, N))
        return out.reshape(*sh, K * N)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        z = _dev.require(arr)
        sh, S = self._stack(z)
        N, K = self._N, len(self._stencils)
        if self._fused is not None:
            d, o0, c0, o1, c1 = zip(*self._fused)
            x = _dev.gradient2(z, S, self.arg_shape, d, o0, c0, o1, c1, adjoint=True)
            return x.reshape(*sh, N)
        z2 = z.reshape(S, K * N)
        out = None
        for k, st in enumerate(self._stencils):
            part = st.adjoint(z2[:, k * N:(k + 1) * N].contiguous())
            out = part if out is None else _dev.axpby(1.0, out, 1.0, part, out=out)
        return out.reshape(*sh, N)

    def visualize(self):
        return "\n".join(f"\nDirection {d} \n" + st.visualize() for d, st in zip(self._directions, self._stencils))


def _gd_stencil(arg_shape, order, diff_kwargs, mode, dtype):
    """PartialDerivative.gaussian_derivative with Gradient / Hessian's `sigma`, `truncate`, `sampling`
    keywords (diff.py:1148-1157: defaults 1.0, 3.0, 1.0)."""
    return PartialDerivative.gaussian_derivative(arg_shape=arg_shape, order=tuple(order),
                                                 sigma=diff_kwargs.get("sigma", 1.0),
                                                 truncate=diff_kwargs.get("truncate", 3.0), mode=mode, dtype=dtype,
                                                 sampling=diff_kwargs.get("sampling", 1.0))


def _check_method(diff_method):
    if diff_method not in ("fd", "gd"):
        raise NotImplementedError(f"diff_method must be 'fd' or 'gd', got {diff_method!r}.")


def Gradient(arg_shape, directions=None, diff_method="fd", mode="constant", gpu=True, dtype=None, parallel=False,
             **diff_kwargs):
    """Gradient operator (diff.py:1113-1265); diff_method "fd" (finite differences) or "gd" (Gaussian
    derivatives: axis d differentiated, every other axis smoothed)."""
    _check_method(diff_method)
    arg_shape = tuple(arg_shape)
    D = len(arg_shape)
    directions = tuple(range(D)) if directions is None else tuple(np.atleast_1d(directions).tolist())
    scheme = diff_kwargs.get("scheme", "forward")
    accuracy = diff_kwargs.get("accuracy", 1)
    sampling = diff_kwargs.get("sampling", 1.0)
    mode = (mode,) * D if isinstance(mode, str) else tuple(mode)
    if len(mode) == 1:
        mode = mode * D
    samp = _tuple(sampling, D)
    sch = _tuple(scheme, D)
    acc = _tuple(accuracy, D)
    stencils = []
    for d in directions:
        order = [0] * D
        order[d] = 1
        if diff_method == "gd":
            stencils.append(_gd_stencil(arg_shape, order, diff_kwargs, mode, dtype))
        else:
            stencils.append(
                PartialDerivative.finite_difference(arg_shape=arg_shape, order=tuple(order), scheme=sch, accuracy=acc,
                                                    mode=mode, dtype=dtype, sampling=samp)
            )
    op = _DiffStack(arg_shape, stencils, directions)
    op._name = "Gradient"
    op.meta = dict(sampling=samp, scheme=sch, accuracy=acc) if diff_method == "fd" else \
        dict(sampling=samp, sigma=_tuple(diff_kwargs.get("sigma", 1.0), D), truncate=_tuple(diff_kwargs.get("truncate", 3.0), D))
    return op


class _Jacobian(pxa.LinOp):
    """block_diag of `n_channels` Gradients (diff.py:1268-1416): (..., C*N) -> (..., C*D*N), channel-major;
    every channel runs through the one gradient launch as a stack row."""

    def __init__(self, grad, n_channels):
        N, K, C = grad._N, len(grad._stencils), int(n_channels)
        super().__init__(shape=(C * K * N, C * N))
        self._grad, self._C, self._N, self._K = grad, C, N, K
        self.arg_shape = (K, *grad.arg_shape)
        self.lipschitz = float(grad.lipschitz)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        sh = x.shape[:-1]
        return self._grad.apply(x.reshape(*sh, self._C, self._N)).reshape(*sh, self._C * self._K * self._N)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        z = _dev.require(arr)
        sh = z.shape[:-1]
        return self._grad.adjoint(z.reshape(*sh, self._C, self._K * self._N)).reshape(*sh, self._C * self._N)

    def unravel(self, arr):
        return arr.reshape(*arr.shape[:-1], -1, *self.arg_shape)

    def ravel(self, arr):
        return arr.reshape(*arr.shape[: -1 - len(self.arg_shape)], -1)


def Jacobian(arg_shape, n_channels, directions=None, diff_method="fd", mode="constant", gpu=True, dtype=None,
             parallel=False, **diff_kwargs):
    """Jacobian of a multi-channel signal (diff.py:1268-1416): the Gradient of each of the `n_channels`
    channels, stacked channel-major."""
    grad = Gradient(arg_shape=arg_shape, directions=directions, diff_method=diff_method, mode=mode, gpu=gpu,
                    dtype=dtype, parallel=parallel, **diff_kwargs)
    if n_channels <= 1:
        grad._name = "Jacobian"
        return grad
    op = _Jacobian(grad, n_channels)
    op._name = "Jacobian"
    return op


def _fd_stencil(arg_shape, order, scheme, accuracy, mode, dtype, sampling):
    return PartialDerivative.finite_difference(arg_shape=arg_shape, order=tuple(order), scheme=scheme, accuracy=accuracy,
                                               mode=mode, dtype=dtype, sampling=sampling)


class _Divergence(pxa.LinOp):
    """Sum(axis=0) o block_diag(partial derivatives) (diff.py:1576-1589): (..., K*N) -> (..., N)."""

    def __init__(self, arg_shape, stencils):
        N = int(np.prod(arg_shape))
        super().__init__(shape=(N, len(stencils) * N))
        self.arg_shape = tuple(arg_shape)
        self._stencils = stencils
        self._N = N
        self.lipschitz = float(np.sqrt(len(stencils)) * max(float(st.lipschitz) for st in stencils))

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        z = _dev.require(arr)
        sh, N, K = z.shape[:-1], self._N, len(self._stencils)
        z2 = z.reshape(-1, K, N)
        out = None
        for k, st in enumerate(self._stencils):
            part = st.apply(z2[:, k].contiguous())
            out = part if out is None else _dev.axpby(1.0, out, 1.0, part, out=out)  # sum over axis 0, in order
        return out.reshape(*sh, N)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        x = _dev.require(arr)
        sh, N, K = x.shape[:-1], self._N, len(self._stencils)
        x2 = x.reshape(-1, N)
        out = _dev.empty((x2.shape[0], K, N), x2)
        for k, st in enumerate(self._stencils):
            out[:, k] = st.adjoint(x2)
        return out.reshape(*sh, K * N)

    def unravel(self, arr):
        return arr.reshape(*arr.shape[:-1], *self.arg_shape)

    def ravel(self, arr):
        return arr.reshape(*arr.shape[: -len(self.arg_shape)], -1)


class _StencilSum(pxa.SquareOp):
    """Sum(axis=0) o vstack(stencils) (Laplacian, diff.py:1923-1936): (..., N) -> (..., N)."""

    def __init__(self, arg_shape, stencils):
        N = int(np.prod(arg_shape))
        super().__init__(shape=(N, N))
        self.arg_shape = tuple(arg_shape)
        self._stencils = stencils
        L2 = sum(float(st.lipschitz) ** 2 for st in stencils)
        self.lipschitz = float(np.sqrt(len(stencils)) * np.sqrt(L2))

    def _sum(self, arr, adjoint):
        x = _dev.require(arr)
        out = None
        for st in self._stencils:
            part = st.adjoint(x) if adjoint else st.apply(x)
            out = part if out is None else _dev.axpby(1.0, out, 1.0, part, out=out)
        return out

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        return self._sum(arr, adjoint=False)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        return self._sum(arr, adjoint=True)

    def unravel(self, arr):
        return arr.reshape(*arr.shape[:-1], *self.arg_shape)

    def ravel(self, arr):
        return arr.reshape(*arr.shape[: -len(self.arg_shape)], -1)


def _hessian_directions(arg_shape, directions):
    """_StackDiffHelper._check_directions_and_order (diff.py:1060-1111): canonical (axes, order) pairs."""
    import itertools

    D = len(arg_shape)

    def _check(ds):
        assert all(0 <= d <= D - 1 for d in ds), "Direction values must be between 0 and the number of dimensions in `arg_shape`."

    if isinstance(directions, (int, np.integer)):
        directions = ([int(directions), int(directions)],)
        _check(directions[0])
    elif isinstance(directions, str):
        assert directions == "all", "Value for `directions` not implemented. The accepted directions types are int, tuple or a str with the value `all`."
        directions = tuple(list(c) for c in itertools.combinations_with_replacement(range(D), 2))
    elif not isinstance(directions[0], (list, tuple, np.ndarray)):
        assert len(directions) == 2, "If `directions` is a tuple, it should contain two elements, corresponding to the i-th an j-th elements (dx_i and dx_j)"
        directions = (list(directions),)
        _check(directions[0])
    else:
        for ds in directions:
            _check(ds)
    axes = [sorted(set(int(v) for v in ds)) for ds in directions]
    order = [3 - len(a) for a in axes]
    return axes, order


def Hessian(arg_shape, directions="all", diff_method="fd", mode="constant", gpu=True, dtype=None, parallel=False,
            **diff_kwargs):
    """Hessian (diff.py:1591-1797): vstack of second-order partial derivatives, upper triangle for "all".
    Diagonal components default to the central scheme, off-diagonal ones to `scheme` (forward)."""
    _check_method(diff_method)
    arg_shape = tuple(arg_shape)
    D = len(arg_shape)
    axes, order = _hessian_directions(arg_shape, directions)
    user_scheme = diff_kwargs.get("scheme", None)
    accuracy = diff_kwargs.get("accuracy", 1)
    sampling = diff_kwargs.get("sampling", 1.0)
    stencils = []
    for ax, o in zip(axes, order):
        full = [0] * D
        for a in ax:
            full[a] = o
        if diff_method == "gd":
            stencils.append(_gd_stencil(arg_shape, full, diff_kwargs, mode, dtype))
            continue
        scheme = user_scheme if user_scheme is not None else ("central" if o == 2 else "forward")
        stencils.append(_fd_stencil(arg_shape, full, _tuple(scheme, D) if isinstance(scheme, str) else scheme,
                                    _tuple(accuracy, D), mode, dtype, _tuple(sampling, D)))
    op = _DiffStack(arg_shape, stencils, [a[0] for a in axes])
    op._name = "Hessian"
    return op


def Laplacian(arg_shape, directions=None, diff_method="fd", mode="constant", gpu=True, dtype=None, parallel=False,
              **diff_kwargs):
    """Laplacian (diff.py:1799-1936): sum of the diagonal Hessian components (central scheme)."""
    arg_shape = tuple(arg_shape)
    D = len(arg_shape)
    directions = tuple(range(D)) if directions is None else tuple(np.atleast_1d(directions).tolist())
    H = Hessian(arg_shape, directions=[(i, i) for i in range(D) if i in directions], diff_method=diff_method,
                mode=mode, gpu=gpu, dtype=dtype, parallel=parallel, **diff_kwargs)
    op = _StencilSum(arg_shape, H._stencils)
    op._name = "Laplacian"
    return op


def Divergence(arg_shape, directions=None, diff_method="fd", mode="constant", gpu=True, dtype=None, parallel=False,
               **diff_kwargs):
    """Divergence (diff.py:1418-1589): Sum(axis=0) o block_diag of per-direction first derivatives,
    with the finite-difference scheme reversed (forward <-> backward; central stays, the default)."""
    _check_method(diff_method)
    arg_shape = tuple(arg_shape)
    D = len(arg_shape)
    change = {"central": "central", "forward": "backward", "backward": "forward"}
    scheme = diff_kwargs.get("scheme", "central")
    scheme = change[scheme] if isinstance(scheme, str) else [change[s] for s in scheme]
    accuracy = diff_kwargs.get("accuracy", 1)
    sampling = diff_kwargs.get("sampling", 1.0)
    directions = tuple(range(D)) if directions is None else tuple(np.atleast_1d(directions).tolist())
    stencils = []
    for d in directions:
        order = [0] * D
        order[d] = 1
        if diff_method == "gd":
            stencils.append(_gd_stencil(arg_shape, order, diff_kwargs, mode, dtype))
            continue
        stencils.append(_fd_stencil(arg_shape, order, _tuple(scheme, D) if isinstance(scheme, str) else tuple(scheme),
                                    _tuple(accuracy, D), mode, dtype, _tuple(sampling, D)))
    op = _Divergence(arg_shape, stencils)
    op._name = "Divergence"
    return op


# ------------------------------------------------------------------ directional family (diff.py:1938-2759)
def _unit(direction, xp_dtype):
    """direction / ||direction||_2 over axis 0, in the direction's dtype (diff.py:2012, 2121, 2268, 2433)."""
    d = np.asarray(direction)
    return (d / np.linalg.norm(d, axis=0, keepdims=True)).astype(xp_dtype)


def _outer_triu(n1, n2):
    """Upper-triangular outer product of two unit directions with the off-diagonal terms doubled, in the
    Hessian's component order (diff.py:2020-2033)."""
    ndim = n1.shape[0]
    o = n1[:, None, ...] * n2[None, ...]
    if ndim == 1:
        return o.reshape(1, *o.shape[2:])
    o = o.reshape(ndim**2, *o.shape[2:])
    dummy = np.arange(ndim**2).reshape(ndim, ndim)
    o[dummy[np.triu_indices(ndim, k=1)].ravel()] *= 2
    return o[dummy[np.triu_indices(ndim, k=0)].ravel()]


class _Directional(pxa.LinOp):
    """Sum o DiagonalOp o diff (the directional operators of diff.py:1938-2759) as the derivative stack
    `diff` (Gradient or Hessian: K components) followed by ONE contraction launch (pxa_dir_contract):
    output group g = sum_j w[g, j] * diff_{j mod K}.  w: host (G, J) or (G, J, *arg_shape) weights."""

    def __init__(self, diff, w, name):
        w = np.asarray(w)
        G, J = w.shape[0], w.shape[1]
        N, K = diff._N, len(diff._stencils)
        assert J % K == 0
        per_pixel = w.ndim > 2
        super().__init__(shape=(G * N, N))
        self._diff, self._G, self._J, self._K, self._N = diff, G, J, K, N
        self.arg_shape = diff.arg_shape
        self._wp = 1 if per_pixel else 0
        from pyxu_amd.util import to_device

        self._w_host = np.ascontiguousarray(w.reshape(G, J, N) if per_pixel else w)
        self._w = to_device(self._w_host.reshape(-1))
        self._name = name
        self.lipschitz = self._chain_lipschitz(self._w_host, G, J, K, float(diff.lipschitz))

    @staticmethod
    def _chain_lipschitz(w, G, J, K, L_diff):
        """The Lipschitz constant the reference's ``Sum * DiagonalOp * diff`` chain carries (ChainRule:
        product of the factors' constants, arithmetic.py:1190-1204, evaluated left to right):
          * Sum over the J summed components: sqrt(J) (reduce.py:103-106);
          * the diagonal part: one DiagonalOp per (group g, run of K consecutive terms) -- max|w|, or 0 / 1
            when the weights are allclose to 0 / 1 (NullOp / IdentityOp, base.py:236-243, 330) -- stacked
            vertically: sqrt(sum L_b^2), or sqrt(max L_b^2) when only the first block is non-zero
            (blocks.py:684-708); a single block is the DiagonalOp itself (DirectionalDerivative);
          * L(diff).
        With J == 1 the reference's Sum is square and the composition loses its constant (inf): kept."""
        if J == 1:
            return float("inf")
        Ls = []
        for g in range(G):
            for c in range(J // K):
                blk = w[g, c * K:(c + 1) * K]
                if np.allclose(blk, 0):
                    Ls.append(0.0)
                elif np.allclose(blk, 1):
                    Ls.append(1.0)
                else:
                    Ls.append(float(np.abs(blk).max()))
        if len(Ls) == 1:
            L_dop = Ls[0]
        else:
            sq = np.array(Ls) ** 2
            L_dop = float(np.sqrt(sq.max() if np.allclose(sq.sum(), sq[0]) else sq.sum()))
        return float(np.sqrt(J)) * L_dop * L_diff

    def _weights(self, x):
        w = self._w
        return w if w.dtype == x.dtype else _dev.cast(w, x)

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        x = _dev.require(arr)
        sh = x.shape[:-1]
        S = int(np.prod(sh)) if len(sh) else 1
        d = self._diff.apply(x.reshape(S, self._N))
        y = _dev.dir_contract(self._weights(x), self._wp, d, S, self._G, self._J, self._K, self._N)
        return y.reshape(*sh, self._G * self._N)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        z = _dev.require(arr)
        sh = z.shape[:-1]
        S = int(np.prod(sh)) if len(sh) else 1
        t = _dev.dir_contract(self._weights(z), self._wp, z.reshape(S, self._G * self._N), S, self._G, self._J, self._K,
                              self._N, adjoint=True)
        return self._diff.adjoint(t.reshape(S, self._K * self._N)).reshape(*sh, self._N)

    def unravel(self, arr):
        return arr.reshape(*arr.shape[:-1], *self.arg_shape) if self._G == 1 else \
            arr.reshape(*arr.shape[:-1], self._G, *self.arg_shape)

    def ravel(self, arr):
        n = len(self.arg_shape) + (0 if self._G == 1 else 1)
        return arr.reshape(*arr.shape[:-n], -1)


def _dir_dtype(d):
    d = d[0] if isinstance(d, (list, tuple)) else d
    return np.asarray(d.cpu() if hasattr(d, "cpu") else d).dtype


def _host(d):
    return np.asarray(d.cpu() if hasattr(d, "cpu") else d)


def DirectionalDerivative(arg_shape, order, directions, diff_method="fd", mode="constant", parallel=False,
                          **diff_kwargs):
    """First / second directional derivative (diff.py:1938-2073): sum_i v_i d_i f, or
    sum_{i<=j} (2 - delta_ij) v_i u_j d_ij f with unit directions v (and u), constant or per pixel."""
    arg_shape = tuple(arg_shape)
    ndim = len(arg_shape)
    assert order in [1, 2], "`order` should be either 1 or 2"
    if order == 1:
        assert not isinstance(directions, (list, tuple)), "`directions` for first directional derivative should be an NDArray"
        d1 = d2 = _host(directions)
    else:
        if isinstance(directions, (list, tuple)):
            assert len(directions) == 2, "`directions` for second directional derivative should be an NDArray or a tuple/list with two NDArrays of the same shape"
            d1, d2 = _host(directions[0]), _host(directions[1])
            assert d1.shape == d2.shape
        else:
            d1 = d2 = _host(directions)
    assert d1.shape[0] == ndim, "The length of `directions` should match `len(arg_shape)`"
    dt = d1.dtype
    if order == 1:
        diff = Gradient(arg_shape=arg_shape, diff_method=diff_method, mode=mode, dtype=dt, **diff_kwargs)
        w = _unit(d1, dt)
    else:
        diff = Hessian(arg_shape=arg_shape, diff_method=diff_method, mode=mode, dtype=dt, **diff_kwargs)
        w = _outer_triu(_unit(d1, dt), _unit(d2, dt))
    return _Directional(diff, w[None], "FirstDirectionalDerivative" if order == 1 else "SecondDirectionalDerivative")


def DirectionalGradient(arg_shape, directions, diff_method="fd", mode="constant", parallel=False, **diff_kwargs):
    """Stack of first directional derivatives along each of `directions` (diff.py:2076-2197)."""
    arg_shape = tuple(arg_shape)
    assert isinstance(directions, (list, tuple))
    dt = _dir_dtype(directions)
    diff = Gradient(arg_shape=arg_shape, diff_method=diff_method, mode=mode, dtype=dt, **diff_kwargs)
    w = np.stack([_unit(_host(d), dt) for d in directions])
    return _Directional(diff, w, "DirectionalGradient")


def DirectionalLaplacian(arg_shape, directions, weights=None, diff_method="fd", mode="constant", parallel=False,
                         **diff_kwargs):
    """Weighted sum of second directional derivatives (diff.py:2200-2364)."""
    arg_shape = tuple(arg_shape)
    assert isinstance(directions, (list, tuple))
    if weights is None:
        weights = [1.0] * len(directions)
    elif len(weights) != len(directions):
        raise ValueError("The number of weights and directions provided differ.")
    dt = _dir_dtype(directions)
    diff = Hessian(arg_shape=arg_shape, diff_method=diff_method, mode=mode, dtype=dt, **diff_kwargs)
    parts = []
    for wt, d in zip(weights, directions):
        n = _unit(_host(d), dt)
        parts.append(wt * _outer_triu(n, n))
    w = np.concatenate(parts, axis=0)[None]  # one output group, L * K terms (term j reads component j % K)
    return _Directional(diff, w, "DirectionalLaplacian")


def DirectionalHessian(arg_shape, directions, diff_method="gd", mode="constant", parallel=False, **diff_kwargs):
    """Second directional derivatives along every pair (i <= j) of `directions` (diff.py:2367-2542)."""
    arg_shape = tuple(arg_shape)
    assert isinstance(directions, (list, tuple))
    dt = _dir_dtype(directions)
    diff = Hessian(arg_shape=arg_shape, diff_method=diff_method, mode=mode, dtype=dt, **diff_kwargs)
    units = [_unit(_host(d), dt) for d in directions]
    w = np.stack([_outer_triu(units[i], units[j]) for i in range(len(units)) for j in range(i, len(units))])
    return _Directional(diff, w, "DirectionalHessian")
