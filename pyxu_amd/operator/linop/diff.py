"""
Finite-difference operators (mirrors reference operator/linop/diff.py): PartialDerivative,
Gradient.

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

__all__ = ["PartialDerivative", "Gradient", "Hessian", "Laplacian", "Divergence", "fd_coefficients"]


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


def Gradient(arg_shape, directions=None, diff_method="fd", mode="constant", gpu=True, dtype=None, parallel=False,
             **diff_kwargs):
    """Gradient operator (diff.py:1113-1265)."""
    if diff_method != "fd":
        raise NotImplementedError("pyxu_amd: only diff_method='fd' (finite differences) is on the hot path.")
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
        stencils.append(
            PartialDerivative.finite_difference(arg_shape=arg_shape, order=tuple(order), scheme=sch, accuracy=acc,
                                                mode=mode, dtype=dtype, sampling=samp)
        )
    op = _DiffStack(arg_shape, stencils, directions)
    op._name = "Gradient"
    op.meta = dict(sampling=samp, scheme=sch, accuracy=acc)
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
    if diff_method != "fd":
        raise NotImplementedError("pyxu_amd: only diff_method='fd' (finite differences) is on the hot path.")
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
    if diff_method != "fd":
        raise NotImplementedError("pyxu_amd: only diff_method='fd' (finite differences) is on the hot path.")
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
        stencils.append(_fd_stencil(arg_shape, order, _tuple(scheme, D) if isinstance(scheme, str) else tuple(scheme),
                                    _tuple(accuracy, D), mode, dtype, _tuple(sampling, D)))
    op = _Divergence(arg_shape, stencils)
    op._name = "Divergence"
    return op
