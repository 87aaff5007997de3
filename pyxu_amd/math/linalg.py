"""Stochastic trace estimation (reference pyxu/math/linalg.py:62-117, Hutch++ = Algorithm 3 of
arXiv:2010.09649) on the MI355X.

The query vectors are drawn on the host with ``numpy.random.default_rng(seed)`` exactly as the reference
draws them (same seed -> same queries), uploaded once, and every product runs on the device: the operator
applied to a stack of query rows (one batched launch per operator stage), the range basis by a
Gram-eigendecomposition QR (the (b, b) Gram matrix on the MFMA / GEMV dense kernels in fp64, its
eigendecomposition on the host, two passes), the projections and the row dot products on the dense and
reduction kernels.  The estimate is basis-independent (tr(Q^T A Q) and (I - Q Q^T) g do not depend on
which orthonormal basis of range(A S) is used), so it agrees with the reference's Householder-QR result
for the same seed up to floating-point rounding; directions of range(A S) below 1e-12 of the largest
Gram eigenvalue are left to the Hutchinson term (still unbiased).
"""
import numpy as np

import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev

__all__ = ["hutchpp"]


def _orth_rows(Y):
    """Orthonormal rows spanning the row space of Y (b, n): Q^T = W^T Y with W from the eigendecomposition
    of the fp64 Gram matrix Y Y^T; two passes (the second cleans up the first's rounding)."""
    work = _dev.cast(Y, _dev.empty((1,), Y).double()) if Y.dtype != _dev._torch().float64 else Y
    for _ in range(2):
        G = _dev.dense_matmat(work, work, 0).cpu().numpy()  # (b, b) = Y Y^T
        G = 0.5 * (G + G.T)
        lam, V = np.linalg.eigh(G)
        keep = lam > 1e-12 * max(lam.max(), 0.0)
        if not np.any(keep):
            return None
        W = V[:, keep] / np.sqrt(lam[keep])  # (b, k)
        Wt = _dev.to_device_like(np.ascontiguousarray(W.T), work)  # (k, b)
        work = _dev.dense_matmat(work, Wt, 1)  # (k, n) = W^T Y
    return _dev.cast(work, Y) if Y.dtype != work.dtype else work


def _trace_rows(op, R):
    """sum_i <op(r_i), r_i> over the rows of R (k, n), accumulated in fp64."""
    AR = _dev.require(op.apply(R)).reshape(R.shape)
    return float(np.sum(_dev.row_reduce(_dev.RED_DOT, AR, R).cpu().numpy()))


def hutchpp(op, m=4002, xp=None, dtype=None, seed=None):
    """Stochastic estimate of tr(op) for a square operator (linalg.py:62-117).  `xp` is accepted for
    signature parity; the arrays always live on the MI355X."""
    if dtype is None:
        dtype = pxrt.getPrecision().value
    dtype = np.dtype(dtype)
    rng = np.random.default_rng(seed=seed)
    s = rng.standard_normal(size=(op.dim, (m + 2) // 4), dtype=dtype)
    g = rng.integers(0, 2, size=(op.dim, (m - 2) // 2)) * 2 - 1
    from pyxu_amd.util import to_device

    with pxrt.Precision(pxrt.Width(dtype)):
        S = to_device(np.ascontiguousarray(s.T))  # (b, n) query rows
        Y = _dev.require(op.apply(S)).reshape(S.shape)  # rows of (A S)^T
        del S
        Qt = _orth_rows(Y)
        del Y
        Gt = to_device(np.ascontiguousarray(g.T.astype(dtype)))  # (r, n)
        if Qt is None:
            tr = 0.0
            Pt = Gt
        else:
            tr = _trace_rows(op, Qt)
            C = _dev.dense_matmat(Qt, Gt, 0)  # (r, k) = G^T Q
            Pt = _dev.axpby(1.0, Gt, -1.0, _dev.dense_matmat(Qt, C, 1))  # G^T - (G^T Q) Q^T
        tr += (2 / (m - 2)) * _trace_rows(op, Pt)
    return float(tr)
