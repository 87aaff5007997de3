"""
Thread-parallel form of the oracle's PGD TV-deblur iteration: the all-core CPU baseline of bench.py.

TEST / MEASUREMENT INFRASTRUCTURE ONLY (like the rest of oracle/): only tests/, smoke() and bench.py's
cpu_baseline leg may import it; the pyxu_amd product path never does.

The reference parallelises its CPU stencils over threads (Numba ``parallel=True``,
operator/linop/stencil/_stencil.py:246-256) or Dask chunks with halo exchange (``map_overlap``,
stencil.py:578-606).  This restatement does the latter with a thread pool: the image rows are cut
into slabs, each worker runs the SAME single-thread oracle code (pyxu_np.pgd's extrapolation, the
deblur_tv_grad rule stack, the step and the prox) on its slab plus a halo of ``2R + 2`` rows and keeps
its interior rows.  Outputs at distance >= 2R + 2 from an artificial cut do not see it (H then H^T
reach R each, the forward difference and its adjoint one each), and every element is computed by the
same arithmetic in the same order, so the result is bit-identical to ``pyxu_np.pgd`` (checked by
tests/test_host_logic.py).  NumPy releases the GIL inside its array loops, so the slabs run
concurrently.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from oracle import pyxu_np as orc

__all__ = ["pgd_tv_threaded", "pgd_tv_images_threaded"]


def _slabs(n0, parts):
    parts = max(1, min(parts, n0))
    q, r = divmod(n0, parts)
    out, lo = [], 0
    for p in range(parts):
        hi = lo + q + (1 if p < r else 0)
        out.append((lo, hi))
        lo = hi
    return out


def pgd_tv_threaded(x0, blur, y, lam, mu, prox, tau, n_iter, threads, d=75):
    """``pyxu_np.pgd(x0, grad, prox, tau, n_iter)`` with ``grad = deblur_tv_grad(., blur, y, lam, mu,
    arg_shape)`` evaluated slab by slab on `threads` worker threads (2-D images, rows = axis 0).
    ``prox(z)`` must be element-wise (PositiveOrthant / L1).  Returns ``(x, x_prev)``."""
    sh = tuple(blur["arg_shape"])
    n0 = sh[0]
    R = max(max(len(k) - 1 - c, c) for k, c in zip(blur["kernel"], blur["center"]))
    halo = 2 * R + 2
    dt = x0.dtype.type
    tau = dt(tau)
    Y = y.reshape(sh)
    slabs = _slabs(n0, threads)
    x = x_prev = x0.reshape(sh)

    def work(args):
        lo, hi, a, X, XP, OUT = args
        ha, hb = max(0, lo - halo), min(n0, hi + halo)
        sub = (hb - ha, *sh[1:])
        # extrapolation (pgd.py:179-181) on slab + halo, same ops as pyxu_np.pgd
        yk = X[ha:hb] - XP[ha:hb]
        yk *= a
        yk += X[ha:hb]
        b = dict(blur, arg_shape=sub)
        g = orc.deblur_tv_grad(yk.reshape(-1), b, Y[ha:hb].reshape(-1), lam, mu, dict(arg_shape=sub)).reshape(sub)
        z = g[lo - ha:hi - ha].copy()
        z *= -tau
        z += yk[lo - ha:hi - ha]
        OUT[lo:hi] = prox(z)

    with ThreadPoolExecutor(max_workers=len(slabs)) as pool:
        for k in range(n_iter):
            a = dt(k / (k + 1 + d))
            out = np.empty(sh, dtype=x0.dtype)
            list(pool.map(work, [(lo, hi, a, x, x_prev, out) for lo, hi in slabs]))
            x_prev, x = x, out
    return x.reshape(-1), x_prev.reshape(-1)


def pgd_tv_images_threaded(x0s, blur, ys, lam, mu, prox, tau, n_iter, threads, d=75):
    """``pyxu_np.pgd`` on each of several INDEPENDENT images (batched stacks, config C5: each image its own
    data y), one image per worker thread at a time -- the reference's stacked-problem parallelism
    (independent leading dims) on a thread pool.  Every image runs the single-thread
    oracle unchanged.  Returns the list of final iterates."""
    sh = tuple(blur["arg_shape"])

    def one(args):
        x0, y = args
        grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
        return orc.pgd(x0, grad, prox, tau, n_iter, d=d)[0]

    with ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
        return list(pool.map(one, zip(x0s, ys)))
