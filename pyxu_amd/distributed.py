"""
Multi-GPU sharding of the proximal-splitting path.

One process per GPU, ``torch.distributed`` with backend ``"nccl"`` (= RCCL over xGMI on MI355X);
``"gloo"`` serves the CPU tests.  The reference has no multi-device solver (its Dask backend chunks
arrays, ``operator/linop/stencil/stencil.py:578-606``); this module adds exactly the two exchange
steps the hot path has, and nothing else:

* **Batched independent stacks** (C5: ``(B, n0, n1)`` batch-as-axis problems).  Axis 0 is split into
  contiguous slabs (:func:`shard_range`); the blur / gradient have size-1 taps on that axis, so a
  slab iterates with no halo and no data-path collective.  The only exchange is the stopping
  criterion: :class:`ShardedRelError` / :class:`ShardedAbsError` all-reduce their two device row
  statistics (sum for L1/L2, max for Linf) once per stop check, so every rank takes the same
  decision as the unsharded solver.  :func:`gather_slabs` assembles ``solution()`` on demand.
* **Row-sharded dense LinOp** (C4: ADMM / CG with ``K`` of shape ``(M, N)``).  Rank r holds rows
  ``shard_range(M)`` of K.  ``apply`` is local (the rank's slice of ``Kx``); ``adjoint`` sums the
  ranks' partial ``K_r^T z_r`` with one all-reduce of ``(B, N)`` values.  Through the operator
  algebra ``K.T * K`` (the CG normal-equation operator of ``QuadraticFunc.prox``,
  ``abc/operator.py:1273-1291``) therefore costs one all-reduce per CG iteration, and the CG
  vectors (x, r, p) and their dot products stay replicated — no further communication.

* **Halo-exchanged volume slabs** (volumes larger than one GPU; the analogue
  of the reference's Dask ``map_overlap``, ``stencil.py:578-606``).  A volume is split along axis 0;
  :class:`SlabLinOp` applies a rank-local operator (Stencil / Gaussian / Gradient / ...) to the
  rank's slab padded with ``halo`` planes received from its two neighbours (point-to-point
  send/recv, zeros beyond the volume) and crops the result; the adjoint sends the halo part of the
  local adjoint back to the neighbours, which add it to their edge planes.  Both are exact: the
  global operator restricted to the slab is Crop o S_local o HaloPad.

Message sizes are a few doubles (stop checks), ``4·N·B`` bytes (C4: 256 KiB per right-hand side at
N = 65 536) or a few planes (halos: R planes of n1·n2 values per neighbour): latency-bound on xGMI,
so RCCL's default (LL/one-shot) protocols are the right choice.
"""
import numpy as np

import pyxu_amd.abc as pxa
import pyxu_amd.runtime as pxrt
from pyxu_amd.opt.stop import AbsError, RelError

__all__ = [
    "world",
    "shard_range",
    "allreduce",
    "gather_slabs",
    "ShardedRelError",
    "ShardedAbsError",
    "RowShardedLinOp",
    "halo_pad",
    "halo_reduce",
    "SlabLinOp",
]


def _dist():
    import torch.distributed as dist

    return dist


def world(group=None):
    """(rank, world_size) of `group` (default group), or (0, 1) when torch.distributed is not initialised."""
    dist = _dist()
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_range(n, rank=None, world_size=None, group=None):
    """Contiguous balanced block [lo, hi) of `n` items owned by `rank`: the first n % world ranks
    own one extra item.  Deterministic, so every rank computes every other rank's range."""
    if rank is None or world_size is None:
        r, w = world(group)
        rank = r if rank is None else rank
        world_size = w if world_size is None else world_size
    if not (0 <= rank < world_size):
        raise ValueError(f"rank {rank} outside [0, {world_size})")
    q, rem = divmod(int(n), int(world_size))
    lo = rank * q + min(rank, rem)
    return lo, lo + q + (1 if rank < rem else 0)


def collectives_at_world1():
    """True when ``PXA_DIST_COLLECTIVES=always``: the collectives below run even in a world of one
    process instead of short-circuiting.  A one-GPU box can then drive the RCCL path end to end
    (a world-size-1 ``nccl`` group: ``tests/test_gpu_rccl.py``); the results must not change."""
    import os

    return os.environ.get("PXA_DIST_COLLECTIVES", "").lower() == "always"


def _initialised():
    dist = _dist()
    return dist.is_available() and dist.is_initialized()


def allreduce(t, op="sum", group=None):
    """In-place all-reduce of tensor `t` over `group` (no-op on one process, unless
    :func:`collectives_at_world1`).  Device tensors go through RCCL, host tensors through gloo; the
    reduction order is the library's (fixed for a given world size)."""
    rank, w = world(group)
    if w == 1 and not (collectives_at_world1() and _initialised()):
        return t
    dist = _dist()
    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
    if t.is_cuda and _host_backend(group):
        h = t.cpu()  # gloo host staging (CPU tests / several ranks sharing one card)
        dist.all_reduce(h, op=ops[op], group=group)
        t.copy_(h)  # gloo host staging
        return t
    dist.all_reduce(t, op=ops[op], group=group)
    return t


def _host_backend(group=None):
    return str(_dist().get_backend(group)).lower() == "gloo"


def gather_slabs(x_local, n_global, group=None):
    """All-gather of contiguous slabs along axis 0 (shard_range partition of `n_global` rows):
    returns the full (n_global, ...) array on every rank.  Unequal slabs are padded to the largest
    one for the collective and trimmed afterwards."""
    import torch

    rank, w = world(group)
    if w == 1 and not (collectives_at_world1() and _initialised()):
        return x_local
    # the pad below copies by raw pointer and all_gather needs dense storage: permuted / strided views of a
    # slab are made contiguous first
    x_local = x_local.contiguous()
    sizes = [shard_range(n_global, r, w)[1] - shard_range(n_global, r, w)[0] for r in range(w)]
    if x_local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank} holds {x_local.shape[0]} rows, expected {sizes[rank]}")
    m = max(sizes)
    buf = x_local
    if x_local.shape[0] != m:  # pad the slab to the largest one (pxa_fill + pxa_copy2d on the device)
        n_row = int(np.prod(x_local.shape[1:]))
        buf = _dev_zeros((m, *x_local.shape[1:]), x_local)
        n_el = x_local.shape[0] * n_row
        _dev_copy_rows(x_local, buf, 1, n_el, n_el, n_el, 0, 0)
    dev = buf.device
    if buf.is_cuda and _host_backend(group):
        buf = buf.cpu()  # gloo host staging
    parts = [torch.empty_like(buf) for _ in range(w)]
    _dist().all_gather(parts, buf, group=group)
    if parts[0].is_cuda:  # RCCL: assemble the slabs on the device (pxa_copy2d)
        from pyxu_amd import xp

        return xp.concatenate([p[:s] for p, s in zip(parts, sizes)], axis=0)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0).to(dev)  # gloo host staging


class _ShardedMixin:
    def _bind_group(self, group):
        self._group = group

    def _reduce(self, stat, op):
        return allreduce(stat.contiguous(), op=op, group=self._group)


class ShardedRelError(_ShardedMixin, RelError):
    """RelError (``opt/stop.py:300-396``) of a problem whose state is split across ranks along the
    last axis (batch-as-axis slabs): ``||x - x_prev|| / ||x_prev||`` with the norms taken over the
    WHOLE state, i.e. the per-rank row statistics all-reduced before the ratio.  Every rank returns
    the same decision."""

    def __init__(self, eps, var="x", f=None, norm=2, satisfy_all=True, group=None):
        super().__init__(eps=eps, var=var, f=f, norm=norm, satisfy_all=satisfy_all)
        self._bind_group(group)


class ShardedAbsError(_ShardedMixin, AbsError):
    """AbsError (``opt/stop.py:222-297``) over a state split across ranks (see ShardedRelError)."""

    def __init__(self, eps, var="x", f=None, norm=2, satisfy_all=True, group=None):
        super().__init__(eps=eps, var=var, f=f, norm=norm, satisfy_all=satisfy_all)
        self._bind_group(group)


def RowShardedLinOp(mat_local, M, group=None, enable_warnings=True):
    """Rank-local row block of a dense ``(M, N)`` operator K (``operator/linop/base.py:334-512``).

    ``mat_local`` holds rows ``shard_range(M)`` of K on this rank's device.  The returned LinOp has
    shape ``(M_r, N)``: ``apply(x)`` gives this rank's slice of ``K x`` (local GEMV, no
    communication), ``adjoint(z_r)`` gives the FULL ``K^T z = sum_r K_r^T z_r`` (local GEMV + one
    all-reduce).  Combined by the operator algebra, ``K.T * K`` is the global normal operator.
    """
    from pyxu_amd.operator.interop import from_source
    from pyxu_amd.operator.linop.base import _ExplicitLinOp

    rank, w = world(group)
    lo, hi = shard_range(M, rank, w)
    if mat_local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: expected rows [{lo}, {hi}) of K, got {mat_local.shape[0]} rows")
    local = _ExplicitLinOp(pxa.LinOp, mat_local, enable_warnings=enable_warnings)

    @pxrt.enforce_precision(i="arr")
    def op_apply(_, arr):
        return local.apply(arr)

    @pxrt.enforce_precision(i="arr")
    def op_adjoint(_, arr):
        return allreduce(local.adjoint(arr).contiguous(), "sum", group)

    op = from_source(
        cls=pxa.LinOp,
        shape=(hi - lo, int(mat_local.shape[1])),
        embed=dict(_name="RowShardedLinOp", _rows=(lo, hi), _M=int(M), _group=group, _local=local),
        apply=op_apply,
        adjoint=op_adjoint,
    )
    return op


# ------------------------------------------------------------------ halo-exchanged slabs
def _p2p(sends, recvs, group=None):
    """Point-to-point exchange: sends = [(tensor, peer)], recvs = [(buffer, peer)], all contiguous.
    Device tensors go through RCCL directly; with gloo they are staged through the host."""
    dist = _dist()
    if not sends and not recvs:
        return
    host = _host_backend(group)
    stage = lambda t: t.cpu() if (host and t.is_cuda) else t  # noqa: E731  (gloo host staging)
    s_bufs = [(stage(t), peer) for t, peer in sends]
    r_bufs = [(stage(b), b, peer) for b, peer in recvs]
    ops = [dist.P2POp(dist.isend, t, _global_rank(peer, group), group) for t, peer in s_bufs]
    ops.extend(dist.P2POp(dist.irecv, h, _global_rank(peer, group), group) for h, _, peer in r_bufs)
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    for h, b, _ in r_bufs:
        if h is not b:
            b.copy_(h)  # gloo host staging


def _global_rank(r, group):
    if group is None:
        return r
    return _dist().get_global_rank(group, r)


# Device-path array movement: every copy, zero fill and accumulation of the exchange runs on the HIP
# kernels (pxa_copy2d / pxa_fill); torch tensors only arise as buffers (and as host tensors in the gloo
# CPU tests, handled by the torch fallbacks below).
def _dev_zeros(shape, like):
    import torch

    if like.is_cuda:
        from pyxu_amd import _dev

        return _dev.zeros(shape, like)
    return torch.zeros(shape, dtype=like.dtype)  # gloo CPU tests


def _dev_copy_rows(src, dst, rows, n, lds, ldd, src_off, dst_off, accumulate=0):
    """dst[dst_off + r ldd + i] (+)= src[src_off + r lds + i], r < rows, i < n (element offsets)."""
    if rows == 0 or n == 0:
        return dst
    if lds < 0 or ldd < n:  # pxa_copy2d's argument contract, checked on the gloo CPU path too
        raise ValueError(f"copy rows: lds={lds}, ldd={ldd} for rows of {n}")
    if src.is_cuda:
        from pyxu_amd import _dev

        return _dev.copy2d(src, dst, rows, n, lds, ldd, src_off=src_off, dst_off=dst_off, accumulate=accumulate)
    s2 = src.reshape(-1).as_strided((rows, n), (lds, 1), src_off)  # gloo CPU tests
    d2 = dst.reshape(-1).as_strided((rows, n), (ldd, 1), dst_off)
    if accumulate:
        d2 += s2
    else:
        d2.copy_(s2)
    return dst


def _planes(x, p0, p1):
    """Contiguous copy of planes [p0, p1) of every stack row of x (S, P, M)."""
    S, P, M = x.shape
    out = _dev_zeros((S, p1 - p0, M), x) if not x.is_cuda else _empty(x, (S, p1 - p0, M))
    return _dev_copy_rows(x, out, S, (p1 - p0) * M, P * M, (p1 - p0) * M, p0 * M, 0)


def _empty(like, shape):
    import torch

    return torch.empty(shape, dtype=like.dtype, device=like.device)


def halo_pad(x, lo, hi, group=None):
    """x: (S, nl, M) slab of axis-0 planes owned by this rank -> (S, lo + nl + hi, M) with the last
    `lo` planes of rank-1 in front, the first `hi` planes of rank+1 behind (zeros beyond the volume).
    The received halos land directly in the padded output (one pxa_copy2d places the slab)."""
    rank, w = world(group)
    S, nl, M = x.shape
    if nl < max(lo, hi) and w > 1:
        raise ValueError(f"slab of {nl} planes is thinner than the halo ({lo}, {hi})")
    x = x if x.is_contiguous() else x.contiguous()
    P = lo + nl + hi
    out = _dev_zeros((S, P, M), x)
    _dev_copy_rows(x, out, S, nl * M, nl * M, P * M, 0, lo * M)
    sends, recvs, land = [], [], []
    if rank > 0:
        if hi:
            sends.append((_planes(x, 0, hi), rank - 1))
        if lo:
            left = _empty(x, (S, lo, M))
            recvs.append((left, rank - 1))
            land.append((left, 0, lo))
    if rank < w - 1:
        if lo:
            sends.append((_planes(x, nl - lo, nl), rank + 1))
        if hi:
            right = _empty(x, (S, hi, M))
            recvs.append((right, rank + 1))
            land.append((right, lo + nl, hi))
    _p2p(sends, recvs, group)
    for buf, p0, n in land:
        _dev_copy_rows(buf, out, S, n * M, n * M, P * M, 0, p0 * M)
    return out


def halo_reduce(xp, lo, hi, group=None):
    """Adjoint of halo_pad: xp (S, lo + nl + hi, M) -> (S, nl, M), the halo planes sent back to the
    neighbours that own them and added to their edge planes (dropped beyond the volume).  Each
    received halo is added to all S stack rows by ONE pxa_copy2d accumulate launch."""
    rank, w = world(group)
    S, P, M = xp.shape
    nl = P - lo - hi
    xp = xp if xp.is_contiguous() else xp.contiguous()
    out = _planes(xp, lo, lo + nl)
    sends, recvs, land = [], [], []
    if rank > 0:
        if lo:
            sends.append((_planes(xp, 0, lo), rank - 1))  # my left halo = rank-1's last lo planes
        if hi:
            from_left = _empty(xp, (S, hi, M))
            recvs.append((from_left, rank - 1))  # rank-1's right halo = my first hi planes
            land.append((from_left, 0, hi))
    if rank < w - 1:
        if hi:
            sends.append((_planes(xp, lo + nl, P), rank + 1))
        if lo:
            from_right = _empty(xp, (S, lo, M))
            recvs.append((from_right, rank + 1))
            land.append((from_right, nl - lo, lo))
    _p2p(sends, recvs, group)
    for buf, p0, n in land:
        _dev_copy_rows(buf, out, S, n * M, n * M, nl * M, 0, p0 * M, accumulate=1)
    return out


class SlabLinOp(pxa.LinOp):
    """This rank's slab (axis 0, :func:`shard_range`) of a linear operator on a volume of
    ``global_shape``, evaluated with halo exchange (module docstring).

    ``make_local(padded_shape)`` builds the rank-local operator on the padded slab
    ``(lo + nl + hi, *global_shape[1:])`` with zero-boundary semantics (e.g.
    ``lambda sh: pyxu_amd.operator.Gaussian(sh, sigma=2)`` or ``Gradient(sh)``); its output may hold
    K blocks of the padded shape (Gradient: K = D, direction-major).  ``halo = (lo, hi)`` must cover
    the operator's reach along axis 0 (planes before / after the output plane).  Input: the rank's
    ``(..., nl * M)`` slab; output ``(..., K * nl * M)``, direction-major like the local operator.
    """

    def __init__(self, make_local, global_shape, halo, group=None):
        global_shape = tuple(int(v) for v in global_shape)
        rank, w = world(group)
        a, b = shard_range(global_shape[0], rank, w)
        self._nl, self._M = b - a, int(np.prod(global_shape[1:]))
        self._halo = (int(halo[0]), int(halo[1]))
        self._group = group
        self._rows = (a, b)
        pshape = (self._halo[0] + self._nl + self._halo[1], *global_shape[1:])
        self._local = make_local(pshape)
        pdim = int(np.prod(pshape))
        if self._local.dim != pdim or self._local.codim % pdim != 0:
            raise ValueError("make_local must return an operator on the padded slab with K * padded outputs")
        self._K = self._local.codim // pdim
        super().__init__(shape=(self._K * self._nl * self._M, self._nl * self._M))
        self.lipschitz = getattr(self._local, "lipschitz", np.inf)

    def _stack(self, arr):
        sh = arr.shape[:-1]
        return sh, int(np.prod(sh)) if len(sh) else 1

    @pxrt.enforce_precision(i="arr")
    def apply(self, arr):
        (lo, hi), nl, M, K = self._halo, self._nl, self._M, self._K
        sh, S = self._stack(arr)
        P = lo + nl + hi
        xp = halo_pad(arr.reshape(S, nl, M), lo, hi, self._group)
        y = self._local.apply(xp.reshape(S, -1))
        y = y if y.is_contiguous() else y.contiguous()
        out = _empty(y, (S * K, nl * M))  # crop: planes [lo, lo + nl) of every (row, block), one launch
        _dev_copy_rows(y, out, S * K, nl * M, P * M, nl * M, lo * M, 0)
        return out.reshape(*sh, K * nl * M)

    @pxrt.enforce_precision(i="arr")
    def adjoint(self, arr):
        (lo, hi), nl, M, K = self._halo, self._nl, self._M, self._K
        sh, S = self._stack(arr)
        P = lo + nl + hi
        a = arr.reshape(S * K, nl * M)
        a = a if a.is_contiguous() else a.contiguous()
        yp = _dev_zeros((S * K, P * M), a)  # embed into the zero-padded slab, one launch
        _dev_copy_rows(a, yp, S * K, nl * M, nl * M, P * M, 0, lo * M)
        xp = self._local.adjoint(yp.reshape(S, -1)).reshape(S, P, M)
        return halo_reduce(xp, lo, hi, self._group).reshape(*sh, nl * M)
