"""
Worker bodies of the multi-process tests (spawned by test_distributed_cpu.py / test_gpu_distributed.py).

Each worker initialises torch.distributed (gloo, 127.0.0.1), runs one scenario and puts
(rank, result-dict) on a queue.  Kept in a module of its own so torch.multiprocessing's spawn can
import it by name.
"""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _init(rank, world, port, backend="gloo"):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":  # RCCL: the rank's device must be bound before the group is created
        import torch

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return dist


def run(rank, world, port, scenario, q, kwargs):
    try:
        kwargs = dict(kwargs)
        dist = _init(rank, world, port, kwargs.pop("_backend", "gloo"))
        out = globals()[scenario](rank, world, **kwargs)
        q.put((rank, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported by the parent
        q.put((rank, {"error": traceback.format_exc()}))


# ------------------------------------------------------------------ CPU scenarios (host logic)
def collectives(rank, world):
    import torch

    import pyxu_amd.distributed as pd

    t = torch.tensor([1.0 + rank, 10.0 * rank], dtype=torch.float64)
    s = pd.allreduce(t.clone(), "sum").tolist()
    m = pd.allreduce(t.clone(), "max").tolist()
    lo, hi = pd.shard_range(5)
    x = torch.arange(lo, hi, dtype=torch.float32).reshape(-1, 1).repeat(1, 3)
    g = pd.gather_slabs(x, 5)
    crit = pd.ShardedRelError(eps=1e-3)
    r = crit._reduce(torch.tensor([[1.0], [2.0]], dtype=torch.float64), "sum").tolist()
    return dict(sum=s, max=m, gathered=g.numpy(), crit_reduce=r)


def batched_pgd_oracle(rank, world, B, sh, iters, eps):
    """C5 host logic: batch-as-axis PGD, slabs of images per rank, global RelError via allreduce.
    The per-slab arithmetic is the CPU oracle (stand-in for the HIP kernels in this CPU test)."""
    import torch

    import oracle as orc
    import pyxu_amd.distributed as pd

    rng = np.random.default_rng(11)
    N = int(np.prod(sh))
    ys = rng.standard_normal((B, N)).astype(np.float32)
    lo, hi = pd.shard_range(B)
    lam, mu = 0.02, 0.01
    taps, c = orc.gaussian_taps(2.0, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    tau = np.float32(1 / np.float32(1 + 8 * lam / mu))
    x = np.zeros((hi - lo, N), np.float32)
    xp = x.copy()
    k = 0
    stopped_at = None
    for k in range(iters):
        a = np.float32(k / (k + 1 + 75))
        yk = (x - xp) * a + x
        z = np.stack([yk[i] - tau * orc.deblur_tv_grad(yk[i], blur, ys[lo + i], lam, mu, dict(arg_shape=sh))
                      for i in range(hi - lo)]).astype(np.float32)
        xn = np.maximum(z, 0).astype(np.float32)
        st = torch.tensor([float(((xn.astype(np.float64) - x) ** 2).sum()), float((x.astype(np.float64) ** 2).sum())],
                          dtype=torch.float64)
        pd.allreduce(st, "sum")
        xp, x = x, xn
        if k > 0 and st[0].item() ** 0.5 <= eps * st[1].item() ** 0.5:
            stopped_at = k
            break
    full = pd.gather_slabs(torch.from_numpy(x), B).numpy()
    return dict(x=full, stopped_at=stopped_at)


def row_sharded_normal_cg(rank, world, M, N, iters):
    """C4 host logic: K row-sharded; K^T K p = allreduce(K_r^T K_r p); CG on (K^T K + I/tau) with
    replicated vectors equals the unsharded CG."""
    import torch

    import oracle as orc
    import pyxu_amd.distributed as pd

    rng = np.random.default_rng(5)
    K = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float64)
    b = rng.standard_normal(N)
    lo, hi = pd.shard_range(M)
    Kr = K[lo:hi]
    tau = 0.7

    def A(p):
        part = torch.from_numpy((Kr.T @ (Kr @ p.T)).T.copy())
        return pd.allreduce(part, "sum").numpy() + p / tau

    x, n = orc.cg(A, b[None, :], max_iter=iters)
    return dict(x=x, n=n)


class _OracleVolumeOp:
    """Host stand-in for a pyxu_amd volume operator (the HIP kernels need a GPU): Gaussian blur on all
    axes ("blur") or the forward-difference Gradient ("grad") through the CPU oracle."""

    def __init__(self, shape, kind, sigma=1.0):
        import oracle as orc

        self.shape, self.kind = tuple(shape), kind
        n = int(np.prod(shape))
        self.dim = n
        self.codim = n * (len(shape) if kind == "grad" else 1)
        taps, c = orc.gaussian_taps(sigma, 3.0, np.float64)
        self._blur = dict(kernel=[taps] * len(shape), center=[c] * len(shape))

    def apply(self, x):
        import torch

        import oracle as orc

        a = x.numpy()
        y = orc.gradient_apply(a, self.shape) if self.kind == "grad" else orc.stencil_apply(a, self.shape, **self._blur)
        return torch.from_numpy(np.ascontiguousarray(y))

    def adjoint(self, z):
        import torch

        import oracle as orc

        a = z.numpy()
        x = orc.gradient_adjoint(a, self.shape) if self.kind == "grad" else orc.stencil_adjoint(a, self.shape, **self._blur)
        return torch.from_numpy(np.ascontiguousarray(x))


def slab_halo_oracle(rank, world, shape, kind, halo, sigma=1.0):
    """SlabLinOp exchange logic on the host: apply / adjoint of this rank's slab (halo-padded local
    operator, cropped / halo-reduced), gathered along axis 0."""
    import torch

    import pyxu_amd.distributed as pd
    import pyxu_amd.runtime as pxrt

    rng = np.random.default_rng(21)
    N = int(np.prod(shape))
    K = len(shape) if kind == "grad" else 1
    x = rng.standard_normal((2, N))
    y = rng.standard_normal((2, K * N))
    lo, hi = pd.shard_range(shape[0])
    M = N // shape[0]
    with pxrt.Precision(pxrt.Width.DOUBLE):
        op = pd.SlabLinOp(lambda sh: _OracleVolumeOp(sh, kind, sigma), shape, halo)
        xl = torch.from_numpy(x.reshape(2, shape[0], M)[:, lo:hi].reshape(2, -1).copy())
        yl = torch.from_numpy(y.reshape(2, K, shape[0], M)[:, :, lo:hi].reshape(2, -1).copy())
        ya = op.apply(xl).reshape(2, K, hi - lo, M)
        xa = op.adjoint(yl).reshape(2, hi - lo, M)
    Y = pd.gather_slabs(ya.permute(2, 0, 1, 3).contiguous(), shape[0]).permute(1, 2, 0, 3).reshape(2, K * N)
    X = pd.gather_slabs(xa.permute(1, 0, 2).contiguous(), shape[0]).permute(1, 0, 2).reshape(2, N)
    return dict(apply=Y.numpy(), adjoint=X.numpy(), x=x, y=y)


# ------------------------------------------------------------------ GPU scenarios (real HIP path)
def gpu_slab_ops(rank, world, shape):
    """SlabLinOp on the MI355X with the real HIP Gaussian / Gradient vs the unsharded operators."""
    import torch

    torch.cuda.set_device(0)
    import pyxu_amd.distributed as pd
    import pyxu_amd.operator as pxo
    import pyxu_amd.runtime as pxrt
    from pyxu_amd.util import to_device, to_NUMPY

    rng = np.random.default_rng(23)
    N = int(np.prod(shape))
    M = N // shape[0]
    lo, hi = pd.shard_range(shape[0])
    out = {}
    with pxrt.Precision(pxrt.Width.SINGLE):
        cases = {"blur": (lambda sh: pxo.Gaussian(arg_shape=sh, sigma=1.5), (5, 5), 1),
                 "grad": (lambda sh: pxo.Gradient(arg_shape=sh), (0, 1), len(shape))}
        for name, (make, halo, K) in cases.items():
            x = rng.standard_normal((2, N)).astype(np.float32)
            y = rng.standard_normal((2, K * N)).astype(np.float32)
            op = pd.SlabLinOp(make, shape, halo)
            xl = to_device(x.reshape(2, shape[0], M)[:, lo:hi].reshape(2, -1).copy())
            yl = to_device(y.reshape(2, K, shape[0], M)[:, :, lo:hi].reshape(2, -1).copy())
            ya = op.apply(xl).reshape(2, K, hi - lo, M)
            xa = op.adjoint(yl).reshape(2, hi - lo, M)
            Y = pd.gather_slabs(ya.permute(2, 0, 1, 3).contiguous(), shape[0]).permute(1, 2, 0, 3).reshape(2, K * N)
            X = pd.gather_slabs(xa.permute(1, 0, 2).contiguous(), shape[0]).permute(1, 0, 2).reshape(2, N)
            # a permuted (non-contiguous) slab view, uneven shards (23 planes over 2 ranks): same result
            X_nc = pd.gather_slabs(xa.permute(1, 0, 2), shape[0]).permute(1, 0, 2).reshape(2, N)
            full = make(shape)
            out[name] = dict(apply=to_NUMPY(Y), adjoint=to_NUMPY(X), adjoint_nc=to_NUMPY(X_nc), apply_ref=to_NUMPY(full.apply(to_device(x))),
                             adjoint_ref=to_NUMPY(full.adjoint(to_device(y))))
    return out

def gpu_batched_pgd(rank, world, B, sh, iters, eps):
    """C5 on the MI355X: each rank solves its slab with the fused kernel; ShardedRelError."""
    import torch

    torch.cuda.set_device(0)
    import pyxu_amd.distributed as pd
    import pyxu_amd.operator as pxo
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd.util import to_device, to_NUMPY

    rng = np.random.default_rng(13)
    N = int(np.prod(sh))
    ys = rng.standard_normal((B, N)).astype(np.float32)
    lam, mu = 0.02, 0.01

    def solve(lo, hi, crit):
        b = hi - lo
        with pxrt.Precision(pxrt.Width.SINGLE):
            H = pxo.Gaussian(arg_shape=(b, *sh), sigma=(0, 2.0, 2.0))
            G = pxo.Gradient(arg_shape=(b, *sh), directions=(1, 2))
            f = 0.5 * pxo.SquaredL2Norm(dim=b * N).asloss(to_device(ys[lo:hi].reshape(-1))) * H + \
                lam * pxo.L21Norm(arg_shape=(2, b, *sh)).moreau_envelope(mu) * G
            f.diff_lipschitz = 1 + 8 * lam / mu
            s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=b * N), show_progress=False)
            s.fit(x0=to_device(np.zeros(b * N, np.float32)), stop_crit=pxst.MaxIter(iters) | crit)
            assert s._plan is not None
            _, hist = s.stats()
            return s.solution(), int(hist["iteration"][-1])

    lo, hi = pd.shard_range(B)
    x_loc, it_sh = solve(lo, hi, pd.ShardedRelError(eps=eps))
    x_all = to_NUMPY(pd.gather_slabs(x_loc.reshape(hi - lo, N), B))
    out = dict(x=x_all, it=it_sh)
    if rank == 0:  # unsharded reference run of the same batched problem
        x_ref, it_ref = solve(0, B, pxst.RelError(eps=eps))
        out.update(x_ref=to_NUMPY(x_ref).reshape(B, N), it_ref=it_ref)
    return out


def gpu_row_sharded_admm(rank, world, M, N, n_iter):
    """C4 on the MI355X: ADMM (prox path, CG x-update) with K row-sharded vs unsharded."""
    import torch

    torch.cuda.set_device(0)
    import pyxu_amd.abc as pxa
    import pyxu_amd.distributed as pd
    import pyxu_amd.operator as pxo
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd.util import to_device, to_NUMPY

    rng = np.random.default_rng(17)
    K = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    xs = np.zeros(N, np.float32)
    xs[rng.choice(N, 8, replace=False)] = rng.standard_normal(8)
    y = (K @ xs).astype(np.float32)
    lam, tau = 0.05, 1.0
    lo, hi = pd.shard_range(M)
    with pxrt.Precision(pxrt.Width.SINGLE):
        Ks = pd.RowShardedLinOp(to_device(K[lo:hi].copy()), M)
        f = 0.5 * pxo.SquaredL2Norm(dim=hi - lo).asloss(to_device(y[lo:hi].copy())) * Ks
        s = pxs.ADMM(f=f, h=lam * pxo.L1Norm(dim=N), show_progress=False)
        s.fit(x0=to_device(np.zeros(N, np.float32)), tau=tau, stop_crit=pxst.MaxIter(n_iter))
        out = dict(x=to_NUMPY(s.solution()))
        from pyxu_amd.opt.solver._normal import normal_form_ex

        Q = f._quad_spec()[0]
        nf = normal_form_ex(Q + pxo.HomothetyOp(cst=1 / tau, dim=N))
        out["sharded_normal"] = nf is not None and nf[3]
        if rank == 0:
            Kf = pxa.LinOp.from_array(to_device(K))
            f1 = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(to_device(y)) * Kf
            s1 = pxs.ADMM(f=f1, h=lam * pxo.L1Norm(dim=N), show_progress=False)
            s1.fit(x0=to_device(np.zeros(N, np.float32)), tau=tau, stop_crit=pxst.MaxIter(n_iter))
            out["x_ref"] = to_NUMPY(s1.solution())
    return out


def gpu_rccl_world1(rank, world, B, sh, iters, eps, M, N, n_iter):
    """The RCCL (``nccl`` backend) path of pyxu_amd.distributed on ONE GPU: a world-size-1 group with
    PXA_DIST_COLLECTIVES=always, so that every collective the sharded solvers issue is a real RCCL call on
    device buffers.  Returns the sharded results next to the unsharded ones, the collectives seen and
    whether librccl is mapped into the process."""
    import torch
    import torch.distributed as dist

    import pyxu_amd.abc as pxa
    import pyxu_amd.distributed as pd
    import pyxu_amd.operator as pxo
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd.util import to_device, to_NUMPY

    assert str(dist.get_backend()).lower() == "nccl" and pd.collectives_at_world1()
    calls = []
    ar0, ag0 = dist.all_reduce, dist.all_gather

    def all_reduce(t, *a, **k):
        calls.append(("all_reduce", bool(t.is_cuda)))
        return ar0(t, *a, **k)

    def all_gather(lst, t, *a, **k):
        calls.append(("all_gather", bool(t.is_cuda)))
        return ag0(lst, t, *a, **k)

    dist.all_reduce, dist.all_gather = all_reduce, all_gather
    out = {}
    # C5: batched PGD (fused kernel) with the global RelError all-reduced through RCCL vs the plain RelError
    rng = np.random.default_rng(13)
    n = int(np.prod(sh))
    ys = rng.standard_normal((B, n)).astype(np.float32)
    lam, mu = 0.02, 0.01

    def solve(crit):
        with pxrt.Precision(pxrt.Width.SINGLE):
            H = pxo.Gaussian(arg_shape=(B, *sh), sigma=(0, 2.0, 2.0))
            G = pxo.Gradient(arg_shape=(B, *sh), directions=(1, 2))
            f = 0.5 * pxo.SquaredL2Norm(dim=B * n).asloss(to_device(ys.reshape(-1))) * H + \
                lam * pxo.L21Norm(arg_shape=(2, B, *sh)).moreau_envelope(mu) * G
            f.diff_lipschitz = 1 + 8 * lam / mu
            s = pxs.PGD(f=f, g=pxo.PositiveOrthant(dim=B * n), show_progress=False)
            s.fit(x0=to_device(np.zeros(B * n, np.float32)), stop_crit=pxst.MaxIter(iters) | crit)
            assert s._plan is not None
            _, hist = s.stats()
            return s.solution(), int(hist["iteration"][-1])

    k0 = len(calls)
    x_sh, it_sh = solve(pd.ShardedRelError(eps=eps))
    out["pgd_collectives"] = calls[k0:]
    x_ref, it_ref = solve(pxst.RelError(eps=eps))
    g = pd.gather_slabs(x_sh.reshape(B, n), B)
    out.update(pgd_x=to_NUMPY(x_sh), pgd_x_ref=to_NUMPY(x_ref), pgd_it=it_sh, pgd_it_ref=it_ref, gathered=to_NUMPY(g),
               gathered_is_cuda=bool(g.is_cuda))
    # C4: RowShardedLinOp (adjoint = local adjoint + RCCL all-reduce) and ADMM through its sharded normal operator
    rng = np.random.default_rng(17)
    K = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float32)
    xs = np.zeros(N, np.float32)
    xs[rng.choice(N, 8, replace=False)] = rng.standard_normal(8)
    y = (K @ xs).astype(np.float32)
    z = rng.standard_normal((3, M)).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        Ks = pd.RowShardedLinOp(to_device(K.copy()), M)
        Kf = pxa.LinOp.from_array(to_device(K))
        k0 = len(calls)
        out["adj_sharded"] = to_NUMPY(Ks.adjoint(to_device(z)))
        out["adj_collectives"] = calls[k0:]
        out["adj_ref"] = to_NUMPY(Kf.adjoint(to_device(z)))
        f = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(to_device(y)) * Ks
        s = pxs.ADMM(f=f, h=0.05 * pxo.L1Norm(dim=N), show_progress=False)
        k0 = len(calls)
        s.fit(x0=to_device(np.zeros(N, np.float32)), tau=1.0, stop_crit=pxst.MaxIter(n_iter))
        out["admm_collectives"] = len(calls) - k0
        out["admm_x"] = to_NUMPY(s.solution())
        f1 = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(to_device(y)) * Kf
        s1 = pxs.ADMM(f=f1, h=0.05 * pxo.L1Norm(dim=N), show_progress=False)
        s1.fit(x0=to_device(np.zeros(N, np.float32)), tau=1.0, stop_crit=pxst.MaxIter(n_iter))
        out["admm_x_ref"] = to_NUMPY(s1.solution())
    dist.all_reduce, dist.all_gather = ar0, ag0
    with open("/proc/self/maps") as fh:
        out["rccl_libs"] = sorted({ln.split()[-1] for ln in fh if "rccl" in ln.lower() and "/" in ln})
    return out


def bench_prime_agreement(rank, world, budgets):
    """bench.prime_loop with a different time budget per rank: the ranks must still run the same
    number of steps (each stop check of the primed solver is a collective)."""
    import itertools
    import time

    import torch.distributed as dist

    import bench

    ctx = bench.Ctx(world, rank, dist, coll_device="cpu")

    def steps():
        for i in itertools.count():
            time.sleep(0.0005 * (rank + 1))  # ranks step at different speeds too
            yield i

    n = bench.prime_loop(ctx, steps(), budgets[rank], chunk=10)
    return {"n": n}
