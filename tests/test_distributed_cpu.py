"""
Multi-process (world_size 2, gloo, CPU) coverage of pyxu_amd.distributed — the N>1 host logic of
SURVEY.md §8(e): balanced slab partition, all-reduce / all-gather glue, the global RelError of
sharded batch-as-axis stacks (C5) and the row-sharded normal operator of ADMM/CG (C4).
The HIP kernels need a GPU, so the per-rank arithmetic here is the CPU oracle; the same scenarios
run on the MI355X through the real kernels in test_gpu_distributed.py.
"""
import socket

import numpy as np
import pytest

import oracle as orc
import pyxu_amd.distributed as pd

torch = pytest.importorskip("torch")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(scenario, world=2, **kwargs):
    import torch.multiprocessing as mp

    import _dist_workers

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dist_workers.run, args=(r, world, port, scenario, q, kwargs)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=240)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
    for r, out in res.items():
        assert "error" not in out, out.get("error")
    return res


@pytest.mark.parametrize("n,w", [(0, 1), (1, 2), (5, 2), (8, 8), (512, 8), (7, 3), (3, 8)])
def test_shard_range_partition(n, w):
    rs = [pd.shard_range(n, r, w) for r in range(w)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c
    sizes = [b - a for a, b in rs]
    assert max(sizes) - min(sizes) <= 1


def test_single_process_is_identity():
    t = torch.tensor([1.0, 2.0])
    assert pd.allreduce(t, "sum") is t
    assert pd.world() == (0, 1)
    assert pd.shard_range(10) == (0, 10)


def test_gloo_collectives_world2():
    res = spawn("collectives")
    for r in (0, 1):
        assert res[r]["sum"] == [3.0, 10.0]
        assert res[r]["max"] == [2.0, 10.0]
        np.testing.assert_array_equal(res[r]["gathered"], np.arange(5, dtype=np.float32)[:, None].repeat(3, 1))
        assert res[r]["crit_reduce"] == [[2.0], [4.0]]


def test_gloo_batched_pgd_global_stop_matches_unsharded():
    """Sharded C5 (5 images over 2 ranks, unequal slabs) == one process on the whole batch,
    including the iteration at which the global RelError stops."""
    B, sh, iters, eps = 5, (12, 16), 200, 1e-2
    res = spawn("batched_pgd_oracle", B=B, sh=sh, iters=iters, eps=eps)
    # unsharded reference: same arithmetic over the whole batch, one process
    rng = np.random.default_rng(11)
    N = int(np.prod(sh))
    ys = rng.standard_normal((B, N)).astype(np.float32)
    lam, mu = 0.02, 0.01
    taps, c = orc.gaussian_taps(2.0, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    tau = np.float32(1 / np.float32(1 + 8 * lam / mu))
    x = np.zeros((B, N), np.float32)
    xp = x.copy()
    stopped = None
    for k in range(iters):
        a = np.float32(k / (k + 1 + 75))
        yk = (x - xp) * a + x
        z = np.stack([yk[i] - tau * orc.deblur_tv_grad(yk[i], blur, ys[i], lam, mu, dict(arg_shape=sh)) for i in range(B)])
        xn = np.maximum(z, 0).astype(np.float32)
        num = ((xn.astype(np.float64) - x) ** 2).sum() ** 0.5
        den = (x.astype(np.float64) ** 2).sum() ** 0.5
        xp, x = x, xn
        if k > 0 and num <= eps * den:
            stopped = k
            break
    assert stopped is not None
    for r in (0, 1):
        assert res[r]["stopped_at"] == stopped
        np.testing.assert_array_equal(res[r]["x"], x)


def test_gloo_row_sharded_normal_cg_matches_unsharded():
    M, N = 48, 40
    res = spawn("row_sharded_normal_cg", M=M, N=N, iters=60)
    rng = np.random.default_rng(5)
    K = (rng.standard_normal((M, N)) / np.sqrt(M)).astype(np.float64)
    b = rng.standard_normal(N)
    x_ref, n_ref = orc.cg(lambda p: (K.T @ (K @ p.T)).T + p / 0.7, b[None, :], max_iter=60)
    for r in (0, 1):
        assert np.linalg.norm(res[r]["x"] - x_ref) <= 1e-10 * np.linalg.norm(x_ref)
    np.testing.assert_array_equal(res[0]["x"], res[1]["x"])  # replicated CG vectors stay identical


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind,halo", [("blur", (3, 3)), ("grad", (0, 1))])
def test_gloo_slab_halo_exchange_matches_global(world, kind, halo):
    """Halo-exchanged slab decomposition: apply / adjoint of each rank's slab,
    gathered, equal the global operator (zero boundary); world 3 exercises a rank with two
    neighbours.  Gaussian sigma=1 has reach 3 planes; the forward difference reaches 1 plane ahead."""
    shape = (10, 6, 7)
    res = spawn("slab_halo_oracle", world=world, shape=shape, kind=kind, halo=halo)
    x, y = res[0]["x"], res[0]["y"]
    if kind == "grad":
        ref_a, ref_t = orc.gradient_apply(x, shape), orc.gradient_adjoint(y, shape)
    else:
        taps, c = orc.gaussian_taps(1.0, 3.0, np.float64)
        kw = dict(kernel=[taps] * 3, center=[c] * 3)
        ref_a, ref_t = orc.stencil_apply(x, shape, **kw), orc.stencil_adjoint(y, shape, **kw)
    for r in range(world):
        np.testing.assert_allclose(res[r]["apply"], ref_a, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(res[r]["adjoint"], ref_t, rtol=1e-12, atol=1e-12)


def test_bench_prime_loop_ranks_agree_on_step_count():
    """bench.py's untimed priming: ranks with different clocks / budgets run the same number of steps,
    so no rank blocks in a stop-check collective that the others never reach (the N>1 bench hang)."""
    res = spawn("bench_prime_agreement", budgets=[0.05, 0.3])
    assert res[0]["n"] == res[1]["n"] and res[0]["n"] >= 10
