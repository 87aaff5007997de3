#!/usr/bin/env python3
"""
Benchmark: PGD solver iterations/s on TV-regularised deblurring (BASELINE.json metric).

Headline workload (BASELINE.json configs[1], C2): 2048 x 2048 image, H = Gaussian(sigma=2) blur (13
taps/axis, zero boundary), f = 1/2||H x - y||^2 + lam * env_mu(L21) o Gradient, g = PositiveOrthant,
lam = mu = 0.01, fp32, synthetic piecewise-constant phantom + 1% noise.  One
"step" = one PGD iteration (Solver._step: stop check every `stop_rate` iterations + m_step) driven
through the pyxu_amd Solver API in MANUAL mode.  `stop_rate` defaults to the largest divisor of
--steps that is <= 50, so the timed window holds exactly steps/stop_rate stop checks and
`ms_per_step` carries their amortised cost.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (no WORLD_SIZE in the environment)
launches N child ranks itself before touching the GPU (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set per child); under torch.distributed.run each process is one
rank.  Every rank solves its own 2048^2 image (independent problems, no data-path collective; the
ranks' images form one batch-as-axis problem for the GLOBAL RelError: one RCCL all-reduce of 2
doubles per stop check) -> weak scaling; value = total image-iterations/s = ranks * K / max_rank(t).

Sub-records on the same line (north_star):
  "stop_rate_1": the headline workload at the reference's default stop_rate = 1 (--sr1-steps, default 200 timed steps);
  "c2_4096": the same PGD at 4096^2 (SURVEY §7's stand-in for the infeasible 4096^3 north_star volume);
  "c5": configs[4], 512 independent 512^2 TV-deblur images as ONE (512, 512, 512) batch-as-axis
        problem sharded over the ranks (512 / N images each: strong scaling), global RelError;
  "c4": configs[3], ADMM with a dense 8192 x 65536 K (MFMA/GEMV dense path) + lam L1; K row-sharded
        over the ranks (one RCCL all-reduce of the 65536-vector per CG iteration);
  "c3": configs[2], PD3O and Condat-Vu on a 1024^3 volume (Gaussian S, anisotropic TV), with the
        per-kernel times of the fused look-ahead step, two launches per iteration: kernel B and kernel D
        (--c3-three-launch: the three-launch step A / B / C; single GPU: replicas only at N > 1);
  "k4": SURVEY §8(d)'s "Gradient + prox" kernel alone (pxa_tv_dual_update) at 2048^2 and 1024^3;
  "dense_mfma": the dense LinOp's MFMA path (8192 x 65536 K, B = 64 / 128 right-hand sides) in TFLOP/s.
Every sub-record (c2_4096, c5, c4, c3 per algorithm, k4 per shape, dense_mfma) carries a `cpu_baseline`: the
oracle (or, for dense_mfma, NumPy's matmul, which is the reference's dense apply) on the host's cores, a bounded
sample whose size and scaling the record states.

Roofline convention.  `frac` is the dominant kernel's time against ITS OWN compulsory bytes (every array
it must read or write, once): the fused PGD launch reads x, x_prev, H^T y and writes x_new = 16 B/pixel.  `frac_survey` keeps SURVEY §8(d)'s 48 B/pixel figure for the same time; that model is not a
bound on a one-launch kernel (it charges intermediates this kernel never materialises).  The kernel's
time (`kernel_ms`) comes from HIP events on its launch stream over a window of K more launches of the same
solver right after the timed region: a timing event anywhere in a window makes the runtime timestamp every
dispatch in it (~1.3 us per 24 us PGD launch, profiles/r04p_timer_ab.txt), so `kernel_ms` carries that
overhead (an upper bound) while the timed region -- hence `value` and `ms_per_step` -- does not
(--kernel-timer-in-region puts the window inside the region, as rounds 1-3 did).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
KERNEL = "pgd_tv2d_kernel"
SURVEY_BYTES_PER_PIXEL = 48  # 8 reads + 4 writes of fp32 per pixel per PGD iteration
MFMA_F32_PEAK_TF = 157.3  # dense fp32 MFMA peak (MI355X_MICROARCH.md, Matrix cores: = the f32 vector peak)
CPU_THREADS_MAX = 16  # the GPU box's CPU share per GPU (gpurun: 16)
# pxa_pgd_tv2d_last_kernel() -> (mode name, own compulsory bytes per pixel): the arrays the launch reads / writes
PGD_MODES = {1: ("x, x_prev, H^T y -> x_new (tile kernel)", 16), 2: ("x, x_prev, H^T y -> x_new (strip kernel)", 16),
             3: ("x, x_prev, H^T y -> x_new (pipelined kernel)", 16)}
PGD_KERNELS = {1: "pgd_tv2d_kernel", 2: "pgd_strip_kernel", 3: "pgd_pipe_kernel"}  # the rocprof name of each mode's kernel


# ----------------------------------------------------------------------------- launcher (no GPU here)
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, port, base=None):
    """Per-child environments of the self-launch (one rank per GPU, rendezvous on 127.0.0.1)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PXA_BENCH_CHILD="1")
        envs.append(e)
    return envs


def launch(argv, n, script=None):
    """Start `n` ranks of this script as child processes and wait for them; rank 0's stdout is ours.
    The parent never initialises the GPU (so no exec-after-GPU-init hazard) and forwards the worst
    exit status; if one rank fails, the others are stopped (they would block in a collective)."""
    envs = rank_envs(n, _free_port())
    cmd = [sys.executable, script or os.path.abspath(__file__), *argv]
    procs = [subprocess.Popen(cmd, env=e, stdout=None if r == 0 else subprocess.DEVNULL) for r, e in enumerate(envs)]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


# ----------------------------------------------------------------------------- workloads
def phantom(shape, rng):
    x = np.zeros(shape, dtype=np.float32)
    for _ in range(12):
        lo = [int(rng.integers(0, n // 2)) for n in shape]
        hi = [l + int(rng.integers(n // 8 + 1, n // 2 + 1)) for l, n in zip(lo, shape)]
        x[tuple(slice(l, h) for l, h in zip(lo, hi))] = rng.uniform(0.2, 1.0)
    return x


def build_problem(n0, n1, seed, lam=0.01, mu=0.01, sigma=2.0):
    """C2: f = 1/2||H.-y||^2 + lam env_mu(L21) o Grad, g = PositiveOrthant on one n0 x n1 image."""
    import pyxu_amd.operator as pxo
    import pyxu_amd.runtime as pxrt
    from pyxu_amd import _dev
    from pyxu_amd.util import to_device

    sh = (n0, n1)
    N = n0 * n1
    rng = np.random.default_rng(seed)
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=sigma, truncate=3.0)
        x_gt = to_device(phantom(sh, rng).reshape(-1))
        y = H.apply(x_gt)
        noise = to_device((0.01 * rng.standard_normal(N)).astype(np.float32))
        y = _dev.axpby(1.0, y, 1.0, noise)
        G = pxo.Gradient(arg_shape=sh)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * G
        f.diff_lipschitz = 1.0 + (lam / mu) * 8.0  # ||H||^2 + lam/mu ||Grad||^2, set analytically (§8(d))
        g = pxo.PositiveOrthant(dim=N)
    return f, g, y


def build_batch_problem(B, n, first, seed, lam=0.01, mu=0.01, sigma=2.0):
    """C5 slab: images [first, first + B) of the global batch as one (B, n, n) batch-as-axis problem
    (size-1 taps on axis 0, Gradient(directions=(1, 2)), distinct y per image)."""
    import pyxu_amd.operator as pxo
    import pyxu_amd.runtime as pxrt
    from pyxu_amd import _dev
    from pyxu_amd.util import to_device

    sh = (B, n, n)
    N = B * n * n
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=(0, sigma, sigma), truncate=3.0)
        x_gt = np.empty((B, n, n), dtype=np.float32)
        for b in range(B):  # image i's phantom depends only on (seed, i): identical for every N
            x_gt[b] = phantom((n, n), np.random.default_rng((seed, first + b)))
        y = H.apply(to_device(x_gt.reshape(-1)))
        noise = np.random.default_rng((seed, first, 1)).standard_normal(N, dtype=np.float32) * np.float32(0.01)
        y = _dev.axpby(1.0, y, 1.0, to_device(noise))
        G = pxo.Gradient(arg_shape=sh, directions=(1, 2))
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * G
        f.diff_lipschitz = 1.0 + (lam / mu) * 8.0
        g = pxo.PositiveOrthant(dim=N)
    return f, g


def auto_stop_rate(steps, cap=50):
    """Largest divisor of `steps` that is <= cap: a window of `steps` consecutive iterations then holds
    exactly steps / stop_rate stop checks wherever it starts."""
    for r in range(min(cap, max(steps, 1)), 0, -1):
        if steps % r == 0:
            return r
    return 1


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def measured_traffic(kernel, key):
    """(HBM bytes per launch, provenance) of `kernel` on workload `key` from the committed rocprofv3 PMC
    passes (profiles/traffic.json, written by scripts/pmc_traffic.py: (2 * FETCH_SIZE + WRITE_SIZE) * 1024,
    the gfx950 correction of MI355X_MICROARCH.md §HBM), or (None, reason).  NOT measured in this run: the
    counters need their own profiler passes (scripts/gpu_r03.sh)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            tab = json.load(fh)
    except (OSError, ValueError):
        return None, "no profiles/traffic.json"
    ent = tab.get(f"{kernel}@{key}")
    if ent is None:
        return None, f"no PMC profile of {kernel}@{key} in profiles/traffic.json"
    return ent.get("hbm_bytes_per_launch"), (f"profiles/traffic.json[{kernel}@{key}] (rocprofv3 PMC pass "
                                             f"{ent.get('tag', '?')}, not this run)")


def cpu_baseline(n0, n1, seed, budget_s, threads, lam=0.01, mu=0.01, sigma=2.0):
    """Oracle (NumPy restatement of the reference PGD path) on the host: same problem; as many PGD
    iterations as fit in about `budget_s` seconds (bounded sample; at least 2).  threads = 1: the
    single-thread oracle (oracle.pgd); threads > 1: its slab-parallel form (oracle.parallel, the
    Dask-map_overlap-style split of the reference, bit-identical results)."""
    import oracle as orc
    from oracle.parallel import pgd_tv_threaded

    sh = (n0, n1)
    N = n0 * n1
    rng = np.random.default_rng(seed)
    taps, c = orc.gaussian_taps(sigma, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    x_gt = phantom(sh, rng).reshape(-1)
    y = orc.stencil_apply(x_gt, sh, [taps, taps], [c, c])
    y = (y + (0.01 * rng.standard_normal(N)).astype(np.float32)).astype(np.float32)
    tau = np.float32(1 / np.float32(1.0 + (lam / mu) * 8.0))
    x0 = np.zeros(N, dtype=np.float32)
    if threads == 1:
        grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
        prox = lambda z, t: orc.positive_orthant_prox(z)
        run = lambda k: orc.pgd(x0, grad, prox, tau, k)
    else:
        run = lambda k: pgd_tv_threaded(x0, blur, y, lam, mu, orc.positive_orthant_prox, tau, k, threads)
    t0 = time.perf_counter()
    run(1)  # warm-up (page-in, allocator) and per-iteration estimate
    t1 = time.perf_counter() - t0
    iters = int(max(2, min(2000, budget_s / max(t1, 1e-3))))
    t0 = time.perf_counter()
    run(iters)
    dt = time.perf_counter() - t0
    return iters / dt, iters, dt


def cpu_threads():
    return max(1, min(CPU_THREADS_MAX, os.cpu_count() or 1))


def cpu_baseline_c5(n, images, seed, budget_s, threads, lam=0.01, mu=0.01, sigma=2.0):
    """C5 (independent n x n TV-deblur images, each its own y): the oracle PGD on `images` of them, one image per
    worker thread (oracle.parallel.pgd_tv_images_threaded); image-iterations/s is size-independent in the
    number of images, so a bounded sample of the 512-image batch measures the batch's rate."""
    import oracle as orc
    from oracle.parallel import pgd_tv_images_threaded

    sh = (n, n)
    taps, c = orc.gaussian_taps(sigma, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    ys = []
    for i in range(images):
        rng = np.random.default_rng((seed, i))
        y = orc.stencil_apply(phantom(sh, rng).reshape(-1), sh, [taps, taps], [c, c])
        ys.append((y + (0.01 * rng.standard_normal(n * n)).astype(np.float32)).astype(np.float32))
    x0s = [np.zeros(n * n, np.float32)] * images
    tau = np.float32(1 / np.float32(1.0 + (lam / mu) * 8.0))
    pos = lambda z, t: orc.positive_orthant_prox(z)
    t0 = time.perf_counter()
    pgd_tv_images_threaded(x0s, blur, ys, lam, mu, pos, tau, 1, threads)
    t1 = time.perf_counter() - t0
    iters = int(max(2, min(500, budget_s / max(t1, 1e-3))))
    t0 = time.perf_counter()
    pgd_tv_images_threaded(x0s, blur, ys, lam, mu, pos, tau, iters, threads)
    dt = time.perf_counter() - t0
    return images * iters / dt, iters, dt


def cpu_baseline_c4(M, N, threads, steps=4, lam=0.01):
    """C4: CG steps of the ADMM x-update (QuadraticFunc.prox, operator.py:1273-1291 -> cg.py:125-153) on the
    host: the oracle's CG (oracle.cg) on K^T K + I/tau with NumPy BLAS on `threads` threads, a dense M x N fp32 K
    generated on the host.  Returns (ms per CG iteration, BLAS threads actually used)."""
    import oracle as orc

    try:
        from threadpoolctl import threadpool_info, threadpool_limits
    except ImportError:  # pragma: no cover
        threadpool_limits, threadpool_info = None, None
    rng = np.random.default_rng(5)
    K = rng.standard_normal((M, N), dtype=np.float32)
    K *= np.float32(1.0 / np.sqrt(M))
    b = rng.standard_normal(N).astype(np.float32)
    A = lambda p: (K.T @ (K @ p.T)).T.astype(p.dtype) + np.float32(1.0) * p
    ctxm = threadpool_limits(limits=threads, user_api="blas") if threadpool_limits else None
    try:
        used = max((i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"), default=1) \
            if threadpool_info else threads
        orc.cg(A, b, max_iter=1)  # page-in, BLAS warm-up
        t0 = time.perf_counter()
        orc.cg(A, b, eps=0.0, max_iter=1)
        t1 = time.perf_counter()
        orc.cg(A, b, eps=0.0, max_iter=1 + steps)
        t2 = time.perf_counter()
    finally:
        if ctxm is not None:
            ctxm.restore_original_limits()
    return 1e3 * ((t2 - t1) - (t1 - t0)) / steps, used


def cpu_baseline_k4(shape, budget_s, sigma=0.28, lam=0.01, rho=1.0, seed=11):
    """K4 (the PDS dual update z <- (1 - rho) z + rho fenchel_prox_{sigma lam L1}(z + sigma Grad w), the
    reference's Moreau form, operator.py:940-944 + diff.py Gradient + norm.py:47-52) with the oracle on one host
    thread, on `shape`.  Returns (ms per update, updates timed, seconds)."""
    import oracle as orc

    rng = np.random.default_rng(seed)
    n = int(np.prod(shape))
    w = rng.standard_normal(n).astype(np.float32)
    z = rng.standard_normal(len(shape) * n).astype(np.float32)
    prox = lambda v, t: orc.l1_prox(v, lam * t)

    def update():
        zin = z + np.float32(sigma) * orc.gradient_apply(w, shape)
        return np.float32(1 - rho) * z + np.float32(rho) * orc.fenchel_prox(prox, zin.astype(np.float32), sigma)

    update()  # page-in
    k, t0 = 0, time.perf_counter()
    while k < 1 or time.perf_counter() - t0 < budget_s:
        update()
        k += 1
    dt = time.perf_counter() - t0
    return 1e3 * dt / k, k, dt


def cpu_baseline_mfma(M, N, B, threads):
    """dense_mfma: the dense LinOp's stacked apply Y = X K^T (base.py:334-512, NumPy's matmul on the host)
    for B right-hand sides, fp32 BLAS on `threads` threads.  Returns (ms per apply, TFLOP/s, BLAS threads)."""
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
    except ImportError:  # pragma: no cover
        threadpool_limits, threadpool_info = None, None
    K = np.full((M, N), 0.5, dtype=np.float32)  # (BLAS time does not depend on the values)
    X = np.full((B, N), 0.25, dtype=np.float32)
    ctxm = threadpool_limits(limits=threads, user_api="blas") if threadpool_limits else None
    try:
        used = max((i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"), default=1) \
            if threadpool_info else threads
        X @ K.T  # page-in, BLAS warm-up
        t0 = time.perf_counter()
        for _ in range(3):
            X @ K.T
        ms = 1e3 * (time.perf_counter() - t0) / 3
    finally:
        if ctxm is not None:
            ctxm.restore_original_limits()
    return ms, 2.0 * M * N * B / (ms * 1e-3) / 1e12, used


def cpu_baseline_c3(n, budget_s, seed=7, lam=0.01, sigma=2.0):
    """C3 (PD3O / Condat-Vu, S = Gaussian(sigma) 3-D blur, K = Gradient, h = lam L1, g = None): the oracle's
    pd3o / condat_vu (pds.py:722-761, 429-442 restated in NumPy, one thread) on an n^3 volume of the same
    problem.  Every operator of the step is an O(voxels) stencil, so the per-voxel cost is size-independent and
    the 1024^3 iteration time is voxels(1024^3) / (voxel-iterations/s of the sample).  Per algorithm: one
    iteration (set-up + page-in), then as many as fit in `budget_s` (at least 1), timed as the difference.
    Returns {algo: (voxel-iterations/s, timed iterations, seconds)}."""
    import oracle as orc

    sh = (n, n, n)
    N = n ** 3
    rng = np.random.default_rng(seed)
    taps, c = orc.gaussian_taps(sigma, 3.0, np.float32)
    K3, C3 = [taps] * 3, [c] * 3
    x_gt = np.zeros(sh, np.float32)
    for _ in range(12):  # piecewise-constant phantom, as bench_c3
        lo = [int(rng.integers(0, n // 2)) for _ in sh]
        hi = [v + int(rng.integers(n // 8 + 1, n // 2 + 1)) for v in lo]
        x_gt[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = float(rng.uniform(0.2, 1.0))
    y = orc.stencil_apply(x_gt.reshape(-1), sh, K3, C3)
    y = (y + (0.01 * rng.standard_normal(N)).astype(np.float32)).astype(np.float32)
    blur = dict(arg_shape=sh, kernel=K3, center=C3)
    grad_f = lambda v: orc.deblur_tv_grad(v, blur, y, 0.0, 1.0, dict(arg_shape=sh))
    Kf = lambda v: orc.gradient_apply(v, arg_shape=sh)
    KT = lambda v: orc.gradient_adjoint(v, arg_shape=sh)
    lam32 = np.float32(lam)
    fprox = lambda v, s_: orc.fenchel_prox(lambda a, t: orc.l1_prox(a, t * lam32), v, s_)
    x0 = np.zeros(N, np.float32)
    out = {}
    for algo in ("pd3o", "cv"):
        if algo == "pd3o":
            tau, sig, _, rho = orc.pd3o_step_sizes(1.0, np.sqrt(12.0), np.float32)
            run = lambda k: orc.pd3o(x0, grad_f, None, Kf, KT, fprox, tau, sig, rho, k)
        else:
            tau, sig, _, rho = orc.condat_vu_step_sizes(1.0, np.sqrt(12.0), np.float32)
            run = lambda k: orc.condat_vu(x0, grad_f, None, Kf, KT, fprox, tau, sig, rho, k)
        t0 = time.perf_counter()
        run(1)
        t1 = time.perf_counter() - t0
        k = int(max(1, min(50, budget_s / max(t1, 1e-3))))
        t0 = time.perf_counter()
        run(1 + k)
        dt = time.perf_counter() - t0 - t1
        dt = dt if dt > 0 else time.perf_counter() - t0
        out[algo] = (N * k / dt, k, dt)
    return out


# ----------------------------------------------------------------------------- timing helpers
class Ctx:
    """Rank bookkeeping of one bench process; the scalar collectives run on the GPU under RCCL and on
    the host under gloo (CPU rehearsals and tests)."""

    def __init__(self, world, rank, dist, coll_device="cuda"):
        self.world, self.rank, self.dist, self.coll_device = world, rank, dist, coll_device

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def _reduce(self, v, op):
        import torch

        t = torch.tensor([float(v)], dtype=torch.float64, device=self.coll_device)
        if self.world > 1:
            self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max_over_ranks(self, v):
        return self._reduce(v, self.dist.ReduceOp.MAX if self.world > 1 else None)

    def sum_over_ranks(self, v):
        return self._reduce(v, self.dist.ReduceOp.SUM if self.world > 1 else None)


def prime_loop(ctx, gen, seconds, chunk=200, sync=None):
    """Untimed priming: run `chunk` steps at a time until `seconds` have passed.  Every continue/stop
    decision is agreed over the ranks (max of the per-rank "time left" flags), so all ranks run the
    same number of steps: each stop check of a distributed solver is a collective, and ranks that ran
    different step counts would block in it.  Returns the number of steps run."""
    n = 0
    t_end = time.perf_counter() + seconds
    while ctx.max_over_ranks(1.0 if time.perf_counter() < t_end else 0.0) > 0:
        for _ in range(chunk):
            next(gen)
        n += chunk
        if sync is not None:
            sync()
    return n


def timed_steps(ctx, gen, warmup, steps, timer=None):
    """W untimed steps, then exactly `steps` steps bracketed by barrier + synchronize on both sides;
    returns the max-over-ranks elapsed seconds."""
    import torch

    from pyxu_amd import _dev

    for _ in range(warmup):
        next(gen)
    torch.cuda.synchronize()
    ctx.barrier()
    if timer is not None:
        _dev.set_launch_timer(timer)
    t0 = time.perf_counter()
    for _ in range(steps):
        next(gen)
    if timer is not None:
        timer.close()  # close the last window right behind the last launch (before the host sync)
    torch.cuda.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    _dev.set_launch_timer(None)
    return ctx.max_over_ranks(elapsed)


def run_pgd(ctx, f, g, stop_rate, warmup, steps, fused, prime_s=0.0, kernel_timer=True):
    """Build a PGD solver in MANUAL mode on (f, g), prime the device, time `steps` steps."""
    import torch

    import pyxu_amd.abc as pxa
    import pyxu_amd.distributed as pdist
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    from pyxu_amd import _dev

    like = torch.empty((1,), dtype=torch.float32, device="cuda")

    def new_solver():
        s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=stop_rate)
        rel = pdist.ShardedRelError(eps=1e-30) if ctx.world > 1 else pxst.RelError(eps=1e-30)
        s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10**9) | rel, mode=pxa.Mode.MANUAL, fused=fused)
        return s, rel

    if prime_s > 0:
        # untimed device priming on a throwaway solver of the same problem: code objects loaded, clocks
        # and caches at steady state before the measured solver's W + K steps (which it does not change)
        s, _ = new_solver()
        gen = s.steps()
        prime_loop(ctx, gen, prime_s, sync=torch.cuda.synchronize)
        del s, gen
    slvr, rel = new_solver()
    # prime the stop-check path once (loads its kernels' code objects) so that a warmup shorter than
    # stop_rate does not leave one-time module loading inside the timed region
    rel.stop({"x": slvr._mstate["x"]})
    rel.stop({"x": slvr._mstate["x"]})
    rel.clear()
    fused_on = slvr._plan is not None
    gen = slvr.steps()
    timer = _dev.LaunchTimer(single=True) if (kernel_timer == "in_region" and fused_on) else None
    elapsed = timed_steps(ctx, gen, warmup, steps, timer)
    if kernel_timer is True and fused_on:
        # the kernel's average launch duration, HIP events on its own stream over a window of `steps` more
        # launches of the same solver right after the timed region: a timing event anywhere in a window makes
        # the runtime timestamp every dispatch of it, ~1.3 us per launch here (profiles/r04p_timer_ab.txt),
        # so the events are kept out of the region the value is measured on (--kernel-timer-in-region:
        # inside it, as rounds 1-3 did)
        timer = _dev.LaunchTimer(single=True)
        torch.cuda.synchronize()
        _dev.set_launch_timer(timer)
        for _ in range(steps):
            next(gen)
        timer.close()
        _dev.set_launch_timer(None)
    kern_ms = timer.mean_ms() if timer is not None else None
    return elapsed, kern_ms, slvr, (timer.launches if timer is not None else 0)


def last_pgd_mode():
    """(mode name, own bytes per pixel) of the fused PGD launch this thread made last."""
    from pyxu_amd._lib import lib

    return PGD_MODES.get(int(lib.pxa_pgd_tv2d_last_kernel()), ("none", 16))


def pxa_lag_depth():
    import pyxu_amd.abc as pxa

    return int(pxa.Solver._LAG)


def last_pgd_kernel():
    """rocprof name of the fused PGD kernel this thread launched last (tile or strip kernel)."""
    from pyxu_amd._lib import lib

    return PGD_KERNELS.get(int(lib.pxa_pgd_tv2d_last_kernel()), KERNEL)


def roofline(pixels, kern_ms, own_bpp, traffic_key, kernel=None, mode=""):
    """The dominant kernel against its own compulsory bytes (frac) and SURVEY §8(d)'s figure (frac_survey)."""
    kernel = kernel or last_pgd_kernel()
    own = own_bpp * pixels
    achieved = own / (kern_ms * 1e-3) / 1e9
    surv = SURVEY_BYTES_PER_PIXEL * pixels
    traffic, src = measured_traffic(kernel, traffic_key)
    rec = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src, "kernel": kernel,
           "mode": mode, "kernel_ms": round(kern_ms, 5), "bytes_per_launch": own,
           "bytes_model": f"own compulsory streams, {own_bpp} B/pixel",
           "frac_survey": round(surv / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "survey_bytes_per_launch": surv}
    if achieved > HBM_PEAK_GBS:  # only possible when the working set is served from the Infinity Cache
        rec["note"] = "above the HBM peak: working set resident in the 256 MiB Infinity Cache"
    return rec


def bench_c2_4096(ctx, args):
    """SURVEY §7's 4096^2 stand-in for the infeasible 4096^3 north_star volume: the headline PGD problem at
    4096 x 4096 (one image per rank), same solver loop and stop criteria."""
    import pyxu_amd.runtime as pxrt

    n = 4096
    f, g, _ = build_problem(n, n, seed=4321 + ctx.rank)
    K = args.c4096_steps
    sr = auto_stop_rate(K)
    with pxrt.Precision(pxrt.Width.SINGLE):
        elapsed, kern_ms, slvr, launches = run_pgd(ctx, f, g, sr, 5, K, True)
    mode, bpp = last_pgd_mode()
    rec = {"workload": f"PGD {n}x{n} Gaussian(sigma=2) deblur + lam*env_mu(L21 o Grad) TV, PositiveOrthant",
           "scaling": "weak", "steps": K, "warmup": 5, "stop_rate": sr, "value": round(ctx.world * K / elapsed, 2),
           "unit": "image-iterations/s", "ms_per_step": round(1e3 * elapsed / K, 4)}
    if kern_ms is not None:
        kern_ms = ctx.max_over_ranks(kern_ms)
        rec["roofline"] = roofline(n * n, kern_ms, bpp, f"{n}x{n}", mode=mode)
        rec["roofline"]["launches_timed"] = launches
    del slvr, f, g
    return rec


# (own compulsory B/voxel of the fused step, SURVEY §8(d) B/voxel): the look-ahead step (pxa_pds_step_la,
# default) and the three-launch step (pxa_pds_step, --c3-three-launch)
C3_BYTES = {True: {"pd3o": (64, 80), "cv": (64, 68)}, False: {"pd3o": (76, 80), "cv": (68, 68)}}
C3_KERNELS = {
    True: ("pds_march_kernel (priming march; absent from primed steps)",
           "pds_plane_kernel (B: in-plane G + point-wise update)",
           "pds_march_kernel (D: z + sigma grad w, fenchel prox, relaxation + the next iteration's axis-0 march)"),
    False: ("pds_axis0_kernel (A: axis-0 march of S0 / S0^T)", "pds_plane_kernel (B: in-plane G + point-wise update)",
            "pds_dual_kernel (C: z + sigma grad w, fenchel prox, relaxation)")}
# own compulsory bytes per voxel of each kernel.  Three-launch: PD3O A u,z(3) in x,Q out;
# B Q,x,u,S^T y in w,u+ out; C w,z(3) in z+(3) out.  CV: A x in Q out; B Q,x,S^T y,z(3) in w,x+ out; C as PD3O.
# Look-ahead: B as above but CV reads K^T z (1 field) instead of z (3); D w,z(3),u+ (CV x+) in z+(3),Q and
# x+ (CV K^T z+) out; the priming march reads u (x), z(3) and writes x (K^T z), Q.
C3_KERNEL_BYTES = {True: {"pd3o": (24, 24, 40), "cv": (24, 24, 40)}, False: {"pd3o": (24, 24, 28), "cv": (8, 32, 28)}}


def bench_c3(ctx, args):
    """configs[2]: PD3O and Condat-Vu on an n^3 volume, S = Gaussian(sigma=2) (13 taps/axis, zero boundary),
    K = Gradient (3 directions), h = lam L1 (anisotropic TV), g = None, fp32; the phantom and the noise are
    generated on the device.  Driven through the Solver API (MANUAL mode, one stop check per window);
    per-kernel times from HIP events recorded inside pxa_pds_step (TUNE_PDS_EVENTS)."""
    import shutil

    import torch

    import pyxu_amd.abc as pxa
    import pyxu_amd.operator as pxo
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd import _dev

    n, K = args.c3_n, args.c3_steps
    la = not args.c3_three_launch
    sh = (n, n, n)
    N = n ** 3
    out = {"workload": f"{n}^3 volume, S = Gaussian(sigma=2), K = Gradient (3 dirs), h = 0.01 L1 (anisotropic TV), g = None",
           "scaling": "replicas (one volume per GPU)", "steps": K}
    gen = torch.Generator(device="cuda").manual_seed(7)
    x_gt = torch.zeros(sh, device="cuda", dtype=torch.float32)
    rng = np.random.default_rng(7)
    for _ in range(12):  # piecewise-constant phantom, written on the device
        lo = [int(rng.integers(0, n // 2)) for _ in sh]
        hi = [l + int(rng.integers(n // 8 + 1, n // 2 + 1)) for l in lo]
        x_gt[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = float(rng.uniform(0.2, 1.0))
    with pxrt.Precision(pxrt.Width.SINGLE):
        S = pxo.Gaussian(arg_shape=sh, sigma=2.0, truncate=3.0)
        y = S.apply(x_gt.reshape(-1))
        del x_gt
        y = _dev.axpby(1.0, y, 0.01, torch.randn(N, device="cuda", dtype=torch.float32, generator=gen), out=y)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * S
        f.diff_lipschitz = 1.0  # ||S||^2 <= 1 for the normalised Gaussian (set analytically, §8(d))
        Kop = pxo.Gradient(arg_shape=sh)
        h = 0.01 * pxo.L1Norm(dim=3 * N)
        for algo, klass in (("pd3o", pxs.PD3O), ("cv", pxs.CondatVu)):
            s = klass(f=f, g=None, h=h, K=Kop, show_progress=False, stop_rate=K)
            s._LOOKAHEAD = la
            s.fit(x0=torch.zeros(N, device="cuda", dtype=torch.float32), stop_crit=pxst.MaxIter(10 ** 9) | pxst.RelError(eps=1e-30),
                  mode=pxa.Mode.MANUAL)
            it = s.steps()
            for _ in range(2):
                next(it)
            torch.cuda.synchronize()
            prev = _dev.tuning(_dev.TUNE_PDS_EVENTS, 1)
            _dev.pds_kernel_ms(reset=True)
            try:
                elapsed = timed_steps(ctx, it, 0, K)
                nrec, ms = _dev.pds_kernel_ms(reset=True)
            finally:
                _dev.tuning(_dev.TUNE_PDS_EVENTS, prev)
            own, surv = C3_BYTES[la][algo]
            step_ms = 1e3 * elapsed / K
            rec = {"value": round(K / elapsed, 3), "unit": "iterations/s", "ms_per_step": round(step_ms, 3),
                   "fused_m_step": s._plan is not None, "lookahead": bool(s._plan and s._plan["la"]), "stop_rate": K,
                   "frac_step_own": round(own * N / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "frac_step_survey": round(surv * N / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
            if nrec > 0:
                kms = [m / nrec for m in ms]
                rec["kernels"] = []
                for name, t, b in zip(C3_KERNELS[la], kms, C3_KERNEL_BYTES[la][algo]):
                    if la and name.startswith("pds_march_kernel (priming") and t < 0.01 * sum(kms):
                        continue  # primed steps run no priming march (the window holds two back-to-back events)
                    ach = b * N / (t * 1e-3) / 1e9 if t > 0 else 0.0
                    ent = {"kernel": name, "kernel_ms": round(t, 4), "bytes_per_voxel": b,
                           "achieved": round(ach, 1), "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}
                    short = name.split(" ")[0]
                    if la and short in ("pds_plane_kernel", "pds_march_kernel") and not name.startswith("pds_march_kernel (priming"):
                        tr, src = measured_traffic(f"{short}_{algo}", f"{n}^3")
                        ent["traffic"], ent["traffic_source"] = tr, src
                        if tr:
                            ent["traffic_bytes_per_voxel"] = round(tr / N, 2)
                    rec["kernels"].append(ent)
                kt = sum(kms)
                rec["roofline"] = {"bound": "hbm", "achieved": round(own * N / (kt * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(own * N / (kt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "traffic": None, "kernel_ms": round(kt, 4), "bytes_model": f"{own} B/voxel, the fused step's own compulsory bytes",
                                   "frac_survey": round(surv * N / (kt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
            out[algo] = rec
            shutil.rmtree(s.workdir, ignore_errors=True)
            del s, it
            torch.cuda.empty_cache()
    del f, S, y, Kop, h
    return out


def bench_c5(ctx, args):
    """configs[4]: 512 x 512^2 batched TV-deblur, images sharded over the ranks (strong scaling)."""
    import pyxu_amd.distributed as pdist
    import pyxu_amd.runtime as pxrt

    total, n = args.c5_images, args.c5_n
    lo, hi = pdist.shard_range(total, ctx.rank, ctx.world)
    f, g = build_batch_problem(hi - lo, n, lo, seed=77)
    K = args.c5_steps
    sr = auto_stop_rate(K)
    with pxrt.Precision(pxrt.Width.SINGLE):
        elapsed, kern_ms, slvr, launches = run_pgd(ctx, f, g, sr, args.c5_warmup, K, True)
    mode, bpp = last_pgd_mode()
    kern_ms = ctx.max_over_ranks(kern_ms if kern_ms is not None else 0.0)
    rec = {"workload": f"PGD {total} x {n}x{n} batch-as-axis Gaussian(sigma=2) + lam*env_mu(L21 o Grad) TV, PositiveOrthant",
           "images": total, "images_per_rank": hi - lo, "scaling": "strong", "steps": K, "warmup": args.c5_warmup,
           "stop_rate": sr, "value": round(total * K / elapsed, 1), "unit": "image-iterations/s",
           "ms_per_step": round(1e3 * elapsed / K, 4), "stop_crit": "MaxIter | RelError (global all-reduce)"}
    if kern_ms > 0:
        rec["roofline"] = roofline((hi - lo) * n * n, kern_ms, bpp, f"{hi - lo}x{n}x{n}", mode=mode)
        rec["roofline"]["per_rank"] = "slowest rank's kernel time"
    del slvr
    return rec


def bench_c4(ctx, args):
    """configs[3]: ADMM + lam L1 on a dense M x N K (QuadraticFunc.prox -> CG on K^T K + I/tau);
    K row-sharded over the ranks: K p local, K^T z = one all-reduce of the N-vector per CG step."""
    import torch

    import pyxu_amd.abc as pxa
    import pyxu_amd.distributed as pdist
    import pyxu_amd.operator as pxo
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd.opt.solver.cg import CG

    M, N = args.c4_m, args.c4_n
    lo, hi = pdist.shard_range(M, ctx.rank, ctx.world)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000 + ctx.rank)
    # synthetic data (torch RNG only creates the inputs; every solver operation is a HIP kernel)
    Kr = torch.randn((hi - lo, N), generator=gen, device="cuda", dtype=torch.float32)
    Kr.mul_(1.0 / np.sqrt(M))
    rng = np.random.default_rng(5)
    xs = np.zeros(N, np.float32)
    xs[rng.choice(N, 64, replace=False)] = rng.standard_normal(64).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        K = pdist.RowShardedLinOp(Kr, M) if ctx.world > 1 else pxa.LinOp.from_array(Kr)
        from pyxu_amd.util import to_device

        from pyxu_amd import _dev

        y = K.apply(to_device(xs))
        y = _dev.axpby(1.0, y, 0.01, torch.randn(y.shape, generator=gen, device="cuda", dtype=torch.float32))
        f = 0.5 * pxo.SquaredL2Norm(dim=hi - lo).asloss(y) * K
        h = args.c4_lam * pxo.L1Norm(dim=N)
        s = pxs.ADMM(f=f, h=h, show_progress=False)
        s.fit(x0=torch.zeros((N,), device="cuda", dtype=torch.float32), tau=1.0,
              stop_crit=pxst.MaxIter(10**9), mode=pxa.Mode.MANUAL)
        it = s.steps()
        for _ in range(args.c4_warmup):
            next(it)
        c0 = CG.steps_taken
        elapsed = timed_steps(ctx, it, 0, args.c4_steps)
        cg_steps = CG.steps_taken - c0  # inner CG iterations of the timed outer iterations
        # the CG operator's kernel alone (HIP events, after the timed region): K^T K p in one pass over K
        normal_ms = None
        from pyxu_amd import _dev

        if ctx.world == 1 and _dev.dense_normal_supported(Kr, y.new_zeros((N,))):
            p = torch.randn((N,), generator=gen, device="cuda", dtype=torch.float32)
            for _ in range(3):
                _dev.dense_normal(Kr, p, 1.0, 1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                _dev.dense_normal(Kr, p, 1.0, 1.0)
            e1.record()
            e1.synchronize()
            normal_ms = e0.elapsed_time(e1) / 10
    per_outer = cg_steps / max(1, args.c4_steps)
    cg_ms = 1e3 * elapsed / max(1.0, per_outer * args.c4_steps)
    one_pass = (hi - lo) * N * 4  # CG's A p reads the local K ONCE (pxa_dense_normal)
    rec = {"workload": f"ADMM dense {M}x{N} K + lam*L1 (x-update: QuadraticFunc.prox -> CG), tau=1",
           "rows_per_rank": hi - lo, "scaling": "strong", "steps": args.c4_steps, "warmup": args.c4_warmup,
           "value": round(args.c4_steps / elapsed, 3), "unit": "ADMM outer iterations/s",
           "ms_per_step": round(1e3 * elapsed / args.c4_steps, 3), "cg_iters_per_outer": round(per_outer, 2),
           "ms_per_cg_iter": round(cg_ms, 4),
           "roofline": {"bound": "hbm", "achieved": round(one_pass / (cg_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(one_pass / (cg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "bytes_model": "one compulsory pass over this rank's K per CG iteration (the one-pass normal operator)",
                        "frac_survey": round(2 * one_pass / (cg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "note": "whole CG iteration (operator + CG vector updates + the outer iteration amortised)"}}
    if normal_ms is not None:  # the fused operator reads K once: its own roofline against one pass
        one = (hi - lo) * N * 4
        tr, src = measured_traffic("normal_group_kernel", f"{hi - lo}x{N}")
        rec["normal_operator"] = {"kernel": "normal_group_kernel + normal_sum/final", "kernel_ms": round(normal_ms, 4),
                                  "achieved": round(one / (normal_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(one / (normal_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "traffic": tr, "traffic_source": src,
                                  "traffic_note": "HBM bytes of the operator pass kernel (normal_group_kernel) per launch",
                                  "note": "K^T K p + p/tau in ONE pass over K (pxa_dense_normal), alg bytes = M N 4"}
    del s, K, Kr
    torch.cuda.empty_cache()
    return rec


def _event_ms(fn, reps, warm=2):
    """Average duration of `fn()` over `reps` back-to-back launches, HIP events on the launch stream (torch's
    current stream, which every pyxu_amd entry point launches on)."""
    import torch

    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def bench_k4(ctx, args):
    """SURVEY §8(d) "Gradient + prox" kernel K4: z <- (1 - rho) z + rho fenchel_prox_{sigma h}(z + sigma Grad w),
    h = lam L1, standalone (pxa_tv_dual_update: kernel C of the three-launch PDS step) on a 2048^2 image and a
    1024^3 volume.  Own bytes = (2D + 1) N 4 (w and z read, z written): SURVEY's figure."""
    import torch

    from pyxu_amd import _dev

    out = {"kernel": "pds_dual_kernel (pxa_tv_dual_update)",
           "op": "z <- (1-rho) z + rho fenchel_prox_{sigma lam L1}(z + sigma Grad w)"}
    gen = torch.Generator(device="cuda").manual_seed(11)
    for key, sh, reps in (("2d_2048", (2048, 2048), 50), ("3d_1024", (args.c3_n,) * 3, 10)):
        if sh[0] <= 0 or key[:2] not in args.k4_which.split(","):
            continue
        D = len(sh)
        N = int(np.prod(sh))
        w = torch.randn(N, generator=gen, device="cuda", dtype=torch.float32)
        z = torch.randn(D * N, generator=gen, device="cuda", dtype=torch.float32).mul_(0.01)
        zo = torch.empty_like(z)
        geom = (1, 1, *sh, 2) if D == 2 else (1, *sh, 3)
        run = lambda: _dev.tv_dual_update(w, z, geom, [-1.0] * 3, [1.0] * 3, 0.28, 0.01, 1.0, 0, relax=0, out=zo)
        ms = _event_ms(run, reps)
        own = (2 * D + 1) * N * 4
        ach = own / (ms * 1e-3) / 1e9
        tkey = "x".join(map(str, sh))
        tr, src = measured_traffic("pds_dual_kernel", tkey)
        out[key] = {"shape": list(sh), "kernel_ms": round(ms, 5), "launches_timed": reps,
                    "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr, "traffic_source": src,
                                 "bytes_per_launch": own, "bytes_model": f"(2D+1) N 4 = {(2 * D + 1) * 4} B/pixel"}}
        del w, z, zo
        torch.cuda.empty_cache()
    return out


def bench_dense_mfma(ctx, args):
    """north_star's dense MFMA path (SURVEY §8(d) C4, B >= 40): Y = X K^T and Y = X K for a dense 8192 x 65536
    K and B stacked right-hand sides (pxa_dense_matmat, v_mfma_f32_32x32x2_f32), HIP-event timed; against the
    fp32 MFMA peak (MI355X_MICROARCH.md: 157.3 TF/s dense)."""
    import torch

    from pyxu_amd import _dev

    M, N = args.c4_m, args.c4_n
    gen = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randn((M, N), generator=gen, device="cuda", dtype=torch.float32).mul_(1.0 / np.sqrt(M))
    out = {"op": "pxa_dense_matmat fp32 (v_mfma_f32_32x32x2_f32)", "M": M, "N": N, "peak_tflops": MFMA_F32_PEAK_TF}
    for B in args.mfma_b:
        for name, trans in (("apply", 0), ("adjoint", 1)):
            X = torch.randn((B, M if trans else N), generator=gen, device="cuda", dtype=torch.float32)
            ms = _event_ms(lambda: _dev.dense_matmat(A, X, trans), 20, warm=5)
            tf = 2.0 * M * N * B / (ms * 1e-3) / 1e12
            out[f"{name}_b{B}"] = {"B": B, "kernel_ms": round(ms, 4), "tflops": round(tf, 2),
                                   "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_F32_PEAK_TF,
                                                "unit": "TFLOP/s", "frac": round(tf / MFMA_F32_PEAK_TF, 4),
                                                "traffic": None}}
            mb = measured_mfma_busy(f"{name}_b{B}")
            if mb is not None:
                out[f"{name}_b{B}"]["mfma_busy"] = mb
            del X
    del A
    torch.cuda.empty_cache()
    return out


def measured_mfma_busy(key):
    """SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs) of the dense MFMA kernel from the committed rocprofv3
    PMC pass (profiles/mfma_busy.json, scripts/pmc_mfma.py), or None.  Not measured in this run."""
    try:
        with open(os.path.join(ROOT, "profiles", "mfma_busy.json")) as fh:
            ent = json.load(fh).get(key)
    except (OSError, ValueError):
        return None
    return ent


def sub_cpu_baselines(sub, args):
    """The oracle on the host beside each sub-record (north_star: every GPU number next to the NumPy path on
    the node's host cores, core count stated); bounded samples, rank 0, N = 1 only."""
    th = cpu_threads()
    model = cpu_model()
    budget = args.sub_cpu_seconds
    if "c2_4096" in sub:
        v, it, dt = cpu_baseline(4096, 4096, seed=4321, budget_s=budget, threads=th)
        sub["c2_4096"]["cpu_baseline"] = {
            "value": round(v, 4), "unit": "image-iterations/s", "cores": th, "kind": "port",
            "sample": f"oracle/ NumPy restatement of the reference PGD path, same 4096x4096 problem, slab-parallel over "
                      f"{th} threads: {it} iterations in {dt:.1f} s on {model}"}
    if "c5" in sub:
        imgs = th
        v, it, dt = cpu_baseline_c5(args.c5_n, imgs, seed=77, budget_s=budget, threads=th)
        sub["c5"]["cpu_baseline"] = {
            "value": round(v, 3), "unit": "image-iterations/s", "cores": th, "kind": "port",
            "sample": f"oracle PGD on {imgs} of the {args.c5_images} independent {args.c5_n}^2 images (one image per "
                      f"thread, {th} threads): {it} iterations each in {dt:.1f} s on {model}"}
    if "c3" in sub and args.c3_cpu_n > 0:
        n3 = args.c3_n
        for algo, (vps, k, dt) in cpu_baseline_c3(args.c3_cpu_n, budget).items():
            if algo in sub["c3"]:
                sub["c3"][algo]["cpu_baseline"] = {
                    "value": round(vps / n3 ** 3, 6), "unit": "iterations/s", "ms_per_step": round(1e3 * n3 ** 3 / vps, 1),
                    "voxel_iterations_per_s": round(vps, 1), "cores": 1, "kind": "port",
                    "sample": f"oracle {'pd3o' if algo == 'pd3o' else 'condat_vu'} (NumPy restatement of pds.py, one "
                              f"thread) on a {args.c3_cpu_n}^3 volume of the same problem: {k} iterations in {dt:.1f} s; "
                              f"{n3}^3 rate = voxel-iterations/s / {n3}^3 (every operator of the step is O(voxels)), "
                              f"on {model}"}
    if "k4" in sub:
        for key, shape in (("2d_2048", (2048, 2048)), ("3d_1024", (256, 256, 256))):
            if key not in sub["k4"]:
                continue
            ms, k, dt = cpu_baseline_k4(shape, min(budget, 3.0))
            full = sub["k4"][key]["shape"]
            scale = float(np.prod(full)) / float(np.prod(shape))
            sub["k4"][key]["cpu_baseline"] = {
                "value": round(ms * scale, 2), "unit": "ms per update", "cores": 1, "kind": "port",
                "sample": f"oracle dual update (Moreau-form fenchel_prox of lam L1, oracle.gradient_apply; one thread) on "
                          f"{'x'.join(map(str, shape))}: {k} updates in {dt:.1f} s"
                          + (f", scaled by the element count to {'x'.join(map(str, full))}" if scale != 1 else "")
                          + f", on {model}"}
    if "dense_mfma" in sub:
        M, N = sub["dense_mfma"]["M"], sub["dense_mfma"]["N"]
        ms, tf, used = cpu_baseline_mfma(M, N, 64, th)
        sub["dense_mfma"]["cpu_baseline"] = {
            "value": round(tf, 3), "unit": "TFLOP/s", "ms_per_apply_b64": round(ms, 2), "cores": used, "kind": "port",
            "sample": f"NumPy X @ K.T (the reference's dense LinOp apply) for B = 64, {M}x{N} fp32 K on the host, BLAS "
                      f"on {used} threads, 3 applies, on {model}"}
    if "c4" in sub:
        ms, used = cpu_baseline_c4(args.c4_m, args.c4_n, th)
        per_outer = sub["c4"].get("cg_iters_per_outer") or 13.0
        sub["c4"]["cpu_baseline"] = {
            "value": round(1e3 / (ms * per_outer), 4), "unit": "ADMM outer iterations/s", "ms_per_cg_iter": round(ms, 2),
            "cores": used, "kind": "port",
            "sample": f"oracle CG (cg.py:125-153) on K^T K + I/tau, dense {args.c4_m}x{args.c4_n} fp32 K on the host, "
                      f"NumPy BLAS on {used} threads, 4 timed CG iterations, outer rate at the GPU run's "
                      f"{per_outer} CG iterations per outer iteration, on {model}"}


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=2048, help="image side (configs[1]: 2048)")
    ap.add_argument("--stop-rate", type=int, default=0, help="stop-criterion rate (0: largest divisor of --steps <= 50)")
    ap.add_argument("--prime-seconds", type=float, default=0.4, help="untimed device priming before the warmup")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline time budget per leg in s (0 = skip)")
    ap.add_argument("--generic", action="store_true", help="disable the fused m_step (rule-by-rule HIP path)")
    ap.add_argument("--no-kernel-timer", action="store_true", help="skip the HIP-event kernel timing window (A/B)")
    ap.add_argument("--kernel-timer-in-region", action="store_true",
                    help="time the kernel with HIP events inside the timed region (they slow its launches)")
    ap.add_argument("--no-sub", action="store_true", help="headline line only (no stop_rate_1 / c5 / c4 records)")
    ap.add_argument("--only", default="", help="run only this sub-record (c2_4096 | c5 | c4 | c3) and print it (profiling)")
    ap.add_argument("--sr1-steps", type=int, default=200, help="stop_rate_1 record: timed steps (at least --steps)")
    ap.add_argument("--sr1-warmup", type=int, default=20, help="stop_rate_1 record: warmup steps (at least --warmup)")
    ap.add_argument("--c4096-steps", type=int, default=50, help="c2_4096 record: timed PGD steps at 4096^2 (0 = skip)")
    ap.add_argument("--c3-n", type=int, default=1024, help="c3 record: volume edge (0 = skip)")
    ap.add_argument("--c3-steps", type=int, default=10)
    ap.add_argument("--c3-three-launch", action="store_true", help="C3 with the three-launch pxa_pds_step (A/B)")
    ap.add_argument("--c3-cpu-n", type=int, default=160, help="c3 CPU baseline: oracle sample volume edge (0 = skip)")
    ap.add_argument("--c5-images", type=int, default=512)
    ap.add_argument("--c5-n", type=int, default=512)
    ap.add_argument("--c5-steps", type=int, default=20)
    ap.add_argument("--c5-warmup", type=int, default=5)
    ap.add_argument("--c4-m", type=int, default=8192)
    ap.add_argument("--c4-n", type=int, default=65536)
    ap.add_argument("--c4-steps", type=int, default=4)
    ap.add_argument("--c4-warmup", type=int, default=1)
    ap.add_argument("--c4-lam", type=float, default=0.01)
    ap.add_argument("--mfma-b", type=lambda s: [int(v) for v in s.split(",") if v], default=[64, 128],
                    help="dense_mfma record: stacked right-hand sides (empty = skip)")
    ap.add_argument("--no-k4", action="store_true", help="skip the k4 (Gradient + prox kernel) record")
    ap.add_argument("--k4-which", default="2d,3d", help="k4 record: shapes to time (2d = 2048^2, 3d = c3-n^3)")
    ap.add_argument("--sub-cpu-seconds", type=float, default=5.0,
                    help="CPU-baseline budget of the c2_4096 / c5 / c4 sub-records in s (0 = skip)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(sys.argv[1:], args.gpus))

    import torch
    import torch.distributed as dist

    import pyxu_amd
    import pyxu_amd.runtime as pxrt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters for rehearsals with more ranks than GPUs (gloo)
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    distributed = world > 1
    backend = None
    if distributed:
        backend = os.environ.get("PXA_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI; gloo for rehearsals
        import datetime

        tmo = datetime.timedelta(seconds=float(os.environ.get("PXA_DIST_TIMEOUT", "120")))  # a hung rendezvous fails
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", dev), timeout=tmo)
        else:
            dist.init_process_group(backend=backend, timeout=tmo)
    if not pyxu_amd.native_loaded():
        raise RuntimeError("libpyxu_amd.so not loaded")
    from pyxu_amd import _dev

    ctx = Ctx(world, rank, dist, coll_device="cpu" if backend == "gloo" else "cuda")

    if args.only:
        fn = {"c2_4096": bench_c2_4096, "c5": bench_c5, "c4": bench_c4, "c3": bench_c3, "k4": bench_k4,
              "dense_mfma": bench_dense_mfma}[args.only]
        rec = fn(ctx, args)
        if rank == 0:
            print(json.dumps({"only": args.only, **rec}), flush=True)
        if distributed:
            dist.destroy_process_group()
        return
    n0 = n1 = args.n
    N = n0 * n1
    sr = args.stop_rate or auto_stop_rate(args.steps)
    f, g, _ = build_problem(n0, n1, seed=1234 + rank)
    with pxrt.Precision(pxrt.Width.SINGLE):
        elapsed_max, kern_ms, slvr, launches = run_pgd(ctx, f, g, sr, args.warmup, args.steps, not args.generic,
                                                       prime_s=args.prime_seconds,
                                                       kernel_timer=("in_region" if args.kernel_timer_in_region else
                                                                     not args.no_kernel_timer))
    fused = slvr._plan is not None
    stack = slvr._plan["stack"] if fused else 1
    mode, bpp = last_pgd_mode()
    del slvr

    sub = {}
    if not args.no_sub:
        # the reference-default stop_rate 1 over a window of its own (--sr1-steps): its lagged stop checks keep up to
        # 8 checks in flight, so a 20-step window after a host synchronisation is mostly pipeline fill and drain
        k1, w1 = max(args.sr1_steps, args.steps), max(args.sr1_warmup, args.warmup)
        with pxrt.Precision(pxrt.Width.SINGLE):
            e1, _, s1, _ = run_pgd(ctx, f, g, 1, w1, k1, not args.generic, kernel_timer=False)
            del s1
        sub["stop_rate_1"] = {"value": round(world * k1 / e1, 2), "unit": "image-iterations/s",
                              "ms_per_step": round(1e3 * e1 / k1, 4), "stop_rate": 1, "steps": k1, "warmup": w1,
                              "stop_checks": "lagged (abc/solver.py _lag_loop, depth %d)" % pxa_lag_depth()}
        del f, g
        torch.cuda.empty_cache()
        if args.c4096_steps > 0:
            sub["c2_4096"] = bench_c2_4096(ctx, args)
            torch.cuda.empty_cache()
        sub["c5"] = bench_c5(ctx, args)
        torch.cuda.empty_cache()
        sub["c4"] = bench_c4(ctx, args)
        torch.cuda.empty_cache()
        if args.c3_n > 0:
            sub["c3"] = bench_c3(ctx, args)
            torch.cuda.empty_cache()
        if not args.no_k4:
            sub["k4"] = bench_k4(ctx, args)
            torch.cuda.empty_cache()
        if args.mfma_b:
            sub["dense_mfma"] = bench_dense_mfma(ctx, args)
            torch.cuda.empty_cache()
        if args.sub_cpu_seconds > 0 and world == 1:
            sub_cpu_baselines(sub, args)

    if rank == 0:
        value = world * args.steps / elapsed_max
        roof = None
        if kern_ms is not None:
            roof = roofline(N * stack, kern_ms, bpp, f"{n0}x{n1}", mode=mode)
            roof["launches_timed"] = launches
            roof["kernel_timer"] = "in_region" if args.kernel_timer_in_region else "post_region"
        cpu = None
        if args.cpu_seconds > 0 and world == 1:
            v1, it1, dt1 = cpu_baseline(n0, n1, seed=1234, budget_s=args.cpu_seconds, threads=1)
            th = max(1, min(CPU_THREADS_MAX, os.cpu_count() or 1))
            vn, itn, dtn = cpu_baseline(n0, n1, seed=1234, budget_s=args.cpu_seconds, threads=th)
            cpu = {"value": round(vn, 4), "unit": "image-iterations/s", "cores": th, "kind": "port",
                   "sample": f"oracle/ NumPy restatement of the reference PGD path, same {n0}x{n1} TV-deblur problem, "
                             f"slab-parallel over {th} threads (oracle/parallel.py, bit-identical to the 1-thread oracle): "
                             f"{itn} iterations in {dtn:.1f} s on {cpu_model()}",
                   "single_core": {"value": round(v1, 4), "cores": 1, "sample": f"{it1} iterations in {dt1:.1f} s"}}
        line = {
            "metric": "solver iterations/s (PGD, TV-regularised deblur)",
            "value": round(value, 2),
            "unit": "image-iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed_max / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (piecewise-constant phantom, Gaussian blur, 1% noise; random dense K for c4)",
            "config": {"workload": f"PGD {n0}x{n1} Gaussian(sigma=2) deblur + lam*env_mu(L21 o Grad) TV, PositiveOrthant",
                       "image": [n0, n1], "images_per_gpu": 1, "stop_rate": sr,
                       "stop_crit": "MaxIter | RelError" + (f" (global, {'RCCL' if backend == 'nccl' else backend} all-reduce)" if world > 1 else ""),
                       "fused_m_step": fused, "pgd_launch": mode,
                       "parallelism": f"independent images x{world} (one per rank)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            **sub,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
