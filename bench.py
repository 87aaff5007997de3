#!/usr/bin/env python3
"""
Benchmark: PGD solver iterations/s on TV-regularised deblurring (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 2048 x 2048 image, H = Gaussian(sigma=2) blur (13 taps/axis,
zero boundary), f = 1/2||H x - y||^2 + lam * env_mu(L21) o Gradient, g = PositiveOrthant,
lam = mu = 0.01, fp32, synthetic piecewise-constant phantom + 1% noise.
One "step" = one PGD iteration (Solver._step: stop check every `stop_rate` iterations + m_step)
driven through the pyxu_amd Solver API in MANUAL mode.

Multi-GPU (torch.distributed.run, one rank per GPU, RCCL): every rank solves its own image
(independent problems shard with no data-path collective) -> weak scaling; value = total
image-iterations/s over all ranks = ranks * K / max_rank(elapsed).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
KERNEL = "pgd_tv2d_kernel"
ALG_BYTES_PER_PIXEL = 48  # 8 reads + 4 writes of fp32 per pixel per PGD iteration
FUSED_BYTES_PER_PIXEL = 16  # compulsory traffic of the one-launch step: x, x_prev, y read + x_new write


def phantom(shape, rng):
    x = np.zeros(shape, dtype=np.float32)
    for _ in range(12):
        lo = [int(rng.integers(0, n // 2)) for n in shape]
        hi = [l + int(rng.integers(n // 8 + 1, n // 2 + 1)) for l, n in zip(lo, shape)]
        x[tuple(slice(l, h) for l, h in zip(lo, hi))] = rng.uniform(0.2, 1.0)
    return x


def build_problem(n0, n1, seed, lam=0.01, mu=0.01, sigma=2.0):
    import pyxu_amd.operator as pxo
    import pyxu_amd.runtime as pxrt
    from pyxu_amd.util import to_device

    sh = (n0, n1)
    N = n0 * n1
    rng = np.random.default_rng(seed)
    with pxrt.Precision(pxrt.Width.SINGLE):
        H = pxo.Gaussian(arg_shape=sh, sigma=sigma, truncate=3.0)
        x_gt = to_device(phantom(sh, rng).reshape(-1))
        y = H.apply(x_gt)
        noise = to_device((0.01 * rng.standard_normal(N)).astype(np.float32))
        from pyxu_amd import _dev

        y = _dev.axpby(1.0, y, 1.0, noise)
        G = pxo.Gradient(arg_shape=sh)
        f = 0.5 * pxo.SquaredL2Norm(dim=N).asloss(y) * H + lam * pxo.L21Norm(arg_shape=(2, *sh)).moreau_envelope(mu) * G
        f.diff_lipschitz = 1.0 + (lam / mu) * 8.0  # ||H||^2 + lam/mu ||Grad||^2, set analytically (§8(d))
        g = pxo.PositiveOrthant(dim=N)
    return f, g, y


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def measured_traffic(kernel, n0, n1):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes (profiles/traffic.json,
    written by scripts/pmc_traffic.py: (2 * FETCH_SIZE + WRITE_SIZE) * 1024, the gfx950 correction of
    MI355X_MICROARCH.md §HBM), or None when no profile of this workload exists."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            tab = json.load(fh)
    except (OSError, ValueError):
        return None
    ent = tab.get(f"{kernel}@{n0}x{n1}")
    return None if ent is None else ent.get("hbm_bytes_per_launch")


def cpu_baseline(n0, n1, seed, budget_s, lam=0.01, mu=0.01, sigma=2.0):
    """Oracle (NumPy restatement of the reference path) on the host: same problem; as many PGD
    iterations as fit in about `budget_s` seconds (bounded sample; at least 2)."""
    import oracle as orc

    sh = (n0, n1)
    N = n0 * n1
    rng = np.random.default_rng(seed)
    taps, c = orc.gaussian_taps(sigma, 3.0, np.float32)
    blur = dict(arg_shape=sh, kernel=[taps, taps], center=[c, c])
    x_gt = phantom(sh, rng).reshape(-1)
    y = orc.stencil_apply(x_gt, sh, [taps, taps], [c, c])
    y = (y + (0.01 * rng.standard_normal(N)).astype(np.float32)).astype(np.float32)
    grad = lambda v: orc.deblur_tv_grad(v, blur, y, lam, mu, dict(arg_shape=sh))
    prox = lambda z, t: orc.positive_orthant_prox(z)
    tau = np.float32(1 / np.float32(1.0 + (lam / mu) * 8.0))
    x0 = np.zeros(N, dtype=np.float32)
    t0 = time.perf_counter()
    orc.pgd(x0, grad, prox, tau, 1)  # warm-up (page-in, allocator) and per-iteration estimate
    t1 = time.perf_counter() - t0
    iters = int(max(2, min(500, budget_s / max(t1, 1e-3))))
    t0 = time.perf_counter()
    orc.pgd(x0, grad, prox, tau, iters)
    dt = time.perf_counter() - t0
    return iters / dt, iters, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=2048, help="image side (configs[1]: 2048)")
    ap.add_argument("--stop-rate", type=int, default=50, help="stop-criterion evaluation rate (reference default 1)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline time budget in s (0 = skip)")
    ap.add_argument("--generic", action="store_true", help="disable the fused m_step (rule-by-rule HIP path)")
    ap.add_argument("--no-kernel-timer", action="store_true", help="skip the in-region HIP-event kernel timing (A/B)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import pyxu_amd
    import pyxu_amd.abc as pxa
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd import _dev

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters for rehearsals with more ranks than GPUs (gloo)
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    distributed = world > 1
    if distributed:
        backend = os.environ.get("PXA_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI; gloo for rehearsals
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend=backend)
    if not pyxu_amd.native_loaded():
        raise RuntimeError("libpyxu_amd.so not loaded")

    n0 = n1 = args.n
    N = n0 * n1
    f, g, y = build_problem(n0, n1, seed=1234 + rank)
    with pxrt.Precision(pxrt.Width.SINGLE):
        slvr = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=args.stop_rate)
        # N>1: the ranks' images form one batch-as-axis problem (C5 semantics): the stop check is the
        # GLOBAL RelError, one RCCL all-reduce of 2 doubles per check (pyxu_amd.distributed)
        import pyxu_amd.distributed as pdist

        rel = pdist.ShardedRelError(eps=1e-30) if distributed else pxst.RelError(eps=1e-30)
        stop = pxst.MaxIter(10**9) | rel
        slvr.fit(x0=_dev.zeros((N,), y), stop_crit=stop, mode=pxa.Mode.MANUAL, fused=not args.generic)
        fused = slvr._plan is not None
        # prime the stop-check path once (loads its kernels' code objects) so that a warmup shorter
        # than stop_rate does not leave one-time module loading inside the timed region
        rel.stop({"x": slvr._mstate["x"]})
        rel.stop({"x": slvr._mstate["x"]})
        rel.clear()
        gen = slvr.steps()
        for _ in range(args.warmup):
            next(gen)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        # one HIP-event window per run of back-to-back fused launches, closed only where other device work
        # (the stop check) is enqueued: an event record between two launches costs a ~11 us bubble
        # (rocprofv3 trace, r01c), so per-10-launch windows would tax the timed step by ~1 us
        timer = _dev.LaunchTimer(window=10**9)
        if not args.no_kernel_timer:
            _dev.set_launch_timer(timer)  # HIP-event windows around the fused-step launches, on their stream
        t0 = time.perf_counter()
        for _ in range(args.steps):
            next(gen)
        timer.interrupt()  # close the last window right behind the last launch (before the host sync)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        _dev.set_launch_timer(None)
        kern_ms = timer.mean_ms() if fused else None

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())

    if rank == 0:
        value = world * args.steps / elapsed_max
        roof = None
        if kern_ms is not None:
            pix = N * slvr._plan["stack"]
            alg_bytes = ALG_BYTES_PER_PIXEL * pix  # 48 B/pixel/iteration
            achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
            traffic = measured_traffic(KERNEL, n0, n1)
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": KERNEL,
                    "kernel_ms": round(kern_ms, 5), "launches_timed": timer.launches,
                    "alg_bytes_per_launch": alg_bytes,
                    "fused_compulsory_bytes_per_launch": FUSED_BYTES_PER_PIXEL * pix,
                    "frac_vs_fused_compulsory": round(FUSED_BYTES_PER_PIXEL * pix / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        cpu = None
        if args.cpu_seconds > 0 and world == 1:
            v, it, dt = cpu_baseline(n0, n1, seed=1234, budget_s=args.cpu_seconds)
            cpu = {"value": round(v, 4), "unit": "image-iterations/s", "cores": 1, "kind": "port",
                   "sample": f"oracle/ NumPy restatement of the reference PGD path (single thread), same {n0}x{n1} "
                             f"TV-deblur problem, {it} iterations in {dt:.1f} s on {cpu_model()}"}
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
            "data": "synthetic (piecewise-constant phantom, Gaussian blur, 1% noise)",
            "config": {"workload": f"PGD {n0}x{n1} Gaussian(sigma=2) deblur + lam*env_mu(L21 o Grad) TV, PositiveOrthant",
                       "image": [n0, n1], "images_per_gpu": 1, "stop_rate": args.stop_rate,
                       "stop_crit": "MaxIter | RelError" + (f" (global, {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} all-reduce)" if world > 1 else ""), "fused_m_step": fused, "parallelism": f"batch-as-axis slabs x{world} (one image per rank)"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
