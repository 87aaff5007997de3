"""C4 benchmark (BASELINE.json configs[3]): ADMM with f = 1/2||K . - y||^2, K dense (M x N) fp32,
h = lam L1 (the "prox" x-update = QuadraticFunc.prox = CG on (K^T K + I/tau), two
passes over K per CG iteration), tau = 1, sparse ground truth (64 non-zeros), y = K x*.

Prints one JSON line: ADMM outer iterations/s, CG inner iterations per outer iteration, ms per CG
iteration, and the effective HBM rate of the two K passes of a CG iteration (2 M N 4 bytes) against
8 TB/s (SURVEY §8(d) C4 unit).  Env: PXA_M, PXA_N (default 8192 x 65536), PXA_OUTER (timed outer
iterations, default 3), PXA_LAM (default 0.1)."""
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import pyxu_amd.abc as pxa
import pyxu_amd.operator as pxo
import pyxu_amd.opt.solver as pxs
import pyxu_amd.opt.stop as pxst
import pyxu_amd.runtime as pxrt
from pyxu_amd import _dev
from pyxu_amd.opt.solver import cg as cg_mod


def main():
    M = int(os.environ.get("PXA_M", "8192"))
    N = int(os.environ.get("PXA_N", "65536"))
    outer = int(os.environ.get("PXA_OUTER", "3"))
    lam = float(os.environ.get("PXA_LAM", "0.1"))
    gen = torch.Generator(device="cuda").manual_seed(0)
    Kd = torch.randn(M, N, device="cuda", dtype=torch.float32, generator=gen) / M**0.5
    rng = np.random.default_rng(0)
    xs = np.zeros(N, dtype=np.float32)
    xs[rng.choice(N, 64, replace=False)] = rng.standard_normal(64).astype(np.float32)
    with pxrt.Precision(pxrt.Width.SINGLE):
        K = pxa.LinOp.from_array(Kd)
        y = K.apply(torch.from_numpy(xs).cuda())
        f = 0.5 * pxo.SquaredL2Norm(dim=M).asloss(y) * K
        h = lam * pxo.L1Norm(dim=N)
        s = pxs.ADMM(f=f, h=h, show_progress=False)
        s.fit(x0=torch.zeros(N, device="cuda", dtype=torch.float32), tau=1.0, stop_crit=pxst.MaxIter(1),
              mode=pxa.Mode.MANUAL)
        # count / time CG inner iterations (test instrumentation around the unchanged m_step)
        stats = {"n": 0}
        orig = cg_mod.CG.m_step

        def counted(self):
            stats["n"] += 1
            return orig(self)

        cg_mod.CG.m_step = counted
        s.m_step()  # warm-up outer iteration
        torch.cuda.synchronize()
        stats["n"] = 0
        t0 = time.perf_counter()
        for _ in range(outer):
            s.m_step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        cg_mod.CG.m_step = orig
        inner = stats["n"] / outer
        # GPU-side time of one CG iteration's two K passes (apply + adjoint), HIP events, back to back
        p = torch.randn(N, device="cuda", dtype=torch.float32, generator=gen)
        for _ in range(3):
            K.adjoint(K.apply(p))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            K.adjoint(K.apply(p))
        e1.record()
        e1.synchronize()
        pair_ms = e0.elapsed_time(e1) / 20
        # the one-pass normal operator that CG now uses for A p (pxa_dense_normal), same vector
        normal_ms = None
        if _dev.dense_normal_supported(Kd, p):
            for _ in range(3):
                _dev.dense_normal(Kd, p, 1.0, 1.0)
            e0.record()
            for _ in range(20):
                _dev.dense_normal(Kd, p, 1.0, 1.0)
            e1.record()
            e1.synchronize()
            normal_ms = e0.elapsed_time(e1) / 20
        shutil.rmtree(s.workdir, ignore_errors=True)
    ms_outer = 1e3 * dt / outer
    ms_cg = ms_outer / max(inner, 1e-9)
    print(json.dumps({"config": "C4", "M": M, "N": N, "lam": lam, "outer_iters": outer,
                      "admm_outer_per_s": round(1e3 / ms_outer, 3), "ms_per_outer": round(ms_outer, 3),
                      "cg_iters_per_outer": round(inner, 2), "ms_per_cg_iter": round(ms_cg, 4),
                      "gemv_pair_ms": round(pair_ms, 4),
                      "gemv_pair_gbs": round(2 * M * N * 4 / (pair_ms * 1e-3) / 1e9, 1),
                      "gemv_pair_frac_8tbs": round(2 * M * N * 4 / (pair_ms * 1e-3) / 8e12, 3),
                      "cg_iter_frac_8tbs": round(2 * M * N * 4 / (ms_cg * 1e-3) / 8e12, 3),
                      "normal_ms": None if normal_ms is None else round(normal_ms, 4),
                      "normal_gbs_of_one_pass": None if normal_ms is None else round(M * N * 4 / (normal_ms * 1e-3) / 1e9, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
