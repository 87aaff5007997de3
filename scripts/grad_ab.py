"""A/B of the gradient kernels (PXA_TUNE_GRAD_KERNEL 0 march + non-temporal stores, 2 march + plain stores,
1 row kernel) at 1024^3 and 256^3 fp32, apply and adjoint, interleaved over 3 rounds (HIP events, 5 calls)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pyxu_amd import _dev  # noqa: E402


def timed(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for sh in ((1024, 1024, 1024), (256, 256, 256)):
    D = len(sh)
    N = sh[0] * sh[1] * sh[2]
    x = torch.randn(N, device="cuda")
    args = (1, list(sh), list(range(D)), [0] * D, [-1.0] * D, [1] * D, [1.0] * D)
    z = _dev.gradient2(x, *args)
    for rnd in range(3):
        for mode in (0, 2, 1):
            old = _dev.tuning(_dev.TUNE_GRAD_KERNEL, mode)
            try:
                ta = timed(lambda: _dev.gradient2(x, *args))
                tj = timed(lambda: _dev.gradient2(z, *args, adjoint=True))
            finally:
                _dev.tuning(_dev.TUNE_GRAD_KERNEL, old)
            print(json.dumps({"shape": sh, "round": rnd, "mode": mode, "apply_ms": round(ta, 4),
                              "adjoint_ms": round(tj, 4), "apply_tbs": round(16 * N / ta / 1e9, 2),
                              "adjoint_tbs": round(16 * N / tj / 1e9, 2)}), flush=True)
    del x, z
    torch.cuda.empty_cache()
