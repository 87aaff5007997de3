"""A/B of pxa_dense_normal at C4's 8192 x 65536 between library builds (HIP events, 20 launches after 3
warm-ups), each in its own process: `PXA_LIB_PATH=<lib> python scripts/normal_ab.py [tuning]` prints one JSON
line with the time and the error against an fp64 torch evaluation of s A^T (A x) + d x (the argument is the
PXA_TUNE_NORMAL_KERNEL value); with --all it runs the shipped library's three kernel settings and
build/libpyxu_amd_r04f.so (the one-workgroup-per-row kernel before its buffer-load rewrite)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(tune):
    sys.path.insert(0, ROOT)
    import torch

    from pyxu_amd import _dev

    M, N = int(os.environ.get("PXA_M", "8192")), int(os.environ.get("PXA_N", "65536"))
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(M, N, device="cuda", generator=g).mul_(M ** -0.5)
    x = torch.randn(N, device="cuda", generator=g)
    if tune:
        _dev.tuning(_dev.TUNE_NORMAL_KERNEL, tune)
    for _ in range(3):
        y = _dev.dense_normal(A, x, 1.0, 1.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = _dev.dense_normal(A, x, 1.0, 1.0)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 20
    A64 = A.double()
    ref = A64.t() @ (A64 @ x.double()) + x.double()
    err = float((y.double() - ref).abs().max() / ref.abs().max())
    print(json.dumps({"lib": os.path.basename(os.environ.get("PXA_LIB_PATH", "libpyxu_amd.so")), "tune": tune,
                      "M": M, "N": N, "ms": round(ms, 4), "TBps": round(M * N * 4 / ms / 1e9, 3), "err": err}),
          flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--all":
        # shipped library: 0 row-split kernel, 1 one workgroup per row, 2 row-split without the exchange;
        # then the library before the rewrite
        runs = [(None, 0), (None, 1), (None, 2), ("build/libpyxu_amd_r04f.so", 0), (None, 0)]
        for lib, tune in runs:
            env = dict(os.environ)
            if lib:
                env["PXA_LIB_PATH"] = os.path.join(ROOT, lib)
            r = subprocess.run([sys.executable, __file__, str(tune)], env=env, timeout=240)
            if r.returncode != 0:
                raise SystemExit(r.returncode)
        return
    one(int(sys.argv[1]) if len(sys.argv) > 1 else 0)


if __name__ == "__main__":
    main()
