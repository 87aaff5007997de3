"""Dense LinOp: K (M x N) fp32, B stacked right-hand sides.
Times apply (Y = X K^T) and adjoint (Y = Z K) through the C-ABI and prints one JSON line per
(B, direction) with ms, TFLOP/s (2 M N B flop) and the A-stream GB/s (4 M N bytes)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pyxu_amd import _dev

M = int(os.environ.get("PXA_M", "8192"))
N = int(os.environ.get("PXA_N", "65536"))
Bs = [int(b) for b in os.environ.get("PXA_B", "1,2,4,8,16,32,64,128").split(",")]
KNOBS = [int(v) for v in os.environ.get("PXA_DENSE_KNOBS", "0,1").split(",")]  # PXA_TUNE_DENSE_KERNEL values
reps = int(os.environ.get("PXA_REPS", "10"))

torch.manual_seed(0)
A = torch.randn(M, N, device="cuda", dtype=torch.float32) / M**0.5
for knob, B in [(k, b) for b in Bs for k in KNOBS]:
    _dev.tuning(_dev.TUNE_DENSE_KERNEL, knob)
    X = torch.randn(B, N, device="cuda", dtype=torch.float32)
    Z = torch.randn(B, M, device="cuda", dtype=torch.float32)
    for name, trans, inp in (("apply", 0, X), ("adjoint", 1, Z)):
        for _ in range(2):
            _dev.dense_matmat(A, inp, trans)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _dev.dense_matmat(A, inp, trans)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"op": name, "M": M, "N": N, "B": B, "ms": round(ms, 4),
                          "tflops": round(2.0 * M * N * B / (ms * 1e-3) / 1e12, 2),
                          "a_stream_gbs": round(4.0 * M * N / (ms * 1e-3) / 1e9, 1),
                          "path": ("gemv" if B < 2 else "mfma-lds" if (B >= 32 and knob == 0) else "mfma-reg")}),
              flush=True)
