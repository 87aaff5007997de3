"""Diagnostic: aligned vs misaligned launches of the PGD tile kernel at 2048^2 -- where do the RelError
partials differ (indices, values, unwritten slots)?  (tests/test_gpu_pgd_variants.py case 0)"""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_pgd_variants as t  # noqa: E402
from pyxu_amd.util import to_NUMPY  # noqa: E402

s = t._plan((2048, 2048), 1, 1, 2.0, "pos")
m, p = s._mstate, s._plan
x, xp, hty = m["x"], m["x_prev"], p["hty"]
for rep in range(3):
    pa, pb, pc = t._parts(s), t._parts(s), t._parts(s)
    a = t._launch(s, x, xp, hty, 0.37, pa)
    b = t._launch(s, t._misaligned(x), t._misaligned(xp), t._misaligned(hty), 0.37, pb)
    c = t._launch(s, x, xp, hty, 0.37, pc)
    torch.cuda.synchronize()
    A, B, C = to_NUMPY(pa), to_NUMPY(pb), to_NUMPY(pc)
    print(f"rep {rep}: x_new a==b {np.array_equal(to_NUMPY(a), to_NUMPY(b))}; parts n={A.size} "
          f"a<0 {(A < 0).sum()} b<0 {(B < 0).sum()} c<0 {(C < 0).sum()} a!=b {(A != B).sum()} a!=c {(A != C).sum()}")
    d = np.nonzero(A != B)[0][:8]
    for i in d:
        print(f"   i={i} (tile {i // 2 // 4}, wave {(i // 2) % 4}, stat {i % 2}) a={A[i]!r} b={B[i]!r} c={C[i]!r}")
