"""Development probe: which host code paths launch dense_matmat (GEMV / MFMA) and dense_normal during the C4
ADMM outer iterations (bench.py --only c4 workload, 3 outer iterations); prints a short call stack per launch."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

counts = collections.Counter()
orig_mm, orig_nm = _dev.dense_matmat, _dev.dense_normal


def tag(kind):
    st = traceback.extract_stack()[-7:-1]
    key = kind + " <- " + " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(st))
    counts[key] += 1


def mm(A, X, trans):
    tag(f"dense_matmat(trans={trans})")
    return orig_mm(A, X, trans)


def nm(*a, **k):
    tag("dense_normal")
    return orig_nm(*a, **k)


_dev.dense_matmat, _dev.dense_normal = mm, nm


class Args:
    c4_m, c4_n, c4_steps, c4_warmup, c4_lam = 8192, 65536, 3, 0, 0.01


ctx = bench.Ctx(1, 0, None)
rec = bench.bench_c4(ctx, Args())
print(rec["value"], rec["ms_per_cg_iter"], rec["cg_iters_per_outer"])
for k, v in sorted(counts.items(), key=lambda kv: -kv[1]):
    print(f"{v:5d}  {k}")
