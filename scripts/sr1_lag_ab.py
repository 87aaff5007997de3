"""A/B of the stop_rate-1 engines on the bench's headline problem (2048^2 PGD, MaxIter | RelError, MANUAL steps()):
the speculative checks (lag 0) against the lagged engine at several depths, with the in-kernel RelError fold or
the fold launch.  Interleaved, each arm K timed steps after W warmup steps (bench.run_pgd's timing)."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
ctx = bench.Ctx(1, 0, None, coll_device="cuda")
f, g, _ = bench.build_problem(2048, 2048, seed=1234)
import pyxu_amd.opt.solver as pxs  # noqa: E402

# (depth, in-kernel fold, window statistics, publication by the next launch)
arms = [(0, False, False, True), (8, False, True, True), (8, False, True, False), (8, False, False, True),
        (4, False, True, True), (2, False, True, True)]
if os.environ.get("SR1_ARMS") == "short":
    arms = [(0, False, False, True), (8, False, True, True), (4, False, True, True), (2, False, True, True)]
res = {}
for rep in range(2):
    for depth, ink, win, pub in arms:
        pxa.Solver._LAG, pxa.Solver._LAG_INKERNEL, pxa.Solver._LAG_WINDOW = depth, ink, win
        pxs.PGD._LAG_PUB = pub
        with pxrt.Precision(pxrt.Width.SINGLE):
            e, _, s, _ = bench.run_pgd(ctx, f, g, 1, 20, K, True, kernel_timer=False)
        del s
        torch.cuda.synchronize()
        key = f"lag{depth}_{'window' if win else 'epilogue'}_{'pub' if (win and pub) else ('inkernel' if ink else 'foldlaunch')}"
        res.setdefault(key, []).append(round(1e3 * e / K, 4))
        print(key, res[key][-1], "ms/step", flush=True)
print(json.dumps({"steps": K, "ms_per_step": res}))
