"""Development probe: where the host spends a PGD step at stop_rate = 1 (2048^2, MaxIter | RelError, the bench's
problem), without cProfile's distortion: perf_counter_ns around the engine's phases, and how often the stop
check's flags had already landed when the host came to wait for them (host-bound) or not (device-bound)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
import pyxu_amd.abc as pxa  # noqa: E402
import pyxu_amd.abc.solver as solver_mod  # noqa: E402
import pyxu_amd.opt.solver as pxs  # noqa: E402
import pyxu_amd.opt.stop as pxst  # noqa: E402
import pyxu_amd.runtime as pxrt  # noqa: E402
from pyxu_amd import _dev  # noqa: E402

acc = collections.Counter()
cnt = collections.Counter()
ON = [False]


def timed(cls, name, label=None):
    fn = getattr(cls, name)
    label = label or f"{cls.__name__}.{name}"

    def wrapper(*a, **k):
        if not ON[0]:
            return fn(*a, **k)
        t0 = time.perf_counter_ns()
        try:
            return fn(*a, **k)
        finally:
            acc[label] += time.perf_counter_ns() - t0
            cnt[label] += 1

    setattr(cls, name, wrapper)


orig_wait = _dev.HostFlagBuffer.wait


def wait(self, seq, spin_s=1e-3):
    if ON[0]:
        cnt["flags ready on arrival"] += int((self.flags == seq).all())
        cnt["flag waits"] += 1
        t0 = time.perf_counter_ns()
        orig_wait(self, seq, spin_s)
        acc["HostFlagBuffer.wait"] += time.perf_counter_ns() - t0
        return
    orig_wait(self, seq, spin_s)


_dev.HostFlagBuffer.wait = wait
timed(pxst.RelError, "stop_async")
timed(pxst.RelError, "_decide")
timed(pxs.PGD, "m_step")
timed(solver_mod.Solver, "_record_batch")
timed(solver_mod.Solver, "_take_capture")
timed(solver_mod.Solver, "_step")
timed(_dev.HostFlagBuffer, "fold")

f, g, _ = bench.build_problem(2048, 2048, seed=1)
N = 1000
with pxrt.Precision(pxrt.Width.SINGLE):
    like = torch.empty((1,), dtype=torch.float32, device="cuda")
    s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=1)
    s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10**9) | pxst.RelError(eps=1e-30), mode=pxa.Mode.MANUAL)
    gen = s.steps()
    for _ in range(200):
        next(gen)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        next(gen)
    torch.cuda.synchronize()
    plain = 1e6 * (time.perf_counter() - t0) / N
    ON[0] = True
    t0 = time.perf_counter()
    for _ in range(N):
        next(gen)
    torch.cuda.synchronize()
    inst = 1e6 * (time.perf_counter() - t0) / N
    ON[0] = False
print(f"plain {plain:.1f} us/step, instrumented {inst:.1f} us/step")
for k, v in acc.most_common():
    print(f"  {k:32s} {v / 1e3 / N:8.2f} us per step  ({cnt[k]} calls)")
print(f"  flags ready on arrival: {cnt['flags ready on arrival']} of {cnt['flag waits']}")
