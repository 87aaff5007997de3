"""Where the driver's short window loses time: bench.py's headline PGD run at the driver's flags
(--steps 20 --warmup 5), with host CLOCK_MONOTONIC stamps (time.perf_counter_ns) around the timed window
and around each step's host work.  Run under `rocprofv3 --kernel-trace` (same clock domain) and read with
--analyze <kernel_trace.csv> <stamps.json>: kernel starts / ends against the window and the host stamps
give the start latency (t0 -> first kernel), the bubbles between kernels, and the tail (last kernel ->
t1).

usage: python scripts/driver_gap_probe.py [steps warmup] > stamps.json
       python scripts/driver_gap_probe.py --analyze <dir with *kernel_trace.csv> stamps.json
"""
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(steps, warmup):
    import torch

    import bench
    import pyxu_amd.abc as pxa
    import pyxu_amd.opt.solver as pxs
    import pyxu_amd.opt.stop as pxst
    import pyxu_amd.runtime as pxrt
    from pyxu_amd import _dev

    torch.cuda.set_device(0)
    # host stamps inside the stop check (no change to the code path: wrappers around the same calls)
    marks_in = []
    orig_wait = _dev.wait_event

    def wait_stamped(ev, *a, **k):
        t = time.perf_counter_ns()
        orig_wait(ev, *a, **k)
        marks_in.append(("wait", t, time.perf_counter_ns()))

    _dev.wait_event = wait_stamped
    orig_spec = pxa.Solver._step_speculative

    def spec_stamped(self, *a, **k):
        t = time.perf_counter_ns()
        r = orig_spec(self, *a, **k)
        marks_in.append(("spec", t, time.perf_counter_ns()))
        return r

    pxa.Solver._step_speculative = spec_stamped
    f, g, _ = bench.build_problem(2048, 2048, seed=1234)
    sr = bench.auto_stop_rate(steps)
    out = []
    with pxrt.Precision(pxrt.Width.SINGLE):
        like = torch.empty((1,), dtype=torch.float32, device="cuda")
        for rep in range(3):
            s = pxs.PGD(f=f, g=g, show_progress=False, stop_rate=sr)
            rel = pxst.RelError(eps=1e-30)
            s.fit(x0=_dev.zeros((f.dim,), like), stop_crit=pxst.MaxIter(10 ** 9) | rel, mode=pxa.Mode.MANUAL)
            rel.stop({"x": s._mstate["x"]})
            rel.stop({"x": s._mstate["x"]})
            rel.clear()
            gen = s.steps()
            for _ in range(warmup):
                next(gen)
            torch.cuda.synchronize()
            t0 = time.perf_counter_ns()
            marks = []
            for _ in range(steps):
                a = time.perf_counter_ns()
                next(gen)
                marks.append((a, time.perf_counter_ns()))
            t_launched = time.perf_counter_ns()
            torch.cuda.synchronize()
            t1 = time.perf_counter_ns()
            out.append({"rep": rep, "t0": t0, "t1": t1, "t_launched": t_launched, "steps": marks,
                        "inner": [m for m in marks_in if m[1] >= t0]})
            marks_in.clear()
            del s, gen
    json.dump(out, sys.stdout)


def analyze(trace_dir, stamps):
    rows = []
    for fn in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    text = open(stamps).read()
    reps, _ = json.JSONDecoder().raw_decode(text[text.index("[{"):])  # the JSON line may share the log
    for rep in reps:
        t0, t1 = rep["t0"], rep["t1"]
        ks = [k for k in rows if t0 <= k[0] <= t1]
        print(f"rep {rep['rep']}: window {(t1 - t0) / 1e3:.1f} us, {len(ks)} kernels")
        if not ks:
            continue
        busy = sum(e - s for s, e, _ in ks)
        print(f"  t0 -> first kernel start {(ks[0][0] - t0) / 1e3:.1f} us; last kernel end -> t1 {(t1 - ks[-1][1]) / 1e3:.1f} us; "
              f"all launched at +{(rep['t_launched'] - t0) / 1e3:.1f} us; kernels busy {busy / 1e3:.1f} us")
        prev_end = ks[0][1]
        for s, e, n in ks[1:]:
            if s - prev_end > 1500:
                print(f"  gap {(s - prev_end) / 1e3:.1f} us before {n} at +{(s - t0) / 1e3:.1f} us")
            prev_end = max(prev_end, e)
        for i, (a, b) in enumerate(rep["steps"]):
            if b - a > 30000:
                print(f"  host step {i}: {(b - a) / 1e3:.1f} us at +{(a - t0) / 1e3:.1f} us")
        for tag, a, b in rep.get("inner", []):
            print(f"  host {tag}: +{(a - t0) / 1e3:.1f} -> +{(b - t0) / 1e3:.1f} us")
        print("  host step starts:", " ".join(f"{(a - t0) / 1e3:.1f}" for a, _ in rep["steps"]))
        import re

        for s, e, n in ks:
            m = re.search(r"(\w+_kernel)", n)
            print(f"    +{(s - t0) / 1e3:7.1f} us  {(e - s) / 1e3:5.1f} us  {m.group(1) if m else n[:40]}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2], sys.argv[3])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 20, int(sys.argv[2]) if len(sys.argv) > 2 else 5)
