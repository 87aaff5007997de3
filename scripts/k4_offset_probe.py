"""K4 (pxa_tv_dual_update, kernel C alone) at 1024^3 with w, z, z_out carved from one allocation at chosen
relative offsets, interleaved, 3 reps: does the placement of the three streams (HBM channel mapping) explain
the 5.0 / 5.7 ms bimodality of the k4 record?  usage: python scripts/k4_offset_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from pyxu_amd import _dev

    n = 1024
    N = n ** 3
    skews = {"aligned": (0, 0), "skew4k": (1024, 2048), "skew64k+": (16384 + 64, 32768 + 192),
             "skew1m": (262144 + 1024, 524288 + 3072)}
    pool = torch.empty(7 * N + 2 * 1024 * 1024, device="cuda", dtype=torch.float32)
    gen = torch.Generator(device="cuda").manual_seed(11)
    for rep in range(3):
        for name, (sz, so) in skews.items():
            w = pool.narrow(0, 0, N)
            z = pool.narrow(0, N + sz, 3 * N)
            zo = pool.narrow(0, 4 * N + sz + so, 3 * N)
            w.normal_(generator=gen)
            z.normal_(generator=gen).mul_(0.01)
            run = lambda: _dev.tv_dual_update(w, z, (1, n, n, n, 3), [-1.0] * 3, [1.0] * 3, 0.28, 0.01, 1.0, 0,
                                              relax=0, out=zo)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 10
            print(json.dumps({"rep": rep, "placement": name, "z_off_floats": N + sz, "zo_off_floats": 4 * N + sz + so,
                              "w_addr_mod_1g": w.data_ptr() % (1 << 30), "kernel_ms": round(ms, 4),
                              "frac": round(28 * N / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
