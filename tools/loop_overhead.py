#!/usr/bin/env python3
"""Split the C3 headline's per-call cost into host and device parts: wall time
of psvi_inner_loop calls of T = 0, 1, 2, 20, 500 steps between synchronises
(as bench.py's timed region), and the device time of the same calls from HIP
events on the stream.  Fixed cost per call = intercept of time vs T."""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))


def main():
    import bench
    from psvi.runtime import InnerLoopPlan

    dev = torch.device("cuda", 0)
    plan = InnerLoopPlan("fullcov", bench.LAYERS, bench.S_PER_GPU, bench.M)
    u, z, w = bench.synthetic_inputs(dev)
    p0 = bench.reference_init_params(bench.LAYERS, dev)
    params, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
    elbo = torch.empty(500, dtype=torch.float64, device=dev)
    plan.inner_loop(u, z, w, params, m, v, 30, bench.LR, seed=1, elbo_out=elbo, ws=ws)
    torch.cuda.synchronize()
    for T in (0, 1, 2, 20, 100, 500):
        walls, devs = [], []
        for rep in range(12 if T == 20 else 5):
            params.copy_(p0)
            m.zero_()
            v.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            plan.inner_loop(u, z, w, params, m, v, T, bench.LR, seed=7, elbo_out=elbo, ws=ws)
            e1.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            devs.append(e0.elapsed_time(e1) * 1e3)
        if T == 20:
            print("  T=20 walls:", " ".join(f"{x:.0f}" for x in walls), " devices:",
                  " ".join(f"{x:.0f}" for x in devs), flush=True)
        wall, dv = sorted(walls)[len(walls) // 2], sorted(devs)[len(devs) // 2]
        print(f"T={T:4d}: wall {wall:9.1f} us  device {dv:9.1f} us  "
              f"wall/step {wall / max(T, 1):7.2f}  device/step {dv / max(T, 1):7.2f}", flush=True)
    t0 = time.perf_counter()
    for _ in range(100):
        torch.cuda.synchronize()
    print(f"idle synchronize: {(time.perf_counter() - t0) * 1e4:.1f} us", flush=True)


if __name__ == "__main__":
    main()
