#!/usr/bin/env python3
"""Inner-loop step time (C3, psvi_inner_loop, Philox) against the update kernel's
c-blocks per chunk (PSVI_DBG_UPD_CHUNK), interleaved rounds in one process.

  python tools/chunk_sweep.py [chunks,...] [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

LAYERS = [(64, 40), (40, 40), (40, 2)]


def main():
    chunks = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,6").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    u = torch.randn(100, 64, generator=g).to(dev)
    z = torch.randint(0, 2, (100,), generator=g).to(torch.int32).to(dev)
    w = torch.full((100,), 8.0, device=dev)
    plans = {}
    for c in chunks:
        InnerLoopPlan("fullcov", LAYERS, 128, 100).lib.psvi_debug_set(9, c)
        plans[c] = InnerLoopPlan("fullcov", LAYERS, 128, 100)
    plans[chunks[0]].lib.psvi_debug_set(9, 0)
    p0 = None
    res = {c: [] for c in chunks}
    T = 200
    for r in range(rounds):
        for c in chunks:
            plan = plans[c]
            if p0 is None:
                p0 = torch.zeros(plan.param_count, device=dev)
            params = p0.clone()
            m, v = torch.zeros_like(params), torch.zeros_like(params)
            ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
            plan.inner_loop(u, z, w, params, m, v, 10, 1e-3, seed=1, ws=ws)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            plan.inner_loop(u, z, w, params, m, v, T, 1e-3, seed=2, ws=ws)
            b.record()
            torch.cuda.synchronize()
            res[c].append(a.elapsed_time(b) / T * 1e3)
    for c in chunks:
        xs = sorted(res[c])
        print(f"chunk {c}: us/step median {xs[len(xs) // 2]:.2f} min {xs[0]:.2f}")


if __name__ == "__main__":
    main()
