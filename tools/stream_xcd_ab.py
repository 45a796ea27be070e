#!/usr/bin/env python3
"""A/B of the streaming update's run placement (diagnostics): C3 inner loop
steps/s with the runs dealt round-robin over XCDs (PSVI_DBG_STREAM_RR = 1)
against one contiguous eighth of the run list per XCD (default), alternating.

  python tools/stream_xcd_ab.py [steps] [rounds]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from bench import LAYERS, LR, M, reference_init_params, synthetic_inputs  # noqa: E402
from psvi.runtime import InnerLoopPlan  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda")
    u, z, w = synthetic_inputs(dev)
    plans = {}
    for rr in (1, 0):
        lib = InnerLoopPlan("fullcov", LAYERS, 128, M).lib
        lib.psvi_debug_set(12, rr)
        plans[rr] = InnerLoopPlan("fullcov", LAYERS, 128, M)
        lib.psvi_debug_set(12, 0)
    res = {0: [], 1: []}
    for _ in range(rounds):
        for rr in (1, 0):
            plan = plans[rr]
            p = reference_init_params(LAYERS, dev)
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
            plan.inner_loop(u, z, w, p, m, v, 20, LR, seed=1, ws=ws)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            plan.inner_loop(u, z, w, p, m, v, steps, LR, seed=2, ws=ws)
            torch.cuda.synchronize()
            res[rr].append(steps / (time.perf_counter() - t0))
    for rr, name in ((1, "round-robin"), (0, "xcd-contiguous")):
        print(f"{name:15s} steps/s: " + " ".join(f"{x:.0f}" for x in res[rr]), flush=True)


if __name__ == "__main__":
    main()
