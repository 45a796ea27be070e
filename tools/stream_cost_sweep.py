#!/usr/bin/env python3
"""Sweep the streaming update's run-partition cost weights (PSVI_DBG_STREAM_COST:
extra cost of a band's first tile and of its diagonal, last, tile) at C3 and
time the inner loop (HIP events around one 200-step psvi_inner_loop call after
a warm-up call), one plan per setting.

  python tools/stream_cost_sweep.py 40:35 90:70 ...   (first%:diag%)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from bench import LAYERS, M, S_PER_GPU, reference_init_params, synthetic_inputs
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime import _lib as L

    if os.environ.get("PSVI_LIB_AB"):  # A/B against another build of the library
        L.LIB_PATH = os.environ["PSVI_LIB_AB"]
    lib = L.load()
    dev = torch.device("cuda", 0)
    u, z, w = synthetic_inputs(dev)
    for arg in sys.argv[1:] or ["40:35"]:
        f, d = (int(x) for x in arg.split(":"))
        lib.psvi_debug_set(34, f + 1000 * d)
        plan = InnerLoopPlan("fullcov", LAYERS, S_PER_GPU, M)
        lib.psvi_debug_set(34, -1)
        res = []
        for rep in range(3):
            p = reference_init_params(LAYERS, dev)
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            plan.inner_loop(u, z, w, p, m, v, 20, 1e-3, seed=1)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            plan.inner_loop(u, z, w, p, m, v, 200, 1e-3, seed=2)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / 200 * 1e3)
        print(f"first {f}% diag {d}%: {min(res):.2f} us/step (reps {', '.join(f'{x:.2f}' for x in res)})",
              flush=True)
        del plan


if __name__ == "__main__":
    main()
