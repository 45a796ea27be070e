#!/usr/bin/env python3
"""A/B of a plan-creation diagnostics switch (psvi_debug_set key, two values):
C3 inner-loop steps/s of a plan created under each value, alternating rounds
(KNOB_S / KNOB_M in the environment: another fn2 shape, e.g. C4's 1024 / 200).

  python tools/knob_ab.py KEY VALUE_A VALUE_B [steps] [rounds]
  e.g. tools/knob_ab.py 14 512 256   (PSVI_DBG_NET_THREADS)
       tools/knob_ab.py 12 0 1       (PSVI_DBG_STREAM_RR)
       tools/knob_ab.py 15 256 512   (PSVI_DBG_NET_WG_TARGET)
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
    key, vals = int(sys.argv[1]), (int(sys.argv[2]), int(sys.argv[3]))
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 300
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    dev = torch.device("cuda")
    S, Mx = int(os.environ.get("KNOB_S", 128)), int(os.environ.get("KNOB_M", M))
    if Mx == M:
        u, z, w = synthetic_inputs(dev)
    else:
        g = torch.Generator().manual_seed(5)
        u = torch.randn(Mx, LAYERS[0][0], generator=g)
        z = (torch.rand(Mx, generator=g) < torch.sigmoid(5.0 * u.sum(1))).to(torch.int32).to(dev)
        u = u.to(dev)
        w = torch.full((Mx,), 1000.0 / Mx, device=dev)
    lib = InnerLoopPlan("fullcov", LAYERS, S, Mx).lib
    default = {14: 0, 12: 0, 15: 256, 5: 256}.get(key, 0)
    plans = {}
    for val in vals:
        lib.psvi_debug_set(key, val)
        plans[val] = InnerLoopPlan("fullcov", LAYERS, S, Mx)
    lib.psvi_debug_set(key, default)
    res = {v: [] for v in vals}
    for _ in range(rounds):
        for val in vals:
            plan = plans[val]
            p = reference_init_params(LAYERS, dev)
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
            plan.inner_loop(u, z, w, p, m, v, 20, LR, seed=1, ws=ws)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            plan.inner_loop(u, z, w, p, m, v, steps, LR, seed=2, ws=ws)
            torch.cuda.synchronize()
            res[val].append(steps / (time.perf_counter() - t0))
    for val in vals:
        print(f"key {key} = {val:5d}: steps/s " + " ".join(f"{x:.0f}" for x in res[val]), flush=True)


if __name__ == "__main__":
    main()
