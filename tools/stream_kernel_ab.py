#!/usr/bin/env python3
"""A/B of the streaming update variants (diagnostics): C3 inner loop steps/s
with the production kernel (PSVI_DBG_UPD_STREAM_OFF = 0: corr / m / v stores
with sc1), the same kernel with plain stores (= 3) and the chunked kernel
(= 1), alternating, plus the update's device time from the loop's own timing
windows.

  python tools/stream_kernel_ab.py [steps] [rounds]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from bench import LAYERS, LR, M, reference_init_params, synthetic_inputs  # noqa: E402
from psvi.runtime import InnerLoopPlan  # noqa: E402

DBG_STREAM_OFF, DBG_LOOP_TIMING = 10, 8
NAMES = {0: "sc1 stores", 3: "plain stores", 1: "chunked"}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda")
    u, z, w = synthetic_inputs(dev)
    plan = InnerLoopPlan("fullcov", LAYERS, 128, M)
    lib = plan.lib
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
    res = {k: [] for k in NAMES}
    upd = {k: [] for k in NAMES}
    for _ in range(rounds):
        for k in NAMES:
            lib.psvi_debug_set(DBG_STREAM_OFF, k)
            p = reference_init_params(LAYERS, dev)
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            plan.inner_loop(u, z, w, p, m, v, 20, LR, seed=1, ws=ws)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            plan.inner_loop(u, z, w, p, m, v, steps, LR, seed=2, ws=ws)
            torch.cuda.synchronize()
            res[k].append(steps / (time.perf_counter() - t0))
            # device time of the update (+ its slot reduce) from the loop's windows
            lib.psvi_debug_set(DBG_LOOP_TIMING, 1)
            plan.inner_loop(u, z, w, p, m, v, 50, LR, seed=3, ws=ws)
            torch.cuda.synchronize()
            out = (ctypes.c_double * 3)()
            lib.psvi_debug_loop_timing(out)
            lib.psvi_debug_set(DBG_LOOP_TIMING, 0)
            upd[k].append(out[1])
            lib.psvi_debug_set(DBG_STREAM_OFF, 0)
    for k, name in NAMES.items():
        print(f"{name:12s} steps/s: " + " ".join(f"{x:.0f}" for x in res[k])
              + "   update+reduce us: " + " ".join(f"{x:.1f}" for x in upd[k]), flush=True)


if __name__ == "__main__":
    main()
