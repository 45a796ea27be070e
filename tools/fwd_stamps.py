#!/usr/bin/env python3
"""Full-cov sample (forward) kernel under the diagnostics API: event timing
and per-workgroup shader-clock stamps under ablation masks (1 loads, 2 MFMAs,
4 x atomics).

  python tools/fwd_stamps.py [c3|c4] [abl,abl,...]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402
from upd_stamps import CFG, timed  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    abls = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    layers, S, M = CFG[name]
    plan = InnerLoopPlan("fullcov", layers, S, M)
    g = torch.Generator().manual_seed(0)
    eps = torch.randn(plan.eps_count, generator=g).cuda()
    params = (torch.randn(plan.param_count, generator=g) * 0.01).cuda()
    xs = torch.empty(plan.xshard_count, device="cuda")
    lib = plan.lib
    maxblk = 1 << 14
    st = torch.zeros(maxblk * 16, dtype=torch.int64, device="cuda")
    for abl in abls:
        lib.psvi_debug_set(6, abl)
        us = timed(lambda: plan.mvn_sample(eps, params, xs))
        st.zero_()
        lib.psvi_debug_set_ptr(7, ctypes.c_void_p(st.data_ptr()))
        plan.mvn_sample(eps, params, xs)
        torch.cuda.synchronize()
        lib.psvi_debug_set_ptr(7, None)
        lib.psvi_debug_set(6, 0)
        t = st.view(maxblk, 16).cpu()
        nblk = int((t[:, 3] != 0).nonzero().max()) + 1
        t = t[:nblk].double()
        print(f"{name} abl={abl}: {us:.1f} us/launch (memset + kernel), {nblk} workgroups")
        rt0, rt1 = t[:, 6], t[:, 7]   # s_memrealtime, 100 MHz, chip-wide
        t0 = rt0.min()
        print(f"  timeline (us): kernel span {float(rt1.max() - t0) / 100:.1f}; item starts p50/p90/max "
              f"{float(torch.quantile((rt0 - t0).float(), 0.5)) / 100:.1f}/"
              f"{float(torch.quantile((rt0 - t0).float(), 0.9)) / 100:.1f}/{float((rt0 - t0).max()) / 100:.1f}; "
              f"item durations p50/max {float(torch.quantile((rt1 - rt0).float(), 0.5)) / 100:.1f}/"
              f"{float((rt1 - rt0).max()) / 100:.1f}")
        for nm, x in (("first stage", t[:, 1] - t[:, 0]), ("stages+mfma", t[:, 2] - t[:, 1]),
                      ("atomics", t[:, 3] - t[:, 2]), ("item total", t[:, 3] - t[:, 0])):
            q = torch.quantile(x.float(), torch.tensor([0.1, 0.5, 0.9, 1.0]))
            print(f"  {nm:12s} p10 {q[0]:8.0f}  p50 {q[1]:8.0f}  p90 {q[2]:8.0f}  max {q[3]:8.0f}")


if __name__ == "__main__":
    main()
