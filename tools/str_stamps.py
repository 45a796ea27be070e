#!/usr/bin/env python3
"""Streaming full-cov update (mvn_stream_kernel) under the diagnostics API:
event-timed launches and per-workgroup shader-clock phase sums, under
ablation masks (1: corr/m/v and eps loads from one L2-resident place,
2: no MFMAs, 4: no corr/m/v stores).  Diagnostic only.

  python tools/str_stamps.py [abl,abl,...]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

PH = ["dL", "diag", "adam+st", "ld issue", "x'", "storeE", "flush", "barrier"]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    abls = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0]
    layers, S, M = [(64, 40), (40, 40), (40, 2)], 128, 100
    plan = InnerLoopPlan("fullcov", layers, S, M)
    g = torch.Generator().manual_seed(0)
    eps = torch.randn(plan.eps_count, generator=g).cuda()
    eps1 = torch.randn(plan.eps_count, generator=g).cuda()
    p = (torch.randn(plan.param_count, generator=g) * 0.01).cuda()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    gs = (torch.randn(plan.xshard_count, generator=g) * 0.01).cuda()
    x = torch.empty(plan.xshard_count, device="cuda")
    ts = plan.tiled_state()
    plan.tiled_convert(p, m, v, ts, True)
    lib = plan.lib
    nwg = 256
    st = torch.zeros(nwg * 16, dtype=torch.int64, device="cuda")
    for abl in abls:
        lib.psvi_debug_set(3, abl)
        us = timed(lambda: plan.mvn_update_tiled(eps, gs, p, m, v, ts, step=1, lr=1e-3,
                                                 eps_next=eps1, x_next=x))
        st.zero_()
        lib.psvi_debug_set_ptr(4, ctypes.c_void_p(st.data_ptr()))
        plan.mvn_update_tiled(eps, gs, p, m, v, ts, step=1, lr=1e-3, eps_next=eps1, x_next=x)
        torch.cuda.synchronize()
        lib.psvi_debug_set_ptr(4, None)
        a = st.cpu().numpy().reshape(nwg, 16).astype(np.float64)
        tiles = a[:, 9]
        tot = a[:, 10] - a[:, 12]
        wall = (a[:, 11] - a[:, 13]) * 10.0  # 100 MHz -> ns
        mhz = tot / np.maximum(wall, 1) * 1e3
        phs = " ".join(f"{n}={a[:, i].sum() / tiles.sum():.0f}" for i, n in enumerate(PH))
        print(f"abl {abl:3d}: {us:7.1f} us/launch | per tile cycles: {phs} | "
              f"tiles/WG {tiles.min():.0f}-{tiles.max():.0f}, WG cycles mean {tot.mean():.0f} "
              f"max {tot.max():.0f}, clock {np.median(mhz):.0f} MHz, WG wall max {wall.max()/1e3:.1f} us")
    lib.psvi_debug_set(3, 0)


if __name__ == "__main__":
    main()
