#!/usr/bin/env python3
"""Device time of one network-kernel launch (HIP events around N launches of
psvi_mvn_phase_net[_draw]) against its workgroups' own life (s_memtime /
s_memrealtime stamps), under ablation masks: what the launch costs beyond the
workgroups' work (dispatch, the end-of-kernel write-back of dirty lines).

  python tools/net_time_probe.py [c3|c4] [abl,abl,...] [--draw]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

CFG = {"c3": ([(64, 40), (40, 40), (40, 2)], 128, 100),
       "c4": ([(64, 40), (40, 40), (40, 2)], 1024, 200)}


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    name = args[0] if args else "c3"
    abls = [int(x) for x in args[1].split(",")] if len(args) > 1 else [0, 16]
    draw = "--draw" in sys.argv
    layers, S, M = CFG[name]
    plan = InnerLoopPlan("fullcov", layers, S, M)
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    u = torch.randn(M, 64, generator=g).to(dev)
    z = torch.randint(0, 2, (M,), generator=g).to(torch.int32).to(dev)
    w = torch.full((M,), 8.0, device=dev)
    xs = (0.1 * torch.randn(plan.xrecv_count, generator=g)).to(dev)
    gs = torch.zeros(plan.xrecv_count, device=dev)
    nll = torch.zeros(1, dtype=torch.float64, device=dev)
    e = torch.empty(plan.eps_count, device=dev)
    nblk = plan.s_local * 8
    st = torch.zeros(nblk * 16, dtype=torch.int64, device=dev)
    lib = plan.lib

    def launch():
        if draw:
            plan.mvn_net(u, z, w, xs, gs, nll, draw=(e, 3, 0))
        else:
            plan.mvn_net(u, z, w, xs, gs, nll)

    for abl in abls:
        lib.psvi_debug_set(1, abl)
        for _ in range(5):
            launch()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        a.record()
        for _ in range(n):
            launch()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / n * 1e3
        st.zero_()
        lib.psvi_debug_set_ptr(2, ctypes.c_void_p(st.data_ptr()))
        launch()
        torch.cuda.synchronize()
        lib.psvi_debug_set_ptr(2, None)
        t = st.view(nblk, 16).cpu()
        t = t[t[:, 0] != 0]
        s0, s1 = t[:, 13].double(), t[:, 14].double()
        span = float((s1.max() - s0.min()) * 0.01)
        life = float(((s1 - s0) * 0.01).median())
        print(f"{name} draw={draw} abl={abl}: {us:.2f} us per launch (events, {n} back to back); "
              f"workgroups: first start -> last end {span:.2f} us, median life {life:.2f} us")
    lib.psvi_debug_set(1, 0)


if __name__ == "__main__":
    main()
