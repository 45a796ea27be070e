#!/usr/bin/env python3
"""Per-phase shader-clock breakdown of the network kernel (s_memtime stamps,
diagnostics API), optionally under ablation masks.

  python tools/net_stamps.py [c3|c4] [abl,abl,...]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

NAMES = ["loads", "fwd", "nll", "bwd2 gemm", "bwd2 out", "bwd1 gemm", "bwd1 out",
         "bwd0 gemm", "bwd0 out"]
CFG = {"c3": ([(64, 40), (40, 40), (40, 2)], 128, 100),
       "c4": ([(64, 40), (40, 40), (40, 2)], 1024, 200)}


def report(name, t, abl):
    t = t[t[:, 0] != 0]
    d = (t[:, 1:12] - t[:, 0:1]).float()
    prev = torch.zeros(d.shape[0])
    print(f"{name} abl={abl}: {t.shape[0]} workgroups; s_memtime ticks, median per phase:")
    for k, nm in enumerate(NAMES):
        cur = d[:, k]
        print(f"  {nm:10s} {float((cur - prev).median()):10.0f}")
        prev = cur
    print(f"  total      {float(d[:, len(NAMES) - 1].median()):10.0f}  "
          f"(max {float(d[:, len(NAMES) - 1].max()):.0f})")


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    abls = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    layers, S, M = CFG[name]
    plan = InnerLoopPlan("fullcov", layers, S, M)
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    u = torch.randn(M, 64, generator=g).to(dev)
    z = torch.randint(0, 2, (M,), generator=g).to(torch.int32).to(dev)
    w = torch.full((M,), 8.0, device=dev)
    xs = torch.randn(plan.xshard_count, generator=g).to(dev) * 0.1
    gs = torch.zeros(plan.xshard_count, device=dev)
    nll = torch.zeros(1, dtype=torch.float64, device=dev)
    nblk = S * 8
    st = torch.zeros(nblk * 16, dtype=torch.int64, device=dev)
    for abl in abls:
        plan.lib.psvi_debug_set(1, abl)
        plan.mvn_net(u, z, w, xs, gs, nll)
        st.zero_()
        plan.lib.psvi_debug_set_ptr(2, ctypes.c_void_p(st.data_ptr()))
        plan.mvn_net(u, z, w, xs, gs, nll)
        torch.cuda.synchronize()
        plan.lib.psvi_debug_set_ptr(2, None)
        plan.lib.psvi_debug_set(1, 0)
        report(name, st.view(nblk, 16).cpu().clone(), abl)


if __name__ == "__main__":
    main()
