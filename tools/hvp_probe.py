#!/usr/bin/env python3
"""Time psvi_hvp at C3 (fn2 64-40-40-2, S=128, M=100; or --cfg c4 / c2) with and
without the mixed products.  Prints ms per call."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))

CFG = {"c3": ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100),
       "c4": ("fullcov", [(64, 40), (40, 40), (40, 2)], 1024, 200),
       "c2": ("meanfield", [(2, 100), (100, 4)], 32, 50)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c3")
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--stamps", action="store_true", help="net_rop_kernel phase clocks")
    ap.add_argument("--dbg", action="append", default=[], help="KEY=VALUE psvi_debug_set before timing")
    a = ap.parse_args()
    from psvi.runtime import InnerLoopPlan, randn_

    fam, layers, S, M = CFG[a.cfg]
    from psvi.runtime import _lib
    for kv in a.dbg:  # before the plan: some keys shape its tables
        k, v = kv.split("=")
        _lib.load().psvi_debug_set(int(k), int(v))
    plan = InnerLoopPlan(fam, layers, S, M)
    g = torch.Generator().manual_seed(0)
    dev = "cuda"
    u = torch.randn(M, layers[0][0], generator=g).to(dev)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).to(dev)
    w = torch.full((M,), 8.0, device=dev)
    p = (0.05 * torch.randn(plan.param_count, generator=g)).to(dev)
    vec = torch.randn(plan.param_count, generator=g).to(dev)
    eps = torch.empty(plan.eps_count, device=dev)
    randn_(eps, 3)
    ws = plan.workspace()
    for mixed in (False, True):
        for _ in range(3):
            plan.hvp(u, z, w, eps, p, vec, mixed=mixed)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.n):
            plan.hvp(u, z, w, eps, p, vec, mixed=mixed)
        torch.cuda.synchronize()
        print(f"{a.cfg} psvi_hvp mixed={mixed} {' '.join(a.dbg)}: {(time.perf_counter() - t0) / a.n * 1e3:.4f} ms",
              flush=True)
    if a.stamps:
        # net_rop_kernel phase clocks (PSVI_DBG_ROP_STAMPS), mean over workgroups
        import ctypes
        import numpy as np
        nwg = S * 2
        st = torch.zeros(nwg * 16, dtype=torch.int64, device=dev)
        plan.lib.psvi_debug_set_ptr(18, ctypes.c_void_p(st.data_ptr()))
        plan.hvp(u, z, w, eps, p, vec, mixed=True)
        torch.cuda.synchronize()
        plan.lib.psvi_debug_set_ptr(18, None)
        v = st.cpu().numpy().reshape(nwg, 16).astype(np.float64)
        v = v[v[:, 15] > 0]
        names = ["weights", "inputs|wgrad", "fwd0", "fwd1", "fwd2", "head", "bwd2", "bwd1", "bwd0",
                 "store|bias"]
        print("net_rop clocks per workgroup (mean): " +
              " ".join(f"{n}={v[:, i].mean():.0f}" for i, n in enumerate(names)) +
              f" total={v[:, :10].sum(1).mean():.0f} chunks={v[:, 15].mean():.1f}", flush=True)


if __name__ == "__main__":
    main()
