#!/usr/bin/env python3
"""Time the LeNet inner loop at C5 (S=256, M=500, MNIST-shaped synthetic u)
through psvi_inner_loop with in-library Philox draws.  Prints ms/step."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "blackbox-coresets-vi_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--M", type=int, default=500)
    ap.add_argument("--T", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--hvp", type=int, default=0, help="also time N psvi_hvp calls")
    ap.add_argument("--abl", type=int, default=0,
                    help="PSVI_DBG_LENET_ABLATION mask (timing diagnostics)")
    a = ap.parse_args()
    from psvi.models import make_lenet
    from psvi.runtime import InnerLoopPlan

    torch.manual_seed(0)
    net = make_lenet(mc_samples=a.S, init_sd=0.05)
    params = torch.nn.utils.parameters_to_vector(net.parameters()).detach().cuda()
    plan = InnerLoopPlan("lenet", [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)],
                         a.S, a.M)
    plan.lib.psvi_debug_set(17, a.abl)
    u = torch.randn(a.M, 1, 28, 28, device="cuda")
    z = torch.randint(0, 10, (a.M,), device="cuda", dtype=torch.int32)
    w = torch.full((a.M,), 60000.0 / a.M, device="cuda")
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device="cuda")
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    plan.inner_loop(u, z, w, params, m, v, 2, 1e-3, seed=1, ws=ws)
    torch.cuda.synchronize()
    for r in range(a.reps):
        t0 = time.perf_counter()
        el = plan.inner_loop(u, z, w, params, m, v, a.T, 1e-3, seed=2 + r, ws=ws)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.T
        print(f"S={a.S} M={a.M} T={a.T}: {dt * 1e3:.3f} ms/step  "
              f"({1.0 / dt:.1f} inner-steps/s)  elbo[0]={el[0].item():.6g} "
              f"elbo[-1]={el[-1].item():.6g}", flush=True)
    if a.hvp:
        from psvi.runtime import randn_

        e = torch.empty(plan.eps_count, device="cuda")
        randn_(e, 9)
        vec = torch.randn(plan.param_count, device="cuda")
        for mixed in (False, True):
            plan.hvp(u, z, w, e, params, vec, mixed=mixed)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.hvp):
                plan.hvp(u, z, w, e, params, vec, mixed=mixed)
            torch.cuda.synchronize()
            print(f"psvi_hvp (mixed={mixed}): {(time.perf_counter() - t0) / a.hvp * 1e3:.3f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
