#!/usr/bin/env python3
"""Per-phase device timing of the inner step (HIP events around N back-to-back
launches of one phase).  Usage: python tools/kernel_bench.py [c3|c4|c2] [iters]
[KEY=VALUE ...] (psvi_debug_set keys, A/B)"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan, randn_  # noqa: E402

CFG = {"c3": ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100),
       "c4": ("fullcov", [(64, 40), (40, 40), (40, 2)], 1024, 200),
       "c2": ("meanfield", [(2, 100), (100, 4)], 32, 50)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    fam, layers, S, M = CFG[name]
    from psvi.runtime import _lib
    for kv in sys.argv[3:]:  # KEY=VALUE: psvi_debug_set before the plan (A/B)
        k, v = kv.split("=")
        _lib.load().psvi_debug_set(int(k), int(v))
    dev = "cuda"
    plan = InnerLoopPlan(fam, layers, S, M)
    g = torch.Generator().manual_seed(0)
    u = torch.randn(M, layers[0][0], generator=g).to(dev)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).to(dev)
    w = torch.full((M,), 800.0 / M, device=dev)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        if fam == "fullcov":
            parts += [0.1 * torch.randn(n, generator=g), torch.full((n,), -4.0),
                      1e-3 * torch.randn((n - 1) * (n - 2) // 2, generator=g)]
        else:
            parts += [0.1 * torch.randn(n, generator=g), torch.full((n,), -4.0)]
    params = torch.cat(parts).to(dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    eps = torch.empty(plan.eps_count, device=dev)
    randn_(eps, 1)
    out = {}
    out["randn"] = timeit(lambda: randn_(eps, 1), iters)
    nll = torch.zeros(1, dtype=torch.float64, device=dev)
    if fam == "fullcov":
        xs = torch.empty(plan.xshard_count, device=dev)
        gs = torch.zeros(plan.xshard_count, device=dev)
        out["sample(memset+fwd)"] = timeit(lambda: plan.mvn_sample(eps, params, xs), iters)
        out["net(+memset)"] = timeit(lambda: plan.mvn_net(u, z, w, xs, gs, nll), iters)
        if os.environ.get("NET_SPLIT"):
            # pseudopoint split over workgroups: plans built after setting the knob
            for below in (1000,):
                plan.lib.psvi_debug_set(5, below)
                p2 = InnerLoopPlan(fam, layers, S, M)
                out[f"net split(<{below})"] = timeit(lambda: p2.mvn_net(u, z, w, xs, gs, nll), iters)
                plan.lib.psvi_debug_set(5, 96)
        if os.environ.get("NET_ABLATION"):
            lib = plan.lib
            for mask in (1, 2, 4, 8, 16, 2 | 8, 1 | 2 | 4 | 8):
                lib.psvi_debug_set(1, mask)
                out[f"net abl={mask}"] = timeit(lambda: plan.mvn_net(u, z, w, xs, gs, nll), iters)
            lib.psvi_debug_set(1, 0)
        st = [1]

        def upd():
            plan.mvn_update(eps, gs, params, m, v, step=st[0], lr=1e-3, kl_out=nll)
            st[0] += 1
        out["update"] = timeit(upd, iters)
        eps2 = torch.empty_like(eps)
        randn_(eps2, 2)
        x2 = torch.empty_like(xs)

        def upd_smp():
            plan.mvn_update(eps, gs, params, m, v, step=st[0], lr=1e-3, kl_out=nll, eps_next=eps2,
                            x_next=x2)
            st[0] += 1
        out["update+next sample (fused)"] = timeit(upd_smp, iters)
    if fam == "fullcov" and plan.tiled_floats:
        ts = plan.tiled_state()
        plan.tiled_convert(params, m, v, ts, True)

        def upd_t(fused):
            kw = dict(eps_next=eps2, x_next=x2) if fused else {}
            plan.mvn_update_tiled(eps, gs, params, m, v, ts, step=st[0], lr=1e-3, kl_out=nll, **kw)
            st[0] += 1
        out["update (tiled)"] = timeit(lambda: upd_t(False), iters)
        out["update+next sample (tiled, fused)"] = timeit(lambda: upd_t(True), iters)
        plan.tiled_convert(params, m, v, ts, False)
        out["tiled convert (both ways)"] = timeit(
            lambda: (plan.tiled_convert(params, m, v, ts, True),
                     plan.tiled_convert(params, m, v, ts, False)), 20)
    if fam == "fullcov":
        T = 20
        elb = torch.empty(T, dtype=torch.float64, device=dev)
        lws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
        out["inner_loop per step (T=20, Philox)"] = timeit(
            lambda: plan.inner_loop(u, z, w, params, m, v, T, 1e-3, seed=3, elbo_out=elb, ws=lws),
            max(5, iters // T)) / T
        grad = torch.empty_like(params)
        out["update(grad mode)"] = timeit(
            lambda: plan.mvn_update(eps, gs, params, grad_out=grad, kl_out=nll), iters)
    ws = plan.workspace()
    e = torch.empty(1, dtype=torch.float64, device=dev)
    st2 = [1]

    def full():
        randn_(eps, st2[0])
        plan.inner_step(u, z, w, eps, params, m, v, step=st2[0], lr=1e-3, elbo_out=e, ws=ws)
        st2[0] += 1
    out["full step (randn + fused)"] = timeit(full, iters)
    print(json.dumps({"config": name, "us": {k: round(x, 2) for k, x in out.items()}}))


if __name__ == "__main__":
    main()
