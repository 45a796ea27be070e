#!/usr/bin/env python3
"""The driver's bench configuration (--steps 20 --warmup 5) dissected: bench's
own headline_world1 (warm-up call, reset, one timed call) repeated in one
process, each timed call also bracketed by HIP events on the stream and a host
timestamp after the enqueue returns, so the wall time per call splits into
host enqueue, device time and the synchronise.

  python3 tools/driver_cfg_probe.py [--reps 6] [--steps 20] [--warmup 5]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))


def main():
    import bench

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--events-first", action="store_true",
                    help="the event-bracketed calls before bench's headline reps")
    ap.add_argument("--pre", default="none",
                    help="before the first headline: none | burn (100 C3 steps, no sync) | "
                         "burnsync<ms> (burn, synchronise, sleep ms) | c4 (bench's C4 line)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rt = bench.Runtime(dev, 1, 0)
    args = argparse.Namespace(steps=a.steps, warmup=a.warmup)
    prep = bench.headline_prep(rt, args)
    if a.pre.startswith("burn"):
        p = prep["p_init"].clone()
        mm, vv = torch.zeros_like(p), torch.zeros_like(p)
        prep["plan"].inner_loop(prep["u"], prep["z"], prep["w"], p, mm, vv, 100, bench.LR,
                                seed=9, ws=prep["ws"])
        if a.pre != "burn":
            torch.cuda.synchronize()
            time.sleep(float(a.pre[len("burnsync"):]) * 1e-3)
    elif a.pre == "c4":
        bench.c4_timings(rt)
    if not a.events_first:
        heads(bench, rt, args, prep, a)
    events(bench, prep, a)
    if a.events_first:
        heads(bench, rt, args, prep, a)


def heads(bench, rt, args, prep, a):
    for rep in range(a.reps):
        el = bench.headline_world1(rt, args, prep)[0]
        print(f"headline_world1 rep {rep}: {el / a.steps * 1e6:7.2f} us/step "
              f"({a.steps / el:9.1f} inner-steps/s)", flush=True)


def events(bench, prep, a):
    plan, u, z, w, p_init = prep["plan"], prep["u"], prep["z"], prep["w"], prep["p_init"]
    ws, elbo_t = prep["ws"], prep["elbo_t"]
    params = p_init.clone()
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    stride = plan.eps_stride
    scratch = [t.clone() for t in (params, m, v)]
    plan.inner_loop(u, z, w, *scratch, 50, bench.LR, seed=1, ws=ws)
    for rep in range(a.reps):
        # bench's headline: the timed call continues the warm-up (resident state)
        params.copy_(p_init)
        m.zero_()
        v.zero_()
        plan.inner_loop(u, z, w, params, m, v, a.warmup, bench.LR, seed=3, ws=ws, keep=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        plan.inner_loop(u, z, w, params, m, v, a.steps, bench.LR, seed=3, step0=a.warmup + 1,
                        offset=a.warmup * stride, elbo_out=elbo_t, ws=ws)
        e1.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        dv = e0.elapsed_time(e1) * 1e3
        print(f"rep {rep}: wall {(t2 - t0) * 1e6:8.1f} us  enqueue {(t1 - t0) * 1e6:7.1f}  "
              f"device {dv:8.1f}  ({(t2 - t0) * 1e6 / a.steps:6.2f} / {dv / a.steps:6.2f} "
              f"us per step)", flush=True)


if __name__ == "__main__":
    main()
