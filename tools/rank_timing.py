#!/usr/bin/env python3
"""Per-rank timing of the world > 1 full-cov inner step on ONE GPU.

The W ranks' plans of one sharded configuration are built in this process;
rank r's step phases run back to back on the GPU with the two all_to_alls
replaced by device copies of exactly the blocks rank r would receive (their
time is reported apart: on the node they are xGMI transfers).  Each phase is
bracketed by HIP events on the launch stream, averaged over --iters steps
after --warmup steps.  This is what one GPU of the 8-GPU node does per step,
minus the wire.

  python tools/rank_timing.py --cfg c4 --world 8 [--ranks 0,3,7] [--iters 50]
  python tools/rank_timing.py --cfg weak --world 8
  python tools/rank_timing.py --cfg c4 --world 8 --schedule run

--schedule phases (default): randn, sample, net, update as separate launches;
--schedule run: ShardedInnerLoop.run()'s steady-state step -- the network
launch also draws the next eps, the update launch also samples the next x.

cfg c4: fn2 64-40-40-2, S = 1024, M = 200 (BASELINE configs[3], strong
scaling); cfg weak: the bench headline at N = world (S = 128 world, M = 100).
Prints one JSON line per rank and a summary line.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

LAYERS = [(64, 40), (40, 40), (40, 2)]


def offs(splits):
    o = [0]
    for x in splits:
        o.append(o[-1] + x)
    return o


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", choices=("c4", "weak"), default="c4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--schedule", choices=("phases", "run"), default="phases")
    ap.add_argument("--dbg", action="append", default=[], help="KEY=VALUE psvi_debug_set before the plans (A/B)")
    a = ap.parse_args()
    from bench import LR, fn2_inputs, reference_init_params
    from psvi.runtime import _lib, randn_
    for kv in a.dbg:
        k, v = kv.split("=")
        _lib.load().psvi_debug_set(int(k), int(v))
    from psvi.runtime.sharded import ShardedInnerLoop

    W = a.world
    S, M = (1024, 200) if a.cfg == "c4" else (128 * W, 100)
    dev = torch.device("cuda", 0)
    loops = [ShardedInnerLoop("fullcov", LAYERS, S, M, W, r, device=dev) for r in range(W)]
    u, z, w = fn2_inputs(LAYERS, M, dev, 5)
    p0 = reference_init_params(LAYERS, dev)
    eps = torch.empty(loops[0].plan.eps_count, device=dev)
    stride = (loops[0].plan.eps_count + 3) // 4 * 4
    ranks = range(W) if a.ranks == "all" else [int(x) for x in a.ranks.split(",")]
    # one pass of every rank so that every x_shard / g_send holds real values
    params = [p0.clone() for _ in range(W)]
    ms = [torch.zeros_like(p0) for _ in range(W)]
    vs = [torch.zeros_like(p0) for _ in range(W)]
    randn_(eps, 11, 0)
    for r in range(W):
        loops[r].phase_sample(eps, params[r])

    def x_exchange(r):
        me = loops[r]
        parts = [loops[p].x_shard[offs(loops[p].x_in)[r]:offs(loops[p].x_in)[r + 1]]
                 for p in range(W)]
        torch.cat(parts, out=me.x_recv)

    def g_exchange(r):
        me = loops[r]
        parts = [loops[q].g_send[offs(loops[q].g_in)[r]:offs(loops[q].g_in)[r + 1]]
                 for q in range(W)]
        torch.cat(parts, out=me.g_shard)

    for r in range(W):
        x_exchange(r)
        loops[r].phase_net(u, z, w)
    names = ["randn", "sample", "x_exchange(copy)", "net", "g_exchange(copy)", "update"]
    if a.schedule == "run":
        names = ["x_exchange(copy)", "net+draw", "g_exchange(copy)", "update+sample"]
        e_nxt = torch.empty_like(eps)
    out = []
    for r in ranks:
        lp = loops[r]
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
              for _ in range(a.iters)]
        for k in range(a.warmup + a.iters):
            e = ev[k - a.warmup] if k >= a.warmup else None
            rec = (lambda i: e[i].record()) if e else (lambda i: None)
            if a.schedule == "run":
                rec(0)
                x_exchange(r)
                rec(1)
                lp.phase_net(u, z, w, draw=(e_nxt, 11, (k + 1) * stride))
                rec(2)
                g_exchange(r)
                rec(3)
                lp.phase_update_sample(eps, params[r], ms[r], vs[r], k + 1, LR, "higher", e_nxt)
                rec(4)
                continue
            rec(0)
            randn_(eps, 11, (k + 1) * stride)
            rec(1)
            lp.phase_sample(eps, params[r])
            rec(2)
            x_exchange(r)
            rec(3)
            lp.phase_net(u, z, w)
            rec(4)
            g_exchange(r)
            rec(5)
            lp.phase_update(eps, params[r], ms[r], vs[r], k + 1, LR, "higher")
            rec(6)
        torch.cuda.synchronize()
        us = {n: 1e3 * sum(e[i].elapsed_time(e[i + 1]) for e in ev) / a.iters
              for i, n in enumerate(names)}
        comp = sum(v for k_, v in us.items() if "exchange" not in k_)
        info = lp.info[r]
        row = dict(rank=r, cfg=a.cfg, schedule=a.schedule, world=W, S=S, M=M, s_local=info["s_count"],
                   rows=info["rows"], us={k_: round(v, 2) for k_, v in us.items()},
                   compute_us=round(comp, 2))
        print(json.dumps(row), flush=True)
        out.append(row)
    worst = max(o["compute_us"] for o in out)
    print(json.dumps(dict(summary=True, cfg=a.cfg, world=W, S=S, M=M,
                          max_compute_us=worst,
                          mean_compute_us=round(sum(o["compute_us"] for o in out) / len(out), 2))),
          flush=True)


if __name__ == "__main__":
    main()
