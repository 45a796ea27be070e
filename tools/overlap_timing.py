#!/usr/bin/env python3
"""The sharded step's exchange overlap on ONE GPU: rank r of a W-rank C4 plan
runs ShardedInnerLoop.run() -- plain (x all_to_all, network, G all_to_all,
update) and overlap=True (sample halves: x(B) beside net(A), G(A) beside
net(B)) -- with each all_to_all replaced by a device copy of the bytes rank r receives
plus a spin of D us per whole exchange (a half exchange: D times its share of
the bytes) on the stream that issues it (standing in for the xGMI transfer).
Per-step device time (HIP events around T steps) against D, and the host's
issue time per step.

  python tools/overlap_timing.py [--world 8] [--rank 0] [--delays 0,10,20,40] [--T 30]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


class SpinComm:
    """all_to_all(_list) as copies of the right sizes + a spin of `us`."""
    name = "device copies + spin"
    host_staged = False

    def __init__(self, dev, us, cycles_per_us):
        self.us, self.cpu = us, cycles_per_us
        self.scratch = torch.randn(1 << 22, device=dev) * 0.1
        self.sink = torch.empty(1 << 22, device=dev)
        self.full = None  # numel of a whole x exchange (set by the caller)

    def _spin(self):
        if self.us > 0:
            torch.cuda._sleep(int(self.us * self.cpu))

    def all_to_all(self, out, inp, out_splits, in_splits):
        out.copy_(self.scratch[:out.numel()])
        self._spin()

    def all_to_all_list(self, outs, ins):
        # one copy of the list's total bytes (timing only: the contents are
        # scratch either way; a per-block copy would time the host, not the
        # GPU), the spin scaled by the share of a whole exchange's bytes
        tot = sum(o.numel() for o in outs)
        if tot:
            self.sink[:tot].copy_(self.scratch[:tot])
        if self.us > 0:
            frac = tot / self.full if self.full else 1.0
            torch.cuda._sleep(int(self.us * frac * self.cpu))

    def all_reduce(self, t):
        pass


def calibrate(dev):
    """torch.cuda._sleep cycles per microsecond on this device."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    n = 2_000_000
    a.record()
    torch.cuda._sleep(n)
    b.record()
    torch.cuda.synchronize()
    return n / (a.elapsed_time(b) * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--delays", default="0,10,20,40")
    ap.add_argument("--T", type=int, default=30)
    a = ap.parse_args()
    from bench import LR, fn2_inputs, reference_init_params
    from psvi.runtime.sharded import ShardedInnerLoop

    dev = torch.device("cuda", 0)
    layers, S, M = [(64, 40), (40, 40), (40, 2)], 1024, 200
    cpu = calibrate(dev)
    u, z, w = fn2_inputs(layers, M, dev, 0)
    out = []
    for us in [float(x) for x in a.delays.split(",")]:
        row = {"delay_us_per_exchange": us}
        for overlap in (False, True):
            comm = SpinComm(dev, us, cpu)
            loop = ShardedInnerLoop("fullcov", layers, S, M, a.world, a.rank, device=dev, comm=comm)
            comm.full = loop.x_recv.numel()
            p = reference_init_params(layers, dev)
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            loop.run(u, z, w, p, m, v, 5, LR, seed=1, overlap=overlap)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h0 = time.perf_counter()
            loop.run(u, z, w, p, m, v, a.T, LR, step0=6, seed=1, offset=5 * loop.plan.eps_stride,
                     overlap=overlap)
            h1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            tag = "overlap" if overlap else "plain"
            row[tag] = round(e0.elapsed_time(e1) / a.T * 1e3, 2)
            row[tag + "_host_issue"] = round((h1 - h0) / a.T * 1e6, 2)
        row["hidden_us"] = round(row["plain"] - row["overlap"], 2)
        out.append(row)
        print(json.dumps(dict(row, world=a.world, rank=a.rank, cfg="c4", unit="us per step")),
              flush=True)


if __name__ == "__main__":
    main()
