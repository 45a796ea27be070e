#!/usr/bin/env python3
"""Diagnostics for the bf16-piece streaming update: psvi_inner_loop (Philox
mode, T steps) with the bf16-piece kernel and with the fp32 streaming kernel
(PSVI_DBG_STREAM_BF_OFF) against the float64 oracle on the same draws;
per layer and parameter group (mean, sd, corr) the l2 and max errors of each
path and where the largest bf16-piece error sits.

  python3 tools/bf_diag.py [c3|small] [T]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import psvi_oracle as O  # noqa: E402
from psvi.runtime import InnerLoopPlan, randn_  # noqa: E402
from psvi.runtime import _lib as L  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    layers = [(64, 40), (40, 40), (40, 2)] if cfg == "c3" else [(7, 5), (5, 3)]
    S, M, seed = 128, 24, 77
    rng = np.random.default_rng(3)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
                  (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
    p0 = np.concatenate(parts).astype(np.float32)
    u = rng.standard_normal((M, layers[0][0])).astype(np.float32)
    z = rng.integers(0, layers[-1][1], M).astype(np.int32)
    w = O.coreset_weights(0.3 * rng.standard_normal(M), 800).astype(np.float32)
    plan = InnerLoopPlan("fullcov", layers, S, M)
    lib = L.load()
    dev = "cuda"
    res = {}
    for bf in (1, 0):
        lib.psvi_debug_set(24, 0 if bf else 1)
        p = torch.tensor(p0, device=dev)
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        e = plan.inner_loop(torch.tensor(u, device=dev), torch.tensor(z, device=dev),
                            torch.tensor(w, device=dev), p, m, v, T, 1e-3, seed=seed)
        res[bf] = [x.cpu().numpy().astype(np.float64) for x in (e, p, m)]
    lib.psvi_debug_set(24, 0)
    draws = []
    for k in range(T):
        e = torch.empty(plan.eps_count, device=dev)
        randn_(e, seed, k * plan.eps_stride)
        draws.append(e.cpu().numpy().astype(np.float64))
    o_e, o_g, o_traj, o_m, _ = O.run_inner_loop("mvn", layers, p0, u, z, w, draws, S, 1e-3, "higher")
    print("elbo bf", res[1][0], "fp32", res[0][0], "oracle", o_e)
    po = 0
    for l, (din, dout) in enumerate(layers):
        n = din * dout + dout
        nc = (n - 1) * (n - 2) // 2
        for name, lo, cnt in (("mean", po, n), ("sd", po + n, n), ("corr", po + 2 * n, nc)):
            sl = slice(lo, lo + cnt)
            out = [f"L{l} {name:4s}"]
            for tag, arr in (("p", 1), ("m", 2)):
                ref = o_traj[-1][sl] if tag == "p" else o_m[sl]
                for bf in (1, 0):
                    d = res[bf][arr][sl] - ref
                    out.append(f"{tag}{'bf' if bf else '32'} l2 {np.linalg.norm(d) / max(np.linalg.norm(ref), 1e-30):.1e}"
                               f" max {np.abs(d).max():.1e}")
            print("  ".join(out))
            if name == "corr":
                d = np.abs(res[1][2][sl] - o_m[sl])
                i = int(d.argmax())
                r = int((1 + np.sqrt(1 + 8 * i)) // 2)
                while r * (r - 1) // 2 > i:
                    r -= 1
                while (r + 1) * r // 2 <= i:
                    r += 1
                c = i - r * (r - 1) // 2
                d32 = abs(res[0][2][lo + i] - o_m[lo + i])
                print(f"      worst bf corr entry: row {r} col {c} (band {r // 64}, tile col {c // 64}): "
                      f"bf {res[1][2][lo + i]:.6e} fp32 {res[0][2][lo + i]:.6e} oracle {o_m[lo + i]:.6e} "
                      f"(fp32 err {d32:.1e})")
        po += 2 * n + nc


if __name__ == "__main__":
    main()
