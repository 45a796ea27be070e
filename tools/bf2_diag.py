#!/usr/bin/env python3
"""One fused step (psvi_inner_loop T = 1, KEEP: the last step is the streaming
update) with the eight-wave and the four-wave bf16-piece kernels
(PSVI_DBG_STREAM_BF2_OFF): where the packed params / m / v and the next
sample x differ (per layer and part, entries off by more than 1e-6 rel)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
from psvi.runtime import InnerLoopPlan  # noqa: E402
from psvi.runtime import _lib as L  # noqa: E402


def main():
    layers = [(64, 40), (40, 40), (40, 2)]
    S, M = 128, 24
    rng = np.random.default_rng(3)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
                  (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
    p0 = np.concatenate(parts).astype(np.float32)
    dev = "cuda"
    u = torch.tensor(rng.standard_normal((M, 64)).astype(np.float32), device=dev)
    z = torch.tensor(rng.integers(0, 2, M).astype(np.int32), device=dev)
    w = torch.full((M,), 8.0, device=dev)
    lib = L.load()
    res = {}
    for off in (0, 1, 2):
        plan = InnerLoopPlan("fullcov", layers, S, M)
        lib.psvi_debug_set(28, 1 if off == 1 else 0)
        p = torch.tensor(p0, device=dev)
        m = 1e-3 * torch.ones_like(p)
        v = 1e-6 * torch.ones_like(p)
        ws = torch.zeros(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
        plan.inner_loop(u, z, w, p, m, v, 1, 1e-3, seed=5, ws=ws, keep=True)
        torch.cuda.synchronize()
        x = ws[:S * plan.xshard_count // S * 4].view(torch.float32)[:plan.xshard_count].clone()
        res[off] = [t.cpu().numpy() for t in (p, m, v, x)]
    lib.psvi_debug_set(28, 0)
    names = ("p", "m", "v", "x")
    for i, nm in enumerate(names):
        a, b = res[0][i], res[2][i]
        d = np.nonzero(a != b)[0]
        print(f"eight-wave run to run, {nm}: {d.size} differ", [(int(k), float(a[k]), float(b[k])) for k in d[:4]])
    bad = np.nonzero((np.abs(res[0][2]) < 1e-30) & (np.abs(res[1][2]) > 1e-20))[0]
    print("v garbage entries:", bad.size, bad[:20])
    for i, nm in enumerate(names):
        a, b = res[0][i], res[1][i]
        d = np.abs(a - b) > 1e-6 * np.maximum(np.abs(b), 1e-30)
        print(f"{nm}: {int(d.sum())} of {d.size} differ; max |d| {np.abs(a - b).max():.3e}")
        worst = np.argsort(-np.abs(a - b))[:8]
        print("   worst:", [(int(i0), float(a[i0]), float(b[i0])) for i0 in worst])
        if nm == "x":
            continue
        po = 0
        for l, (din, dout) in enumerate(layers):
            n = din * dout + dout
            nc = (n - 1) * (n - 2) // 2
            for part, lo, cnt in (("mean", po, n), ("sd", po + n, n), ("corr", po + 2 * n, nc)):
                dd = d[lo:lo + cnt]
                if dd.any():
                    idx = np.nonzero(dd)[0]
                    rows = []
                    for i0 in idx[:6]:
                        if part == "corr":
                            r = int((1 + np.sqrt(1 + 8 * i0)) // 2)
                            while r * (r - 1) // 2 > i0:
                                r -= 1
                            while (r + 1) * r // 2 <= i0:
                                r += 1
                            rows.append((r, i0 - r * (r - 1) // 2))
                        else:
                            rows.append(int(i0))
                    print(f"   L{l} {part}: {int(dd.sum())} differ, first {rows}; "
                          f"values {[(float(a[lo + i0]), float(b[lo + i0])) for i0 in idx[:3]]}")
            po += 2 * n + nc


if __name__ == "__main__":
    main()
