"""Bisect the network phase of the row-sharded full-cov step (C4 at world 8):
world-1 G / NLL against the world-W network kernel (multi-source x, role
split, pseudopoint chunks) on identical x, varying the split knob.

  python tools/net_msrc_probe.py [W] [S] [M]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]

from psvi.runtime import InnerLoopPlan, _lib  # noqa: E402
from psvi.runtime.sharded import ShardedInnerLoop  # noqa: E402
from test_hip_fullsize import make_case  # noqa: E402

DEV = "cuda"
W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
M = int(sys.argv[3]) if len(sys.argv) > 3 else 200
layers = [(64, 40), (40, 40), (40, 2)]
lib = _lib.load()
params, u, z, w, eps = make_case("fullcov", layers, S, M, 3)
t = lambda x, d=torch.float32: torch.tensor(x, dtype=d, device=DEV)
du, dz, dw, de, dp = t(u), t(z, torch.int32), t(w), t(eps), t(params)


def world1(split_below):
    lib.psvi_debug_set(5, split_below)
    plan = InnerLoopPlan("fullcov", layers, S, M)
    lib.psvi_debug_set(5, 256)
    xs = torch.empty(plan.xshard_count, device=DEV)
    gs = torch.empty(plan.xshard_count, device=DEV)
    nll = torch.zeros(1, dtype=torch.float64, device=DEV)
    plan.mvn_sample(de, dp, xs)
    plan.mvn_net(du, dz, dw, xs, gs, nll)
    torch.cuda.synchronize()
    return xs.view(S, -1), gs.view(S, -1).cpu().numpy(), nll.item()


def worldW(split_below, X):
    lib.psvi_debug_set(5, split_below)
    loops = [ShardedInnerLoop("fullcov", layers, S, M, W, r) for r in range(W)]
    lib.psvi_debug_set(5, 256)
    info = loops[0].info
    n_l = [a * b + b for a, b in layers]
    woff = np.concatenate([[0], np.cumsum(n_l)]).astype(int)
    G = np.zeros((S, woff[-1]))
    nll = 0.0
    for r in range(W):
        me = info[r]
        s0, sc = me["s_offset"], me["s_count"]
        # x_recv: this rank's samples, blocked by source rank q: [sc][rows_q]
        parts = []
        for q in range(W):
            cols = []
            for (l, lo, cnt, _) in info[q]["runs"]:
                cols.append(X[s0:s0 + sc, woff[l] + lo:woff[l] + lo + cnt])
            parts.append(torch.cat(cols, 1).reshape(-1))
        loops[r].x_recv.copy_(torch.cat(parts))
        loops[r].phase_net(du, dz, dw)
        torch.cuda.synchronize()
        nll += loops[r].parts[0].item()
        gsend = loops[r].g_send.cpu().numpy()
        o = 0
        for q in range(W):
            blk = gsend[o:o + sc * info[q]["rows"]].reshape(sc, info[q]["rows"])
            for (l, lo, cnt, c) in info[q]["runs"]:
                G[s0:s0 + sc, woff[l] + lo:woff[l] + lo + cnt] = blk[:, c:c + cnt]
            o += sc * info[q]["rows"]
    return G, nll


def cmp(name, G, nll, G1, nll1):
    per = np.linalg.norm(G - G1, axis=1) / np.maximum(np.linalg.norm(G1, axis=1), 1e-30)
    print(f"{name}: nll {nll:.6f} vs {nll1:.6f} (rel {abs(nll - nll1) / abs(nll1):.2e}); "
          f"samples off {int((per > 1e-4).sum())} max per-sample {per.max():.2e}", flush=True)


X1, G1, nll1 = world1(256)
print(f"world 1 default: nll {nll1:.6f}")
Xb, G1b, nll1b = world1(1 << 20)   # roles 2 on one source
cmp("world 1, roles 2", G1b, nll1b, G1, nll1)
for sb, nm in ((256, "default"), (0, "roles 1"), (1 << 20, "roles 2")):
    for rep in range(2):
        G, nll = worldW(sb, X1)
        cmp(f"world {W} {nm} rep {rep}", G, nll, G1, nll1)
