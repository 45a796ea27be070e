#!/usr/bin/env python3
"""Per-phase / per-segment HIP-vs-oracle errors for a full-cov config."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import psvi_oracle as O  # noqa: E402
from psvi.runtime import InnerLoopPlan  # noqa: E402
from test_hip_fullsize import make_case  # noqa: E402


def plan_mc(plan):
    M = plan.M
    for m in range(1, M + 1):
        pass
    return "?"


def main(S, M, layers=((64, 40), (40, 40), (40, 2))):
    layers = [tuple(l) for l in layers]
    params, u, z, w, eps = make_case("fullcov", layers, S, M, 3)
    plan = InnerLoopPlan("fullcov", layers, S, M)
    t = lambda x, d=torch.float32: torch.tensor(x, dtype=d, device="cuda")
    dp, du, dz, dw, de = t(params), t(u), t(z, torch.int32), t(w), t(eps)
    xs = torch.empty(plan.xshard_count, device="cuda")
    gs = torch.zeros(plan.xshard_count, device="cuda")
    nll = torch.zeros(1, dtype=torch.float64, device="cuda")
    plan.mvn_sample(de, dp, xs)
    plan.mvn_net(du, dz, dw, xs, gs, nll)
    grad = torch.empty_like(dp)
    kl = torch.zeros(1, dtype=torch.float64, device="cuda")
    plan.mvn_update(de, gs, dp, grad_out=grad, kl_out=kl)
    torch.cuda.synchronize()
    X = xs.view(S, -1).cpu().numpy().astype(np.float64)
    G = gs.view(S, -1).cpu().numpy().astype(np.float64)
    # oracle pieces
    po = eo = col = 0
    Ws, bs, Xo = [], [], []
    for din, dout in layers:
        n = din * dout + dout
        nc = (n - 1) * (n - 2) // 2
        L = O.mvn_dense_L(params[po + n:po + 2 * n], params[po + 2 * n:po + 2 * n + nc], n)
        E = eps[eo:eo + S * n].reshape(S, n).astype(np.float64)
        Xl = params[po:po + n][None] + E @ L.T
        Xo.append(Xl)
        Ws.append(Xl[:, :din * dout].reshape(S, dout, din))
        bs.append(Xl[:, din * dout:])
        po += 2 * n + nc
        eo += S * n
    Xo = np.concatenate(Xo, 1)
    print(f"S={S} M={M}  X l2rel {O.np.linalg.norm(X - Xo) / np.linalg.norm(Xo):.3e}")
    data, dWs, dbs = O.net_forward_backward(u.astype(np.float64), z, w.astype(np.float64), Ws, bs)
    Go = np.concatenate([np.concatenate([dWs[l].reshape(S, -1), dbs[l]], 1) for l in range(len(layers))], 1)
    print(f"  G l2rel {np.linalg.norm(G - Go) / np.linalg.norm(Go):.3e}  nll {nll.item():.6f} vs {data:.6f}"
          f"  mc={plan_mc(plan)}")
    col = 0
    for li, (din, dout) in enumerate(layers):
        n = din * dout + dout
        d = np.abs(G[:, col:col + n] - Go[:, col:col + n])
        s_w, i_w = np.unravel_index(np.argmax(d), d.shape)
        rows_bad = np.where(d.max(1) > 1e-3 * np.abs(Go[:, col:col + n]).max())[0]
        print(f"  G layer {li}: l2rel {np.linalg.norm(d) / np.linalg.norm(Go[:, col:col + n]):.3e} "
              f"worst (s={s_w}, i={i_w}) bad samples {rows_bad[:12].tolist()} (#{len(rows_bad)})")
        col += n
    val, go = O.mvn_elbo_grad(layers, params, u, z, w, eps, S)
    g = grad.cpu().numpy()
    po = 0
    for li, (din, dout) in enumerate(layers):
        n = din * dout + dout
        nc = (n - 1) * (n - 2) // 2
        for nm, a, b in (("mean", po, po + n), ("sd", po + n, po + 2 * n), ("corr", po + 2 * n, po + 2 * n + nc)):
            e = np.linalg.norm(g[a:b] - go[a:b]) / max(np.linalg.norm(go[a:b]), 1e-30)
            print(f"  layer {li} {nm:5s} l2rel {e:.3e}  worst idx {a + int(np.argmax(np.abs(g[a:b] - go[a:b])))}")
        po += 2 * n + nc


if __name__ == "__main__":
    for S, M in ((1024, 100), (128, 200), (64, 200), (1024, 200), (16, 100)):
        main(S, M)
