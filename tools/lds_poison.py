#!/usr/bin/env python3
"""Network kernel with its LDS poisoned with NaN before use (ablation bit 128):
every word it reads must be one it wrote (the padding contract).  Prints the
NLL and the gradient's finiteness per configuration, poisoned and not.

  python tools/lds_poison.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

MF3 = [(7, 33), (33, 5), (5, 3)]
FC2 = [(9, 5), (5, 3)]
FN2 = [(64, 40), (40, 40), (40, 2)]
CFGS = [("fullcov", FN2, 128, 100), ("fullcov", FN2, 1024, 200), ("fullcov", FC2, 130, 129),
        ("fullcov", FC2, 33, 7), ("meanfield", MF3, 130, 129), ("meanfield", MF3, 130, 100),
        ("meanfield", MF3, 130, 7), ("meanfield", MF3, 33, 129), ("meanfield", MF3, 256, 129),
        ("meanfield", MF3, 128, 129), ("meanfield", [(64, 64), (64, 10)], 16, 200)]


def params(fam, layers, gen):
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        if fam == "meanfield":
            parts += [0.3 * torch.randn(n, generator=gen), -4 + 3 * torch.rand(n, generator=gen)]
        else:
            parts += [0.1 * torch.randn(n, generator=gen), -5 + 2 * torch.rand(n, generator=gen),
                      (0.15 / n ** 0.5) * torch.randn((n - 1) * (n - 2) // 2, generator=gen)]
    return torch.cat(parts)


def main():
    g = torch.Generator().manual_seed(0)
    for fam, layers, S, M in CFGS:
        plan = InnerLoopPlan(fam, layers, S, M)
        D = layers[0][0]
        u = torch.randn(M, D, generator=g).cuda()
        z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).cuda()
        w = torch.full((M,), 3.0).cuda()
        p = params(fam, layers, g).cuda()
        assert p.numel() == plan.param_count
        eps = torch.randn(plan.eps_count, generator=g).cuda()
        res = []
        for abl in [0, 128] + [128 | (r << 8) for r in range(1, 7)]:
            plan.lib.psvi_debug_set(1, abl)
            try:
                e, gr = plan.elbo_grad(u, z, w, eps, p)
                torch.cuda.synchronize()
            finally:
                plan.lib.psvi_debug_set(1, 0)
            res.append((float(e.item()), bool(torch.isfinite(gr).all())))
        tag = " ".join(f"{'ok' if (r[1] and r[0] == r[0]) else 'NaN'}" for r in res)
        print(f"{fam} {layers} S={S} M={M}: plain elbo {res[0][0]:.6g} | plain, all, weights, X0, "
              f"tables, X_l, G_l, dl: {tag}", flush=True)


if __name__ == "__main__":
    main()
