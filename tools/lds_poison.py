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

CFGS = [("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100), ("fullcov", [(64, 40), (40, 40), (40, 2)], 1024, 200),
        ("fullcov", [(9, 5), (5, 3)], 130, 129), ("meanfield", [(7, 33), (33, 5), (5, 3)], 130, 129),
        ("fullcov", [(9, 5), (5, 3)], 33, 7), ("meanfield", [(64, 64), (64, 10)], 16, 200)]


def main():
    g = torch.Generator().manual_seed(0)
    for fam, layers, S, M in CFGS:
        plan = InnerLoopPlan(fam, layers, S, M)
        D = layers[0][0]
        u = torch.randn(M, D, generator=g).cuda()
        z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).cuda()
        w = torch.full((M,), 3.0).cuda()
        p = (torch.randn(plan.param_count, generator=g) * 0.05).cuda()
        if fam == "fullcov":
            # sd entries in a sane range
            pass
        eps = torch.randn(plan.eps_count, generator=g).cuda()
        res = []
        for abl in (0, 128):
            plan.lib.psvi_debug_set(1, abl)
            try:
                e, gr = plan.elbo_grad(u, z, w, eps, p)
                torch.cuda.synchronize()
            finally:
                plan.lib.psvi_debug_set(1, 0)
            res.append((float(e.item()), bool(torch.isfinite(gr).all())))
        print(f"{fam} {layers} S={S} M={M}: plain elbo {res[0][0]:.6g} grad finite {res[0][1]}; "
              f"poisoned elbo {res[1][0]:.6g} grad finite {res[1][1]}", flush=True)


if __name__ == "__main__":
    main()
