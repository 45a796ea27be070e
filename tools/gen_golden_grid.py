#!/usr/bin/env python3
"""Golden vectors for PSVI.pred_on_grid (psvi/inference/psvi_classes.py:1130-1175).

Runs ONLY in the development container (the reference is mounted read-only at
/root/reference).  Like tools/gen_golden_outer.py, the parent re-launches this
script in a child interpreter whose sys.path holds the reference and not this
repo.  The child sets up a reference PSVI object the way gen_golden_outer's
evaluate fixtures do (float64, every Monte-Carlo draw rounded to fp32 and
recorded), calls the reference's own ``pred_on_grid`` with and without the
importance-weight correction, and writes the draws and the grid probabilities
into tests/golden/p*.npz (data only).

Usage:  python tools/gen_golden_grid.py
"""
import json
import os
import subprocess
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _child():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gen_golden import _install_stubs

    _install_stubs()
    import numpy as np
    import torch
    import torch.distributions.multivariate_normal as mvn_mod
    import torch.distributions.normal as normal_mod
    import torch.nn as nn
    from torch.nn.utils import parameters_to_vector

    from psvi.inference.psvi_classes import PSVIAV, PSVILearnV
    from psvi.models.neural_net import (VILinear, VILinearMultivariateNormal,
                                        categorical_fn, make_fc2net, make_fcnet)

    torch.set_default_dtype(torch.float64)
    draws = []

    def wrap(orig):
        def f(shape, dtype, device):
            out = orig(shape, dtype=dtype, device=device).float().to(dtype)
            draws.append(out.detach().clone().reshape(-1))
            return out
        return f

    for m in (normal_mod, mvn_mod):
        m._standard_normal = wrap(m._standard_normal)

    gen = torch.Generator().manual_seed(2718)

    def perturb(model, mu_scale, rho_lo, rho_hi, corr_scale):
        with torch.no_grad():
            for name, p in model.named_parameters():
                leaf = name.split(".")[-1]
                if leaf in ("weight", "bias", "mean"):
                    p.copy_(mu_scale * torch.randn(p.shape, generator=gen))
                elif leaf in ("_weight_sd", "_bias_sd", "_sd"):
                    p.copy_(rho_lo + (rho_hi - rho_lo) * torch.rand(p.shape, generator=gen))
                elif leaf == "_corr":
                    p.copy_(corr_scale * torch.randn(p.shape, generator=gen))
                p.copy_(p.float().double())  # fp32-representable parameters

    def layer_sizes(model):
        return [[m.in_features, m.out_features] for m in model.modules()
                if isinstance(m, (VILinear, VILinearMultivariateNormal))]

    def run_grid(name, family, model, cls, M, C, S, N, seed, n_dim, v_scale=0.3, alpha=None):
        torch.manual_seed(seed)
        u = (1.5 * torch.randn(M, 2, generator=gen)).float().double()
        z = torch.tensor([float(i % C) for i in range(M)])
        v = (v_scale * torch.randn(M, generator=gen)).float().double()
        obj = cls.__new__(cls)
        obj.u, obj.z, obj.v, obj.N = u, z, v, N
        obj.distr_fn, obj.learn_z = categorical_fn, False
        obj.mc_samples, obj.nc, obj.num_pseudo = S, C, M
        obj.device = torch.device("cpu")
        if cls is PSVIAV:
            obj.alpha = torch.tensor([alpha])
            obj.f = lambda *x: torch.exp(obj.alpha) * torch.softmax(x[0], x[1])
        else:
            obj.f = torch.softmax
        obj.model = model
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        out = {}
        for tag, corr in (("", True), ("_nc", False)):
            draws.clear()
            probs = obj.pred_on_grid(n_test_per_dim=n_dim, correction=corr)
            out["eps" + tag] = torch.cat(draws).numpy().astype(np.float32)
            out["probs" + tag] = probs.numpy()
        w = (obj.N * obj.f(obj.v, 0)).detach()
        cfg = dict(family=family, layers=layer_sizes(model), S=S, M=M, N=N, prior_sd=1.0,
                   f="exp_alpha_softmax" if cls is PSVIAV else "softmax", alpha=alpha, seed=seed,
                   n_test_per_dim=n_dim)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), config=np.array(json.dumps(cfg)),
                            params0=p0.numpy().astype(np.float32),
                            u=u.numpy().astype(np.float32), z=z.numpy().astype(np.float32),
                            v=v.numpy().astype(np.float32), w=w.numpy(), **out)
        print(f"wrote {name}: grid {tuple(out['probs'].shape)} "
              f"max {float(out['probs'].max()):.4f} min {float(out['probs'].min()):.3e}")

    with torch.no_grad():
        # logistic_regression (psvi_classes.py:694-699), mean-field
        model = nn.Sequential(VILinear(2, 3, init_sd=0.1, mc_samples=8))
        perturb(model, 0.5, -3.0, 0.5, 0.0)
        run_grid("p1_grid_logreg", "mf", model, PSVILearnV, M=9, C=3, S=8, N=800, seed=51,
                 n_dim=21)
        # fn 1 x 50 mean-field, PSVIAV weights
        model = make_fcnet(2, 50, 4, n_layers=1, mc_samples=16, init_sd=0.1)
        perturb(model, 0.3, -4.0, -1.0, 0.0)
        run_grid("p2_grid_fn_av", "mf", model, PSVIAV, M=12, C=4, S=16, N=800, seed=52,
                 n_dim=17, alpha=0.25)
        # fn2 full-cov (make_fc2net), nonzero _corr
        model = make_fc2net(2, 8, 2, mc_samples=16, init_sd=1e-2)
        perturb(model, 0.5, -3.5, -2.0, 0.01)
        run_grid("p3_grid_fn2", "mvn", model, PSVILearnV, M=10, C=2, S=16, N=800, seed=53,
                 n_dim=19)


def main():
    if "--child" in sys.argv:
        _child()
        return
    os.makedirs(OUT, exist_ok=True)
    env = dict(os.environ)
    env["PYTHONPATH"] = REF
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    subprocess.run([sys.executable, "-B", os.path.abspath(__file__), "--child"],
                   env=env, check=True, cwd="/tmp")


if __name__ == "__main__":
    main()
