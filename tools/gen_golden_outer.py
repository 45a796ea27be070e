#!/usr/bin/env python3
"""Golden vectors for the outer objective PSVI.psvi_elbo (+ sampled_nkl).

Runs ONLY in the development container (the reference is mounted read-only at
/root/reference).  Like tools/gen_golden.py, the parent re-launches this
script in a child interpreter whose sys.path holds the reference and not this
repo.  The child drives the reference's own

  * ``PSVI.psvi_elbo``                 psvi/inference/psvi_classes.py:445-486
  * ``VIMixin.sampled_nkl``            psvi/models/neural_net.py:110-115
  * ``MultivariateNormalVIMixin.sampled_nkl``  neural_net.py:438-442

in float64 (``torch.set_default_dtype(torch.float64)``: the reference's fp32
``MultivariateNormal.log_prob`` triangular solve loses the sampled-KL term at
realistic sizes), with every Monte-Carlo draw rounded
to fp32 first so the HIP path (fp32 eps) sees the identical noise.  It records
the loss and ``loss.backward()``'s gradients w.r.t. the model parameters, u, v
(and alpha for PSVIAV) into tests/golden/o*.npz (data only).

Usage:  python tools/gen_golden_outer.py
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

    gen = torch.Generator().manual_seed(4321)

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

    def run(name, family, model, cls, M, Nx, D, C, S, N, seed, v_scale=0.0, alpha=None,
            note="", shape=None):
        torch.manual_seed(seed)
        dims = shape or (D,)
        u = torch.randn(M, *dims, generator=gen).float().double().requires_grad_(True)
        z = torch.tensor([float(i % C) for i in range(M)])
        xb = torch.randn(Nx, *dims, generator=gen).float().double()
        yb = torch.randint(0, C, (Nx,), generator=gen).double()
        v = (v_scale * torch.randn(M, generator=gen)).float().double().requires_grad_(True)
        obj = cls.__new__(cls)
        obj.u, obj.z, obj.v, obj.N = u, z, v, N
        obj.distr_fn = categorical_fn
        obj.learn_z = False
        obj.mc_samples = S
        obj.nc = C
        if cls is PSVIAV:
            obj.alpha = torch.tensor([alpha], requires_grad=True)
            obj.f = lambda *x: torch.exp(obj.alpha) * torch.softmax(x[0], x[1])
        else:
            obj.f = torch.softmax
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        draws.clear()
        loss = obj.psvi_elbo(xb, yb, model=model)
        eps = torch.cat(draws).numpy()
        loss.backward()
        gp = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).numpy()
        # the identity behind the sampled-KL restatement: L^-1 (x_s - mean) = eps_s
        if family == "mvn":
            off = 0
            for mod in model.modules():
                if isinstance(mod, VILinearMultivariateNormal):
                    n = mod.num_params
                    x = torch.cat([getattr(mod, k).flatten(1) for k in mod.param_names], 1)
                    e = torch.tensor(eps[off:off + S * n]).reshape(S, n)
                    sol = torch.linalg.solve_triangular(mod.scale_tril.detach(),
                                                        (x.detach() - mod.mean.detach()).T,
                                                        upper=False).T
                    assert float((sol - e).abs().max()) < 1e-8, name
                    off += S * n
        w = (obj.N * obj.f(obj.v, 0)).detach()
        cfg = dict(family=family, layers=layer_sizes(model), S=S, M=M, Nx=Nx, N=N,
                   prior_sd=1.0, f="exp_alpha_softmax" if cls is PSVIAV else "softmax",
                   alpha=alpha, seed=seed, note=note)
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            config=np.array(json.dumps(cfg)),
            params0=p0.numpy().astype(np.float32),
            u=u.detach().numpy().astype(np.float32), z=z.numpy().astype(np.float32),
            xb=xb.numpy().astype(np.float32), yb=yb.numpy().astype(np.float32),
            v=v.detach().numpy().astype(np.float32), w=w.numpy(),
            eps=eps.astype(np.float32),
            loss=np.array(float(loss.detach())),
            grad_params=gp, grad_u=u.grad.numpy(), grad_v=v.grad.numpy(),
            grad_alpha=(obj.alpha.grad.numpy() if cls is PSVIAV else np.zeros(1)),
        )
        print(f"wrote {name}: P={p0.numel()} loss={float(loss):.6f}")

    # O1: logistic_regression (psvi_classes.py:694-699), perturbed posterior
    model = nn.Sequential(VILinear(2, 2, init_sd=0.1, mc_samples=4))
    perturb(model, 0.5, -3.0, 0.5, 0.0)
    run("o1_logreg", "mf", model, PSVILearnV, M=10, Nx=16, D=2, C=2, S=4, N=800, seed=1,
        v_scale=0.3, note="logreg, PSVILearnV")

    # O2: fn 1x100 (C2 shape), PSVIAV weights
    model = make_fcnet(2, 100, 4, n_layers=1, mc_samples=32, init_sd=0.1)
    perturb(model, 0.3, -4.0, -1.0, 0.0)
    run("o2_fn_c2_av", "mf", model, PSVIAV, M=50, Nx=32, D=2, C=4, S=32, N=800, seed=2,
        v_scale=0.3, alpha=0.25, note="fn C2 shape, PSVIAV")

    # O3: deeper mean-field MLP, odd sizes
    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05)
    perturb(model, 0.4, -3.0, -1.0, 0.0)
    run("o3_fn_deep", "mf", model, PSVILearnV, M=13, Nx=9, D=5, C=3, S=6, N=500, seed=3,
        v_scale=0.2, note="2 hidden layers")

    # O4: fn2-tiny full-cov (make_fc2net), nonzero _corr
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
    perturb(model, 0.3, -3.5, -2.5, 0.002)
    run("o4_fn2_tiny", "mvn", model, PSVILearnV, M=10, Nx=12, D=8, C=3, S=16, N=800, seed=4,
        v_scale=0.2, note="fn2 tiny perturbed")

    # O5: fn2-mid full-cov, PSVIAV
    model = make_fc2net(16, 8, 2, mc_samples=32, init_sd=1e-2)
    perturb(model, 0.2, -3.5, -2.5, 0.001)
    run("o5_fn2_mid_av", "mvn", model, PSVIAV, M=20, Nx=24, D=16, C=2, S=32, N=800, seed=5,
        v_scale=0.2, alpha=-0.3, note="fn2 mid, PSVIAV")

    # O6: logistic_regression_fullcov
    model = nn.Sequential(VILinearMultivariateNormal(2, 2, init_sd=0.1, mc_samples=4))
    perturb(model, 0.5, -3.0, -1.0, 0.02)
    run("o6_logreg_fullcov", "mvn", model, PSVILearnV, M=10, Nx=16, D=2, C=2, S=4, N=800,
        seed=6, v_scale=0.3, note="logistic_regression_fullcov")

    # evaluate (psvi_classes.py:1031-1108): one test batch, correction on and off
    def run_eval(name, family, model, cls, M, Nt, D, C, S, N, seed, v_scale=0.0, alpha=None,
                 shape=None):
        torch.manual_seed(seed)
        dims = shape or (D,)
        u = torch.randn(M, *dims, generator=gen).float().double()
        z = torch.tensor([float(i % C) for i in range(M)])
        xt = torch.randn(Nt, *dims, generator=gen).float().double()
        yt = torch.randint(0, C, (Nt,), generator=gen).double()
        v = (v_scale * torch.randn(M, generator=gen)).float().double()
        obj = cls.__new__(cls)
        obj.u, obj.z, obj.v, obj.N = u, z, v, N
        obj.distr_fn, obj.learn_z = categorical_fn, False
        obj.mc_samples, obj.nc, obj.num_pseudo = S, C, M
        obj.compute_weights_entropy, obj.device = True, torch.device("cpu")
        obj.test_loader = [(xt, yt)]
        obj.results = {"alpha": []}
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
            acc, nll, ent, ness, vent = obj.evaluate(correction=corr)
            out["eps" + tag] = torch.cat(draws).numpy().astype(np.float32)
            out["acc" + tag] = np.array(float(acc))
            out["nll" + tag] = np.array(float(nll))
            out["went" + tag] = np.array(float(ent))
            out["ness" + tag] = np.array(float(ness))
            out["vent" + tag] = np.array(float(vent))
        w = (obj.N * obj.f(obj.v, 0)).detach()
        cfg = dict(family=family, layers=layer_sizes(model), S=S, M=M, Nt=Nt, N=N, prior_sd=1.0,
                   f="exp_alpha_softmax" if cls is PSVIAV else "softmax", alpha=alpha, seed=seed)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), config=np.array(json.dumps(cfg)),
                            params0=p0.numpy().astype(np.float32),
                            u=u.numpy().astype(np.float32), z=z.numpy().astype(np.float32),
                            xt=xt.numpy().astype(np.float32), yt=yt.numpy().astype(np.float32),
                            v=v.numpy().astype(np.float32), w=w.numpy(), **out)
        print(f"wrote {name}: acc={float(out['acc']):.4f} nll={float(out['nll']):.4f} "
              f"ness={float(out['ness']):.4f}")

    with torch.no_grad():
        model = nn.Sequential(VILinear(2, 2, init_sd=0.1, mc_samples=8))
        perturb(model, 0.5, -3.0, 0.5, 0.0)
        run_eval("e1_logreg", "mf", model, PSVILearnV, M=10, Nt=40, D=2, C=2, S=8, N=800,
                 seed=41, v_scale=0.3)
        model = make_fcnet(2, 100, 4, n_layers=1, mc_samples=16, init_sd=0.1)
        perturb(model, 0.3, -4.0, -1.0, 0.0)
        run_eval("e2_fn_av", "mf", model, PSVIAV, M=20, Nt=64, D=2, C=4, S=16, N=800, seed=42,
                 v_scale=0.3, alpha=0.25)
        model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
        perturb(model, 0.3, -3.5, -2.5, 0.002)
        run_eval("e3_fn2_tiny", "mvn", model, PSVILearnV, M=10, Nt=50, D=8, C=3, S=16, N=800,
                 seed=43, v_scale=0.2)
        model = nn.Sequential(VILinearMultivariateNormal(2, 2, init_sd=0.1, mc_samples=4))
        perturb(model, 0.5, -3.0, -1.0, 0.02)
        run_eval("e4_logreg_fullcov", "mvn", model, PSVILearnV, M=10, Nt=30, D=2, C=2, S=4,
                 N=800, seed=44, v_scale=0.3)

    # LeNet (make_lenet, neural_net.py:334-359): sampled_nkl over VILinear only,
    # the last layer one shared sample; MNIST-shaped rows
    from psvi.models.neural_net import make_lenet

    model = make_lenet(mc_samples=3, init_sd=0.05)
    perturb(model, 0.15, -4.0, -2.0, 0.0)
    run("o7_lenet", "lenet", model, PSVILearnV, M=4, Nx=5, D=784, C=10, S=3, N=60000, seed=7,
        v_scale=0.3, note="lenet, PSVILearnV", shape=(1, 28, 28))
    model = make_lenet(mc_samples=4, init_sd=0.05)
    perturb(model, 0.2, -3.5, -2.0, 0.0)
    run("o8_lenet_av", "lenet", model, PSVIAV, M=3, Nx=4, D=784, C=10, S=4, N=60000, seed=8,
        v_scale=0.3, alpha=0.2, note="lenet, PSVIAV", shape=(1, 28, 28))
    with torch.no_grad():
        # mild weights: test probabilities stay above fp32's clamp (1.2e-7), which
        # the float64 reference run would not apply
        model = make_lenet(mc_samples=4, init_sd=0.05)
        perturb(model, 0.03, -4.0, -2.0, 0.0)
        run_eval("e5_lenet", "lenet", model, PSVILearnV, M=4, Nt=12, D=784, C=10, S=4,
                 N=60000, seed=45, v_scale=0.3, shape=(1, 28, 28))


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
