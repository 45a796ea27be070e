#!/usr/bin/env python3
"""Golden vectors for the PSVI plugin variants (one whole outer step each).

Runs ONLY in the development container (the reference is mounted read-only at
/root/reference); like tools/gen_golden_hyper.py the parent re-launches this
script in a child interpreter whose sys.path holds the reference and not this
repo.  In float64 with every Monte-Carlo draw rounded to fp32, the child runs
the reference's own trainer methods of

  * PSVIAV        nested_step / hyper_step  (psvi_classes.py:1475-1620):
                  hparams [u, v, alpha], optim_alpha stepped;
  * PSVIFixedU    nested_step / hyper_step  (1622-1740): u frozen, only v moves;
  * PSVIAFixedU   nested_step / hyper_step  (1743-1883): u frozen, v and alpha;
  * PSVI_Ablated  psvi_elbo, nested_step, hyper_step (1388-1408): the outer
                  objective  mean_s data_nll_s - mean_s sampled_nkl_s  over the
                  data batch only (VILinear layers' sampled KL);
  * PSVI_No_IW    nested_step / hyper_step with mc_samples = 1 (1411-1472): the
                  inner objective of a single-sample VILinear model has 2-d
                  logits, which inner_elbo unsqueezes to (M, 1, C), so
                  Categorical.log_prob(z) broadcasts to (M, M) -- every pseudo
                  row is scored against every pseudo label.

and records every draw in call order (inner objective / outer objective), the
inputs, the outputs (loss, u, v, alpha, their gradients, final parameters) and
-- for nested steps -- the reference's own fp32 replay of the same draws
(the rounding bar of the unrolled hypergradient, as gen_golden_hyper does).
Trainer calls the reference cannot run (PSVIFixedU.hyper_step: a 3-way
DifferentiableAdam fp_map on the plain parameter list, psvi_classes.py:1710;
PSVI_Ablated on a full-covariance model: no VILinear module, so sampled_nkl is
the int 0) are recorded as the exception type they raise.

Usage:  python tools/gen_golden_variants.py
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
    import copy

    import numpy as np
    import torch
    import torch.distributions.multivariate_normal as mvn_mod
    import torch.distributions.normal as normal_mod
    import torch.nn as nn
    from torch.nn.utils import parameters_to_vector

    from psvi.inference import psvi_classes as PC
    from psvi.models.neural_net import (VILinear, VILinearMultivariateNormal, categorical_fn,
                                        make_fc2net, make_fcnet, make_lenet)

    torch.set_default_dtype(torch.float64)
    draws, replay = [], []

    def wrap(orig):
        def f(shape, dtype, device):
            if replay:
                out = replay.pop(0).reshape(shape).to(dtype)
            else:
                out = orig(shape, dtype=dtype, device=device).float().to(dtype)
            draws.append(out.detach().clone().reshape(-1))
            return out
        return f

    for m in (normal_mod, mvn_mod):
        m._standard_normal = wrap(m._standard_normal)

    gen = torch.Generator().manual_seed(4242)

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
                p.copy_(p.float().double())

    def layer_sizes(model):
        return [[m.in_features, m.out_features] for m in model.modules()
                if isinstance(m, (VILinear, VILinearMultivariateNormal))]

    LR = dict(lr0net=1e-3, lr0u=1e-3, lr0v=1e-2, lr0alpha=1e-2)

    def make_obj(cls, model, S, N, C, u0, v0, alpha0, T):
        """A reference variant instance without its dataset plumbing: the fields
        nested_step / hyper_step / psvi_elbo read (psvi_classes.py:83-227 and
        the subclasses' __init__)."""
        obj = cls.__new__(cls)
        obj.model = model
        obj.u = u0.detach().clone().requires_grad_(True)
        obj.z = torch.tensor([float(i % C) for i in range(u0.shape[0])])
        obj.v = v0.detach().clone().requires_grad_(True)
        obj.N, obj.nc, obj.mc_samples = N, C, S
        obj.distr_fn = categorical_fn
        obj.learn_z, obj.learn_v, obj.parameterised = False, True, True
        obj.inner_it, obj.register_elbos, obj.log_every = T, False, 10
        obj.scheduler_optim_net, obj.optim_z = None, None
        obj.f = torch.softmax
        obj.optim_net = torch.optim.Adam(list(model.parameters()), LR["lr0net"])
        obj.optim_u = torch.optim.Adam([obj.u], LR["lr0u"])
        obj.optim_v = torch.optim.Adam([obj.v], LR["lr0v"])
        if alpha0 is not None:
            obj.alpha = torch.tensor([alpha0]).requires_grad_(True)
            obj.f = lambda *x: torch.exp(obj.alpha) * torch.softmax(x[0], x[1])
            obj.optim_alpha = torch.optim.Adam([obj.alpha], LR["lr0alpha"])
        return obj

    def grad_np(t):
        return None if t.grad is None else t.grad.detach().numpy()

    def run(name, cls_name, trainer, family, model, M, Nx, D, C, S, N, T, K=3, seed=0,
            alpha0=None, approx="CG_normaleq", shape=None, note=""):
        cls = getattr(PC, cls_name)
        torch.manual_seed(seed)
        model32 = copy.deepcopy(model).float()
        u0 = torch.randn(M, *(shape or (D,)), generator=gen).float().double()
        v0 = (0.2 * torch.randn(M, generator=gen)).float().double()
        xb = torch.randn(Nx, *(shape or (D,)), generator=gen).float().double()
        yb = torch.randint(0, C, (Nx,), generator=gen).double()
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        obj = make_obj(cls, model, S, N, C, u0, v0, alpha0, T)
        cfg = dict(family=family, layers=layer_sizes(model), S=S, M=M, N=N, Nx=Nx, T=T, K=K,
                   prior_sd=1.0, cls=cls_name, trainer=trainer, seed=seed, approx=approx,
                   alpha0=alpha0, linsys_lr=1e-4, note=note, **LR)
        arrays = dict(params0=p0.numpy().astype(np.float32), u0=u0.numpy().astype(np.float32),
                      v0=v0.numpy().astype(np.float32), z=obj.z.numpy().astype(np.float32),
                      xb=xb.numpy().astype(np.float32), yb=yb.numpy().astype(np.float32))
        draws.clear()
        sizes, n_prev = [], [0]
        orig_inner, orig_outer = obj.inner_elbo, obj.psvi_elbo

        def tag(kind, orig):
            def f(*a, **k):
                r = orig(*a, **k)
                sizes.append((kind, len(draws) - n_prev[0]))
                n_prev[0] = len(draws)
                return r
            return f

        obj.inner_elbo, obj.psvi_elbo = tag("inner", orig_inner), tag("outer", orig_outer)
        try:
            if trainer == "psvi_elbo":
                loss = obj.psvi_elbo(xb, yb, model=model)
                loss.backward()
                out = float(loss.detach())
            elif trainer == "nested":
                out = float(obj.nested_step(xb, yb).detach())
            else:
                out = float(obj.hyper_step(xb, yb, K=K, linsys_lr=1e-4, hypergrad_approx=approx))
        except Exception as exc:  # the reference's own failure: record its type
            cfg["raises"] = type(exc).__name__
            cfg["message"] = str(exc)[:200]
            np.savez_compressed(os.path.join(OUT, name + ".npz"),
                                config=np.array(json.dumps(cfg)), **arrays)
            print(f"wrote {name}: reference raises {type(exc).__name__}: {str(exc)[:80]}")
            return
        recorded = [d.clone() for d in draws]
        cuts = np.cumsum([0] + [c for _, c in sizes])
        eps = [torch.cat(recorded[cuts[i]:cuts[i + 1]]).numpy().astype(np.float32)
               if cuts[i + 1] > cuts[i] else np.zeros(0, np.float32) for i in range(len(sizes))]
        cfg["calls"] = [k for k, _ in sizes]
        res = dict(out=np.array(out), u=obj.u.detach().numpy(), v=obj.v.detach().numpy(),
                   params=parameters_to_vector(model.parameters()).detach().numpy())
        for key, t in (("u_grad", obj.u), ("v_grad", obj.v)) + (
                (("alpha_grad", obj.alpha),) if alpha0 is not None else ()):
            g = grad_np(t)
            if g is not None:
                res[key] = g
        if alpha0 is not None:
            res["alpha"] = obj.alpha.detach().numpy()
        if trainer == "psvi_elbo":
            res["grad_params"] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).numpy()
        inner = [e for k, e in zip(cfg["calls"], eps) if k == "inner"]
        outer = [e for k, e in zip(cfg["calls"], eps) if k == "outer"]
        if inner:
            res["eps_inner"] = np.stack(inner)
        if outer:
            res["eps_outer"] = np.stack(outer)
        if trainer == "nested":
            # the reference's own fp32 run on the identical draws
            torch.set_default_dtype(torch.float32)
            replay[:] = [d.float() for d in recorded]
            o32 = make_obj(cls, model32, S, N, C, u0.float(), v0.float(), alpha0, T)
            o32.nested_step(xb.float(), yb.float())
            assert not replay
            for key, t in (("u_grad", o32.u), ("v_grad", o32.v)) + (
                    (("alpha_grad", o32.alpha),) if alpha0 is not None else ()):
                g = grad_np(t)
                if g is not None:
                    res[key + "_fp32"] = g.astype(np.float64)
            torch.set_default_dtype(torch.float64)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), config=np.array(json.dumps(cfg)),
                            **arrays, **res)
        print(f"wrote {name}: out={out:.6f} calls={len(sizes)} keys={sorted(res)}")

    def fn_deep(S):
        m = make_fcnet(5, 7, 3, n_layers=2, mc_samples=S, init_sd=0.05)
        perturb(m, 0.4, -3.0, -1.0, 0.0)
        return m

    def fn2_tiny(S):
        m = make_fc2net(8, 6, 3, mc_samples=S, init_sd=1e-2)
        perturb(m, 0.3, -3.5, -2.5, 0.002)
        return m

    def logreg(S):
        m = nn.Sequential(VILinear(2, 2, init_sd=0.1, mc_samples=S))
        perturb(m, 0.5, -3.0, 0.5, 0.0)
        return m

    # PSVIAV: u, v and alpha learned
    run("v01_av_nested_fn", "PSVIAV", "nested", "mf", fn_deep(6), M=13, Nx=9, D=5, C=3, S=6,
        N=500, T=4, seed=41, alpha0=0.3)
    run("v02_av_hyper_fn2", "PSVIAV", "hyper", "mvn", fn2_tiny(16), M=10, Nx=12, D=8, C=3,
        S=16, N=800, T=3, K=4, seed=42, alpha0=-0.2)
    # PSVIFixedU: u frozen
    run("v03_fixedu_nested_fn2", "PSVIFixedU", "nested", "mvn", fn2_tiny(16), M=10, Nx=12, D=8,
        C=3, S=16, N=800, T=3, seed=43)
    run("v04_fixedu_hyper_fn", "PSVIFixedU", "hyper", "mf", fn_deep(6), M=13, Nx=9, D=5, C=3,
        S=6, N=500, T=3, K=3, seed=44)
    # PSVIAFixedU: u frozen, v and alpha learned
    run("v05_afixedu_nested_fn", "PSVIAFixedU", "nested", "mf", fn_deep(6), M=13, Nx=9, D=5,
        C=3, S=6, N=500, T=4, seed=45, alpha0=0.1)
    run("v06_afixedu_hyper_fn2", "PSVIAFixedU", "hyper", "mvn", fn2_tiny(16), M=10, Nx=12, D=8,
        C=3, S=16, N=800, T=3, K=4, seed=46, alpha0=0.25)
    # PSVI_Ablated: mean data NLL minus mean sampled KL over the data batch
    run("v07_ablated_elbo_fn", "PSVI_Ablated", "psvi_elbo", "mf", fn_deep(6), M=13, Nx=9, D=5,
        C=3, S=6, N=500, T=0, seed=47)
    run("v08_ablated_nested_fn", "PSVI_Ablated", "nested", "mf", fn_deep(6), M=13, Nx=9, D=5,
        C=3, S=6, N=500, T=4, seed=48)
    run("v09_ablated_hyper_logreg", "PSVI_Ablated", "hyper", "mf", logreg(4), M=10, Nx=16, D=2,
        C=2, S=4, N=800, T=3, K=3, seed=49)
    run("v10_ablated_elbo_fn2", "PSVI_Ablated", "psvi_elbo", "mvn", fn2_tiny(4), M=10, Nx=12,
        D=8, C=3, S=4, N=800, T=0, seed=50)
    # PSVI_No_IW: single-sample training (the (M, M) broadcast inner objective)
    run("v11_noiw_nested_logreg", "PSVI_No_IW", "nested", "mf", logreg(1), M=10, Nx=16, D=2,
        C=2, S=1, N=800, T=4, seed=51)
    run("v12_noiw_hyper_fn", "PSVI_No_IW", "hyper", "mf", fn_deep(1), M=13, Nx=9, D=5, C=3,
        S=1, N=500, T=3, K=3, seed=52)
    run("v13_noiw_nested_fn", "PSVI_No_IW", "nested", "mf", fn_deep(1), M=13, Nx=9, D=5, C=3,
        S=1, N=500, T=3, seed=53)
    # LeNet (C5's architecture, the reference's psvi_alpha_fixed_u run): hyper_step
    m = make_lenet(mc_samples=2, init_sd=0.05)
    perturb(m, 0.1, -4.0, -2.0, 0.0)
    run("v14_afixedu_hyper_lenet", "PSVIAFixedU", "hyper", "lenet", m, M=4, Nx=6, D=784, C=10,
        S=2, N=60000, T=2, K=3, seed=54, alpha0=0.0, shape=(1, 28, 28))


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
