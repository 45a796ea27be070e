#!/usr/bin/env python3
"""Golden vectors for soft labels (learn_z) and the truncated nested step.

Runs ONLY in the development container (the reference is mounted read-only at
/root/reference); like tools/gen_golden_variants.py the parent re-launches this
script in a child interpreter whose sys.path holds the reference and not this
repo.  In float64 with every Monte-Carlo draw rounded to fp32 (draws recorded
in call order), the child runs the reference's own methods:

  * learn_z (psvi_classes.py:450-505, 541-600, 869-870, 1587-1620,
    1852-1884): z = one-hot label logits with requires_grad, the inner
    objective's KLDivLoss against softmax(z, 0), psvi_elbo's against
    softmax(cat(z, nc onehot(y)), 0), optim_z stepped --
    w01 PSVILearnV.nested_step (mean-field fn), w02 PSVIAFixedU.nested_step
    (LeNet, the reference's psvi_alpha_fixed_u learn_z run), w04 psvi_elbo
    (full-covariance fn2) and w05 inner_elbo (mean-field) with their
    backward into z, u, v and the parameters;
  * truncated nested_step (561-583): inner_it - K steps of
    torch.optim.Adam(lr=1e-4) whose backward accumulates (no zero_grad in
    the loop) into the network's, u's and v's gradients, then K unrolled
    steps -- w03 (mean-field fn).

Usage:  python tools/gen_golden_softlabels.py
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

    gen = torch.Generator().manual_seed(777)

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

    LR = dict(lr0net=1e-3, lr0u=1e-3, lr0v=1e-2, lr0alpha=1e-2, lr0z=1e-2)

    def make_obj(cls, model, S, N, C, u0, v0, z0, alpha0, T, learn_z):
        obj = cls.__new__(cls)
        obj.model = model
        obj.u = u0.detach().clone().requires_grad_(True)
        obj.v = v0.detach().clone().requires_grad_(True)
        obj.N, obj.nc, obj.mc_samples = N, C, S
        obj.distr_fn = categorical_fn
        obj.learn_v, obj.parameterised, obj.learn_z = True, True, learn_z
        obj.inner_it, obj.register_elbos, obj.log_every = T, False, 10
        obj.scheduler_optim_net = None
        obj.f = torch.softmax
        if learn_z:
            obj.z = z0.detach().clone().requires_grad_(True)
            obj.optim_z = torch.optim.Adam([obj.z], LR["lr0z"])
        else:
            obj.z = z0.detach().clone()
            obj.optim_z = None
        obj.optim_net = torch.optim.Adam(list(model.parameters()), LR["lr0net"])
        obj.optim_u = torch.optim.Adam([obj.u], LR["lr0u"])
        obj.optim_v = torch.optim.Adam([obj.v], LR["lr0v"])
        if alpha0 is not None:
            obj.alpha = torch.tensor([alpha0]).requires_grad_(True)
            obj.f = lambda *x: torch.exp(obj.alpha) * torch.softmax(x[0], x[1])
            obj.optim_alpha = torch.optim.Adam([obj.alpha], LR["lr0alpha"])
        return obj

    def run(name, cls_name, trainer, family, model, M, Nx, D, C, S, N, T, seed, learn_z=True,
            alpha0=None, K=2, shape=None):
        cls = getattr(PC, cls_name)
        torch.manual_seed(seed)
        model32 = copy.deepcopy(model).float()
        u0 = torch.randn(M, *(shape or (D,)), generator=gen).float().double()
        v0 = (0.2 * torch.randn(M, generator=gen)).float().double()
        zc = torch.tensor([i % C for i in range(M)])
        if learn_z:   # one-hot logits, moved off the one-hot point so softmax(z, 0) is generic
            z0 = (torch.nn.functional.one_hot(zc, C).double()
                  + 0.3 * torch.randn(M, C, generator=gen)).float().double()
        else:
            z0 = zc.double()
        xb = torch.randn(Nx, *(shape or (D,)), generator=gen).float().double()
        yb = torch.randint(0, C, (Nx,), generator=gen).double()
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        obj = make_obj(cls, model, S, N, C, u0, v0, z0, alpha0, T, learn_z)
        cfg = dict(family=family, layers=layer_sizes(model), S=S, M=M, N=N, Nx=Nx, T=T, K=K,
                   prior_sd=1.0, cls=cls_name, trainer=trainer, seed=seed, alpha0=alpha0,
                   learn_z=learn_z, C=C, **LR)
        arrays = dict(params0=p0.numpy().astype(np.float32), u0=u0.numpy().astype(np.float32),
                      v0=v0.numpy().astype(np.float32), z0=z0.numpy().astype(np.float32),
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

        def call(o, x, y):
            if trainer == "psvi_elbo":
                loss = o.psvi_elbo(x, y, model=o.model)
                loss.backward()
                return float(loss.detach())
            if trainer == "inner_elbo":
                loss = o.inner_elbo(model=o.model)
                loss.backward()
                return float(loss.detach())
            if trainer == "truncated":
                return float(o.nested_step(x, y, truncated=True, K=K).detach())
            return float(o.nested_step(x, y).detach())

        out = call(obj, xb, yb)
        recorded = [d.clone() for d in draws]
        cuts = np.cumsum([0] + [c for _, c in sizes])
        eps = [torch.cat(recorded[cuts[i]:cuts[i + 1]]).numpy().astype(np.float32)
               for i in range(len(sizes))]
        cfg["calls"] = [k for k, _ in sizes]
        res = dict(out=np.array(out), u=obj.u.detach().numpy(), v=obj.v.detach().numpy(),
                   z=obj.z.detach().numpy(),
                   params=parameters_to_vector(model.parameters()).detach().numpy())
        tracked = [("u_grad", obj.u), ("v_grad", obj.v)]
        if learn_z:
            tracked.append(("z_grad", obj.z))
        if alpha0 is not None:
            tracked.append(("alpha_grad", obj.alpha))
            res["alpha"] = obj.alpha.detach().numpy()
        for key, t in tracked:
            if t.grad is not None:
                res[key] = t.grad.detach().numpy()
        if trainer in ("psvi_elbo", "inner_elbo"):
            res["grad_params"] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).numpy()
        inner = [e for k, e in zip(cfg["calls"], eps) if k == "inner"]
        outer = [e for k, e in zip(cfg["calls"], eps) if k == "outer"]
        if inner:
            res["eps_inner"] = np.stack(inner)
        if outer:
            res["eps_outer"] = np.stack(outer)
        if trainer in ("nested", "truncated"):
            # the reference's own fp32 run on the identical draws
            torch.set_default_dtype(torch.float32)
            replay[:] = [d.float() for d in recorded]
            o32 = make_obj(cls, model32, S, N, C, u0.float(), v0.float(), z0.float(), alpha0, T,
                           learn_z)
            call(o32, xb.float(), yb.float())
            assert not replay
            for key, t in [("u_grad", o32.u), ("v_grad", o32.v)] + (
                    [("z_grad", o32.z)] if learn_z else []) + (
                    [("alpha_grad", o32.alpha)] if alpha0 is not None else []):
                if t.grad is not None:
                    res[key + "_fp32"] = t.grad.detach().numpy().astype(np.float64)
            torch.set_default_dtype(torch.float64)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), config=np.array(json.dumps(cfg)),
                            **arrays, **res)
        print(f"wrote {name}: out={out:.6f} calls={cfg['calls']} keys={sorted(res)}")

    def fn_deep(S):
        m = make_fcnet(5, 7, 3, n_layers=2, mc_samples=S, init_sd=0.05)
        perturb(m, 0.4, -3.0, -1.0, 0.0)
        return m

    def fn2_tiny(S):
        m = make_fc2net(8, 6, 3, mc_samples=S, init_sd=1e-2)
        perturb(m, 0.3, -3.5, -2.5, 0.002)
        return m

    run("w01_learnz_nested_fn", "PSVILearnV", "nested", "mf", fn_deep(6), M=12, Nx=9, D=5, C=3,
        S=6, N=500, T=3, seed=61)
    m = make_lenet(mc_samples=2, init_sd=0.05)
    perturb(m, 0.1, -4.0, -2.0, 0.0)
    run("w02_learnz_afixedu_nested_lenet", "PSVIAFixedU", "nested", "lenet", m, M=4, Nx=6, D=784,
        C=10, S=2, N=60000, T=2, seed=62, alpha0=0.0, shape=(1, 28, 28))
    run("w03_truncated_nested_fn", "PSVILearnV", "truncated", "mf", fn_deep(6), M=13, Nx=9, D=5,
        C=3, S=6, N=500, T=5, K=2, seed=63, learn_z=False)
    run("w04_learnz_psvi_elbo_fn2", "PSVILearnV", "psvi_elbo", "mvn", fn2_tiny(4), M=10, Nx=12,
        D=8, C=3, S=4, N=800, T=0, seed=64)
    run("w05_learnz_inner_elbo_fn", "PSVILearnV", "inner_elbo", "mf", fn_deep(6), M=12, Nx=1,
        D=5, C=3, S=6, N=500, T=0, seed=65)


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
