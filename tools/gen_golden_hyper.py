#!/usr/bin/env python3
"""Golden vectors for the second-order path of the ``hyper`` trainer.

Runs ONLY in the development container (the reference is mounted read-only at
/root/reference); the parent re-launches this script in a child interpreter
whose sys.path holds the reference and not this repo (both are ``psvi``).
In float64 with every Monte-Carlo draw rounded to fp32 (the HIP path's eps),
the child records

  * h*.npz -- the Hessian-vector product of the reference's inner objective
    and its mixed products, by double backward exactly as hypergrad takes them
    (psvi/hypergrad/hypergradients.py:199-244 torch_grad / jvp through
    GradientDescent's fp_map, diff_optimizers.py:51-60, 157-159):
        g = d inner_elbo / d params (create_graph);  s = g . vec
        ds / d params (= H vec), ds / d u, ds / d v
    with inner_elbo(model=fmodel, params=p, hyperopt=True) on a
    monkeypatch'ed model (psvi_classes.py:602-650);
  * n*.npz -- one full PSVI.nested_step (psvi_classes.py:541-600): T higher-Adam
    steps in innerloop_ctx, psvi_elbo.backward() through the unroll, the u / v
    Adam steps, with every draw;
  * y*.npz -- one full PSVI.hyper_step (psvi_classes.py:602-687): the T-step
    first-order inner loop (hypergrad DifferentiableAdam), CG_normaleq with K
    iterations, the u / v Adam steps, the returned outer loss -- and every
    draw in call order, so the HIP path can replay it.

Usage:  python tools/gen_golden_hyper.py
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

    from psvi.inference.psvi_classes import PSVILearnV
    from psvi.models.neural_net import (VILinear, VILinearMultivariateNormal,
                                        categorical_fn, make_fc2net, make_fcnet)
    from psvi.robust_higher.patch import monkeypatch

    import copy

    torch.set_default_dtype(torch.float64)
    draws = []
    replay = []  # fp32 re-runs: the recorded draws, in order

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

    def make_obj(model, M, D, C, S, N, uv=None, shape=None):
        if uv is None:
            u = torch.randn(M, *(shape or (D,)), generator=gen).float().double().requires_grad_(True)
            v = (0.2 * torch.randn(M, generator=gen)).float().double().requires_grad_(True)
        else:
            u, v = (t.detach().clone().requires_grad_(True) for t in uv)
        z = torch.tensor([float(i % C) for i in range(M)])
        obj = PSVILearnV.__new__(PSVILearnV)
        obj.model = model
        obj.u, obj.z, obj.v, obj.N = u, z, v, N
        obj.distr_fn = categorical_fn
        obj.learn_z, obj.learn_v, obj.parameterised = False, True, True
        obj.mc_samples = S
        obj.nc = C
        obj.f = torch.softmax
        return obj

    def cfg_of(family, model, S, M, N, **kw):
        c = dict(family=family, layers=layer_sizes(model), S=S, M=M, N=N, prior_sd=1.0,
                 f="softmax")
        c.update(kw)
        return c

    def run_hvp(name, family, model, M, D, C, S, N, seed, note="", shape=None):
        torch.manual_seed(seed)
        obj = make_obj(model, M, D, C, S, N, shape=shape)
        fmodel = monkeypatch(model, copy_initial_weights=True)
        params = [p.detach().clone().requires_grad_(True) for p in fmodel.parameters()]
        p0 = torch.cat([p.detach().reshape(-1) for p in params])
        vec = torch.randn(p0.numel(), generator=gen).float().double()
        draws.clear()
        loss = obj.inner_elbo(model=fmodel, params=params, hyperopt=True)
        eps = torch.cat(draws).numpy()
        g = torch.autograd.grad(loss, params, create_graph=True)
        gvec = torch.cat([x.reshape(-1) for x in g])
        s = (gvec * vec).sum()
        out = torch.autograd.grad(s, params + [obj.u, obj.v])
        hv = torch.cat([x.reshape(-1) for x in out[:len(params)]])
        w = (obj.N * obj.f(obj.v, 0)).detach()
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            config=np.array(json.dumps(cfg_of(family, model, S, M, N, seed=seed, note=note))),
            params0=p0.numpy().astype(np.float32), u=obj.u.detach().numpy().astype(np.float32),
            z=obj.z.numpy().astype(np.float32), v=obj.v.detach().numpy().astype(np.float32),
            w=w.numpy(), eps=eps.astype(np.float32), vec=vec.numpy().astype(np.float32),
            elbo=np.array(float(loss.detach())), grad=gvec.detach().numpy(), hv=hv.numpy(),
            d_u=out[-2].numpy(), d_v=out[-1].numpy())
        print(f"wrote {name}: P={p0.numel()} elbo={float(loss):.6f}")

    def run_hyper_step(name, family, model, M, Nx, D, C, S, N, seed, T, K, note="",
                       approx="CG_normaleq", shape=None):
        torch.manual_seed(seed)
        obj = make_obj(model, M, D, C, S, N, shape=shape)
        obj.inner_it = T
        lr0net, lr0u, lr0v = 1e-3, 1e-3, 1e-2
        obj.optim_net = torch.optim.Adam(list(model.parameters()), lr0net)
        obj.optim_u = torch.optim.Adam([obj.u], lr0u)
        obj.optim_v = torch.optim.Adam([obj.v], lr0v)
        xb = torch.randn(Nx, *(shape or (D,)), generator=gen).float().double()
        yb = torch.randint(0, C, (Nx,), generator=gen).double()
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        u0, v0 = obj.u.detach().clone(), obj.v.detach().clone()
        draws.clear()
        sizes = []
        n_prev = [0]

        # draw counts per call (to split the recorded stream)
        orig_inner, orig_outer = obj.inner_elbo, obj.psvi_elbo

        def inner(*a, **k):
            r = orig_inner(*a, **k)
            sizes.append(("inner", len(draws) - n_prev[0]))
            n_prev[0] = len(draws)
            return r

        def outer(*a, **k):
            r = orig_outer(*a, **k)
            sizes.append(("outer", len(draws) - n_prev[0]))
            n_prev[0] = len(draws)
            return r

        obj.inner_elbo, obj.psvi_elbo = inner, outer
        ll = obj.hyper_step(xb, yb, K=K, hypergrad_approx=approx)
        calls = [k for k, _ in sizes]
        eps = [torch.cat(draws[sum(c for _, c in sizes[:i]):sum(c for _, c in sizes[:i + 1])])
               .numpy().astype(np.float32) for i in range(len(sizes))]
        ne = {k: len(e) for k, e in zip(calls, eps)}
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            config=np.array(json.dumps(cfg_of(family, model, S, M, N, Nx=Nx, T=T, K=K,
                                              lr0net=lr0net, lr0u=lr0u, lr0v=lr0v,
                                              linsys_lr=1e-4, calls=calls, seed=seed,
                                              approx=approx, note=note))),
            params0=p0.numpy().astype(np.float32), u0=u0.numpy().astype(np.float32),
            v0=v0.numpy().astype(np.float32), z=obj.z.numpy().astype(np.float32),
            xb=xb.numpy().astype(np.float32), yb=yb.numpy().astype(np.float32),
            eps_inner=np.stack([e for k, e in zip(calls, eps) if k == "inner"]),
            eps_outer=np.stack([e for k, e in zip(calls, eps) if k == "outer"]),
            ll=np.array(float(ll)),
            u=obj.u.detach().numpy(), v=obj.v.detach().numpy(),
            u_grad=obj.u.grad.numpy(), v_grad=obj.v.grad.numpy(),
            params=parameters_to_vector(model.parameters()).detach().numpy())
        print(f"wrote {name}: calls={len(calls)} ll={float(ll):.6f} eps sizes={ne}")

    def run_nested_step(name, family, model, M, Nx, D, C, S, N, seed, T, note=""):
        """PSVI.nested_step (psvi_classes.py:541-600): T higher-Adam steps on
        inner_elbo in innerloop_ctx, psvi_elbo.backward() through the unroll,
        then the u / v Adam steps; fmodel's parameters copied into the model."""
        torch.manual_seed(seed)
        model32 = copy.deepcopy(model).float()
        obj = make_obj(model, M, D, C, S, N)
        obj.inner_it, obj.register_elbos, obj.log_every = T, False, 10
        obj.scheduler_optim_net = None
        lr0net, lr0u, lr0v = 1e-3, 1e-3, 1e-2
        obj.optim_net = torch.optim.Adam(list(model.parameters()), lr0net)
        obj.optim_u = torch.optim.Adam([obj.u], lr0u)
        obj.optim_v = torch.optim.Adam([obj.v], lr0v)
        xb = torch.randn(Nx, D, generator=gen).float().double()
        yb = torch.randint(0, C, (Nx,), generator=gen).double()
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        u0, v0 = obj.u.detach().clone(), obj.v.detach().clone()
        draws.clear()
        sizes, n_prev = [], [0]
        orig_inner, orig_outer = obj.inner_elbo, obj.psvi_elbo

        def inner(*a, **k):
            r = orig_inner(*a, **k)
            sizes.append(len(draws) - n_prev[0])
            n_prev[0] = len(draws)
            return r

        def outer(*a, **k):
            r = orig_outer(*a, **k)
            sizes.append(len(draws) - n_prev[0])
            n_prev[0] = len(draws)
            return r

        obj.inner_elbo, obj.psvi_elbo = inner, outer
        loss = obj.nested_step(xb, yb)
        recorded = [d.clone() for d in draws]
        # the reference's own fp32 run on the identical draws (its native dtype):
        # how far fp32 rounding alone moves the unrolled hypergradient
        torch.set_default_dtype(torch.float32)
        replay[:] = [d.float() for d in recorded]
        o32 = make_obj(model32, M, D, C, S, N, uv=(u0.float(), v0.float()))
        o32.inner_it, o32.register_elbos, o32.log_every = T, False, 10
        o32.scheduler_optim_net = None
        o32.optim_net = torch.optim.Adam(list(model32.parameters()), lr0net)
        o32.optim_u = torch.optim.Adam([o32.u], lr0u)
        o32.optim_v = torch.optim.Adam([o32.v], lr0v)
        o32.nested_step(xb.float(), yb.float())
        assert not replay
        u_grad32, v_grad32 = o32.u.grad.double().numpy(), o32.v.grad.double().numpy()
        torch.set_default_dtype(torch.float64)
        draws[:] = recorded
        cuts = np.cumsum([0] + sizes)
        eps = [torch.cat(draws[cuts[i]:cuts[i + 1]]).numpy().astype(np.float32)
               for i in range(len(sizes))]
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            config=np.array(json.dumps(cfg_of(family, model, S, M, N, Nx=Nx, T=T,
                                              lr0net=lr0net, lr0u=lr0u, lr0v=lr0v, seed=seed,
                                              note=note))),
            params0=p0.numpy().astype(np.float32), u0=u0.numpy().astype(np.float32),
            v0=v0.numpy().astype(np.float32), z=obj.z.numpy().astype(np.float32),
            xb=xb.numpy().astype(np.float32), yb=yb.numpy().astype(np.float32),
            eps_inner=np.stack(eps[:T]), eps_outer=eps[T][None],
            loss=np.array(float(loss.detach())),
            u=obj.u.detach().numpy(), v=obj.v.detach().numpy(),
            u_grad=obj.u.grad.numpy(), v_grad=obj.v.grad.numpy(),
            u_grad_fp32=u_grad32, v_grad_fp32=v_grad32,
            params=parameters_to_vector(model.parameters()).detach().numpy())
        e32 = np.linalg.norm(u_grad32 - obj.u.grad.numpy()) / np.linalg.norm(obj.u.grad.numpy())
        print(f"wrote {name}: calls={len(sizes)} loss={float(loss):.6f} "
              f"(reference fp32 u_grad l2rel vs fp64: {e32:.2e})")

    # HVP fixtures
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
    perturb(model, 0.3, -3.5, -2.5, 0.002)
    run_hvp("h1_fn2_tiny", "mvn", model, M=10, D=8, C=3, S=16, N=800, seed=11)

    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05)
    perturb(model, 0.4, -3.0, -1.0, 0.0)
    run_hvp("h2_fn_deep", "mf", model, M=13, D=5, C=3, S=6, N=500, seed=12)

    model = make_fcnet(2, 20, 4, n_layers=1, mc_samples=8, init_sd=0.1)
    perturb(model, 0.3, -4.0, -1.0, 0.0)
    run_hvp("h3_fn_shallow", "mf", model, M=12, D=2, C=4, S=8, N=800, seed=13)

    model = nn.Sequential(VILinearMultivariateNormal(2, 2, init_sd=0.1, mc_samples=4))
    perturb(model, 0.5, -3.0, -1.0, 0.02)
    run_hvp("h4_logreg_fullcov", "mvn", model, M=10, D=2, C=2, S=4, N=800, seed=14)

    # one whole hyper_step each
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
    perturb(model, 0.3, -3.5, -2.5, 0.002)
    run_hyper_step("y1_fn2_tiny", "mvn", model, M=10, Nx=12, D=8, C=3, S=16, N=800, seed=21,
                   T=3, K=4)

    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05)
    perturb(model, 0.4, -3.0, -1.0, 0.0)
    run_hyper_step("y2_fn_deep", "mf", model, M=13, Nx=9, D=5, C=3, S=6, N=500, seed=22,
                   T=3, K=4)

    # one whole nested_step each (the reference's default trainer)
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
    perturb(model, 0.3, -3.5, -2.5, 0.002)
    run_nested_step("n1_fn2_tiny", "mvn", model, M=10, Nx=12, D=8, C=3, S=16, N=800, seed=31,
                    T=4)

    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05)
    perturb(model, 0.4, -3.0, -1.0, 0.0)
    run_nested_step("n2_fn_deep", "mf", model, M=13, Nx=9, D=5, C=3, S=6, N=500, seed=32, T=4)

    model = nn.Sequential(VILinear(2, 2, init_sd=0.1, mc_samples=4))
    perturb(model, 0.5, -3.0, 0.5, 0.0)
    run_nested_step("n3_logreg", "mf", model, M=10, Nx=16, D=2, C=2, S=4, N=800, seed=33, T=5)

    # hypergrad_approx="fixed_point" (hypergradients.py:83-140, stochastic)
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
    perturb(model, 0.3, -3.5, -2.5, 0.002)
    run_hyper_step("y3_fn2_tiny_fp", "mvn", model, M=10, Nx=12, D=8, C=3, S=16, N=800,
                   seed=23, T=3, K=4, approx="fixed_point")

    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05)
    perturb(model, 0.4, -3.0, -1.0, 0.0)
    run_hyper_step("y4_fn_deep_fp", "mf", model, M=13, Nx=9, D=5, C=3, S=6, N=500, seed=24,
                   T=3, K=4, approx="fixed_point")

    # LeNet (make_lenet, C5's architecture): double backward through the conv
    # towers, and one whole hyper_step (C5's trainer) with CG_normaleq
    from psvi.models.neural_net import make_lenet

    model = make_lenet(mc_samples=3, init_sd=0.05)
    perturb(model, 0.15, -4.0, -2.0, 0.0)
    run_hvp("h5_lenet", "lenet", model, M=4, D=784, C=10, S=3, N=60000, seed=15,
            shape=(1, 28, 28))
    model = make_lenet(mc_samples=2, init_sd=0.05)
    perturb(model, 0.1, -4.0, -2.0, 0.0)
    run_hyper_step("y5_lenet", "lenet", model, M=4, Nx=6, D=784, C=10, S=2, N=60000,
                   seed=25, T=2, K=3, shape=(1, 28, 28))


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
