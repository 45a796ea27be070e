#!/usr/bin/env python3
"""Golden-vector generator for the coreset-ELBO inner loop.

Runs ONLY in the development container, where the reference tree is mounted
read-only at /root/reference.  The parent process re-launches this script in a
child interpreter whose sys.path holds the reference (and NOT this repo: both
packages are called ``psvi``).  The child drives the reference's own hot path

  * ``PSVI.inner_elbo``            psvi/inference/psvi_classes.py:488-511
  * ``innerloop_ctx`` + ``DifferentiableAdam.step``
                                   psvi/robust_higher/__init__.py:27-95,
                                   psvi/robust_higher/optim.py:152-257, 299-367
  * hypergrad ``DifferentiableAdam`` / ``adam_step`` (trainer ``hyper``)
                                   psvi/hypergrad/diff_optimizers.py:107-213

and records every Monte-Carlo draw by wrapping torch's ``_standard_normal``
inside ``torch.distributions.normal`` / ``multivariate_normal`` (the only
entropy source on the path: Normal.rsample / MultivariateNormal.rsample).
Outputs are small ``.npz`` fixtures under tests/golden/ (data only: inputs,
noise, expected ELBOs, gradients and Adam trajectories).

Usage:  python tools/gen_golden.py            (writes tests/golden/*.npz)
"""
import json
import os
import subprocess
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _install_stubs():
    """Modules imported at psvi.inference import time but never on the hot path
    (datasets / selection code only: experiments_utils.py:14,23, utils.py:28)."""
    import types

    for name in ["arff", "faiss", "torchvision", "torchvision.transforms",
                 "torchvision.datasets"]:
        mod = types.ModuleType(name)
        sys.modules[name] = mod
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torchvision"].datasets = sys.modules["torchvision.datasets"]


class _Recorder:
    """Wraps torch.distributions.utils._standard_normal as seen by Normal and
    MultivariateNormal; every draw is appended (in draw order) while active."""

    def __init__(self):
        import torch.distributions.multivariate_normal as mvn_mod
        import torch.distributions.normal as normal_mod

        self.mods = [normal_mod, mvn_mod]
        self.orig = [m._standard_normal for m in self.mods]
        self.active = False
        self.draws = []

        def wrap(orig):
            def f(shape, dtype, device):
                out = orig(shape, dtype=dtype, device=device)
                if self.active:
                    self.draws.append(out.detach().clone().reshape(-1))
                return out
            return f

        for m, o in zip(self.mods, self.orig):
            m._standard_normal = wrap(o)

    def start(self):
        self.draws = []
        self.active = True

    def stop(self):
        self.active = False
        import torch
        return torch.cat(self.draws) if self.draws else torch.zeros(0)


def _child():
    _install_stubs()
    import numpy as np
    import torch
    import torch.nn as nn
    from torch.nn.utils import parameters_to_vector

    from psvi.hypergrad import diff_optimizers as hgopt
    from psvi.inference.psvi_classes import PSVIAV, PSVILearnV
    from psvi.models.neural_net import (VILinear, VILinearMultivariateNormal,
                                        categorical_fn, make_fc2net, make_fcnet)
    from psvi.robust_higher import innerloop_ctx
    from psvi.robust_higher.patch import monkeypatch

    torch.set_default_dtype(torch.float32)
    rec = _Recorder()

    def make_obj(cls, u, z, v, N, alpha=None):
        # Bypass PSVI.__init__ (it needs datasets/dataloaders); inner_elbo only
        # reads u, z, v, N, f, distr_fn, learn_z (psvi_classes.py:488-511).
        obj = cls.__new__(cls)
        obj.u, obj.z, obj.v, obj.N = u, z, v, N
        obj.distr_fn = categorical_fn
        obj.learn_z = False
        if cls is PSVIAV:
            obj.alpha = torch.tensor([alpha])
            obj.f = lambda *x: torch.exp(obj.alpha) * torch.softmax(x[0], x[1])
        elif cls is PSVILearnV:
            obj.f = torch.softmax
        else:
            obj.f = lambda *x: x[0]
        return obj

    def weights(obj):
        return (obj.N * obj.f(obj.v, 0)).detach()

    def perturb(model, gen, mu_scale, rho_lo, rho_hi, corr_scale):
        with torch.no_grad():
            for name, p in model.named_parameters():
                leaf = name.split(".")[-1]
                if leaf in ("weight", "bias", "mean"):
                    p.copy_(mu_scale * torch.randn(p.shape, generator=gen))
                elif leaf in ("_weight_sd", "_bias_sd", "_sd"):
                    p.copy_(rho_lo + (rho_hi - rho_lo) * torch.rand(p.shape, generator=gen))
                elif leaf == "_corr":
                    p.copy_(corr_scale * torch.randn(p.shape, generator=gen))

    def layer_sizes(model):
        out = []
        for m in model.modules():
            if isinstance(m, (VILinear, VILinearMultivariateNormal)):
                out.append([m.in_features, m.out_features])
        return out

    def run_nested(name, family, model, cls, u, z, v, N, lr, T, seed, meta, alpha=None):
        """nested trainer inner loop: psvi_classes.py:549-555 (higher Adam)."""
        obj = make_obj(cls, u, z, v, N, alpha)
        p0 = parameters_to_vector(model.parameters()).detach().clone()
        optim_net = torch.optim.Adam(list(model.parameters()), lr)
        eps, elbos, params = [], [], []
        grad0 = None
        with innerloop_ctx(model, optim_net) as (fmodel, diffopt):
            for t in range(T):
                torch.manual_seed(seed + t)
                rec.start()
                loss = obj.inner_elbo(model=fmodel)
                eps.append(rec.stop().numpy())
                elbos.append(float(loss.detach()))
                if t == 0:
                    g = torch.autograd.grad(loss, list(fmodel.parameters()),
                                            retain_graph=True)
                    grad0 = torch.cat([x.reshape(-1) for x in g]).detach().numpy()
                diffopt.step(loss)
                params.append(parameters_to_vector(fmodel.parameters()).detach().numpy())
            st = diffopt.state[0]
            m_vec = np.concatenate([st[i]["exp_avg"].detach().reshape(-1).numpy()
                                    for i in range(len(st))])
            v_vec = np.concatenate([st[i]["exp_avg_sq"].detach().reshape(-1).numpy()
                                    for i in range(len(st))])
        save(name, family, model, obj, u, z, p0, eps, elbos, grad0, params, m_vec,
             v_vec, lr, T, seed, "higher", meta)

    def run_hyper(name, family, model, cls, u, z, v, N, lr, T, seed, meta, alpha=None):
        """hyper trainer inner loop: psvi_classes.py:615-666 (hypergrad adam_step,
        first order, step_cnt persists across the T steps)."""
        obj = make_obj(cls, u, z, v, N, alpha)
        fmodel = monkeypatch(model, copy_initial_weights=True)
        p0 = parameters_to_vector(model.parameters()).detach().clone()

        def inner_loss(p, hp):
            return obj.inner_elbo(model=fmodel, params=p, hyperopt=True)

        opt = hgopt.DifferentiableAdam(inner_loss, step_size=lr)
        params = [p.detach().clone().requires_grad_(True) for p in fmodel.parameters()]
        hist = [opt.get_opt_params(params)]
        eps, elbos, out_params = [], [], []
        grad0 = None
        n = len(params)
        for t in range(T):
            torch.manual_seed(seed + t)
            if t == 0:
                rec.start()
                l0 = inner_loss(hist[-1][:n], [u])
                rec.stop()
                g = torch.autograd.grad(l0, hist[-1][:n])
                grad0 = torch.cat([x.reshape(-1) for x in g]).detach().numpy()
                torch.manual_seed(seed + t)
            rec.start()
            hist.append(opt(hist[-1], [u], create_graph=False))
            eps.append(rec.stop().numpy())
            elbos.append(float(opt.curr_loss.detach()))
            out_params.append(torch.cat([x.detach().reshape(-1) for x in hist[-1][:n]]).numpy())
        m_vec = torch.cat([x.detach().reshape(-1) for x in hist[-1][n:2 * n]]).numpy()
        v_vec = torch.cat([x.detach().reshape(-1) for x in hist[-1][2 * n:]]).numpy()
        save(name, family, model, obj, u, z, p0, eps, elbos, grad0, out_params, m_vec,
             v_vec, lr, T, seed, "hypergrad", meta)

    def save(name, family, model, obj, u, z, p0, eps, elbos, grad0, params, m_vec,
             v_vec, lr, T, seed, adam, meta):
        sizes = layer_sizes(model)
        cfg = dict(family=family, layers=sizes, S=meta["S"], M=int(u.shape[0]),
                   N=int(obj.N), lr=lr, T=T, seed=seed, adam=adam,
                   prior_sd=1.0, f=meta.get("f", "softmax"),
                   alpha=meta.get("alpha"), note=meta.get("note", ""))
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            config=np.array(json.dumps(cfg)),
            u=u.detach().numpy().astype(np.float32),
            z=z.detach().numpy().astype(np.float32),
            v=obj.v.detach().numpy().astype(np.float32),
            w=weights(obj).numpy().astype(np.float32),
            params0=p0.numpy().astype(np.float32),
            eps=np.stack(eps).astype(np.float32),
            elbo=np.array(elbos, dtype=np.float64),
            grad0=grad0.astype(np.float32),
            params=np.stack(params).astype(np.float32),
            adam_m=m_vec.astype(np.float32),
            adam_v=v_vec.astype(np.float32),
        )
        print(f"wrote {name}: P={p0.numel()} elbo={elbos}")

    # -- data -------------------------------------------------------------
    from sklearn.datasets import make_moons

    X, Y = make_moons(1000, noise=0.1, random_state=42)
    X = torch.tensor(X[:800], dtype=torch.float32)
    Y = torch.tensor(Y[:800], dtype=torch.float32)

    def per_class(X, Y, nc, M):
        ppc = [M // nc] * nc
        ppc[-1] = M - sum(ppc[:-1])
        us, zs = [], []
        for c in range(nc):
            idx = (Y == c).nonzero().reshape(-1)[: ppc[c]]
            us.append(X[idx])
            zs.append(torch.full((ppc[c],), float(c)))
        return torch.cat(us), torch.cat(zs)

    gen = torch.Generator().manual_seed(1234)

    # G1: C1 exact -- logistic_regression (psvi_classes.py:694-699), halfmoon, M=10, S=4
    torch.manual_seed(0)
    u, z = per_class(X, Y, 2, 10)
    model = nn.Sequential(VILinear(2, 2, init_sd=1e-6, mc_samples=4))
    run_nested("g1_logreg_c1", "mf", model, PSVILearnV, u, z, torch.zeros(10), 800,
               1e-3, 3, 10, dict(S=4, note="C1 exact, init_sd=1e-6"))

    # G1r: logreg with a perturbed posterior (exercises the sigma*eps path)
    torch.manual_seed(0)
    model = nn.Sequential(VILinear(2, 2, init_sd=0.1, mc_samples=4))
    perturb(model, gen, 0.5, -3.0, 0.5, 0.0)
    run_nested("g1r_logreg_rand", "mf", model, PSVILearnV, u, z, torch.zeros(10), 800,
               1e-3, 3, 20, dict(S=4, note="logreg perturbed"))

    # G2: C2 exact -- fn 1x100, four_blobs-shaped (D=2, C=4), M=50, S=32
    torch.manual_seed(0)
    u2 = torch.randn(50, 2, generator=gen) * 2.0
    z2 = torch.tensor([float(i // 13) if i < 39 else 3.0 for i in range(50)])
    model = make_fcnet(2, 100, 4, n_layers=1, mc_samples=32, init_sd=1e-6)
    run_nested("g2_fn_c2", "mf", model, PSVILearnV, u2, z2, torch.zeros(50), 800,
               1e-3, 3, 30, dict(S=32, note="C2 exact, init_sd=1e-6"))

    # G2r: C2 shape, perturbed posterior, PSVIAV weights f = exp(alpha) softmax(v)
    torch.manual_seed(0)
    model = make_fcnet(2, 100, 4, n_layers=1, mc_samples=32, init_sd=0.1)
    perturb(model, gen, 0.3, -4.0, -1.0, 0.0)
    v2 = 0.3 * torch.randn(50, generator=gen)
    run_nested("g2r_fn_c2_rand_av", "mf", model, PSVIAV, u2, z2, v2, 800, 1e-3, 3, 40,
               dict(S=32, f="exp_alpha_softmax", alpha=0.25, note="C2 shape perturbed, PSVIAV"),
               alpha=0.25)

    # G2h: same model family under the hyper trainer's first-order hypergrad Adam
    torch.manual_seed(0)
    model = make_fcnet(2, 100, 4, n_layers=1, mc_samples=32, init_sd=0.1)
    perturb(model, gen, 0.3, -4.0, -1.0, 0.0)
    run_hyper("g2h_fn_c2_hyper", "mf", model, PSVILearnV, u2, z2, torch.zeros(50), 800,
              1e-3, 3, 50, dict(S=32, note="hypergrad adam_step"))

    # G2d: deeper mean-field MLP (2 hidden layers, odd sizes), M not divisible by C
    torch.manual_seed(0)
    u3 = torch.randn(13, 5, generator=gen)
    z3 = torch.tensor([float(i % 3) for i in range(13)])
    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05)
    perturb(model, gen, 0.4, -3.0, -1.0, 0.0)
    run_nested("g2d_fn_deep", "mf", model, PSVILearnV, u3, z3, torch.zeros(13), 500,
               1e-3, 3, 60, dict(S=6, note="2 hidden layers"))

    # G3: fn2-tiny (make_fc2net, 2 hidden layers of full-cov VI), D=8 H=6 C=3, M=10, S=16
    torch.manual_seed(0)
    u4 = torch.randn(10, 8, generator=gen)
    z4 = torch.tensor([float(i % 3) for i in range(10)])
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-6)
    run_nested("g3_fn2_tiny", "mvn", model, PSVILearnV, u4, z4, torch.zeros(10), 800,
               1e-3, 3, 70, dict(S=16, note="fn2 tiny, reference init"))

    torch.manual_seed(0)
    model = make_fc2net(8, 6, 3, mc_samples=16, init_sd=1e-2)
    perturb(model, gen, 0.3, -4.0, -2.0, 0.02)
    run_nested("g3r_fn2_tiny_rand", "mvn", model, PSVILearnV, u4, z4, torch.zeros(10), 800,
               1e-3, 3, 80, dict(S=16, note="fn2 tiny perturbed (nonzero _corr)"))

    # G4: fn2-mid D=16 H=8 C=2, M=20, S=32
    torch.manual_seed(0)
    u5 = torch.randn(20, 16, generator=gen)
    z5 = torch.tensor([float(i % 2) for i in range(20)])
    model = make_fc2net(16, 8, 2, mc_samples=32, init_sd=1e-6)
    run_nested("g4_fn2_mid", "mvn", model, PSVILearnV, u5, z5, torch.zeros(20), 800,
               1e-3, 3, 90, dict(S=32, note="fn2 mid, reference init"))

    torch.manual_seed(0)
    model = make_fc2net(16, 8, 2, mc_samples=32, init_sd=1e-2)
    perturb(model, gen, 0.2, -5.0, -2.5, 0.01)
    v5 = 0.2 * torch.randn(20, generator=gen)
    run_hyper("g4h_fn2_mid_hyper", "mvn", model, PSVIAV, u5, z5, v5, 800, 1e-3, 3, 100,
              dict(S=32, f="exp_alpha_softmax", alpha=-0.3, note="fn2 hyper, PSVIAV"),
              alpha=-0.3)

    # G5: logistic_regression_fullcov (single VILinearMultivariateNormal layer)
    torch.manual_seed(0)
    model = nn.Sequential(VILinearMultivariateNormal(2, 2, init_sd=0.1, mc_samples=4))
    perturb(model, gen, 0.5, -3.0, -1.0, 0.05)
    run_nested("g5_logreg_fullcov", "mvn", model, PSVILearnV, u, z, torch.zeros(10), 800,
               1e-3, 3, 110, dict(S=4, note="logistic_regression_fullcov"))

    # L1/L2: lenet (make_lenet, neural_net.py:334-359): VIConv2d + BatchMaxPool2d +
    # VILinear, the last layer one shared sample (its default mc_samples=1,
    # init_sd=0.01); MNIST-shaped u.  cfg["layers"] lists the VILinear layers only.
    from psvi.models.neural_net import make_lenet

    torch.manual_seed(0)
    u6 = torch.randn(4, 1, 28, 28, generator=gen)
    z6 = torch.tensor([1.0, 7.0, 3.0, 9.0])
    model = make_lenet(mc_samples=3, init_sd=0.05)
    perturb(model, gen, 0.15, -4.0, -2.0, 0.0)
    run_nested("l1_lenet_tiny", "lenet", model, PSVILearnV, u6, z6, torch.zeros(4), 60000,
               1e-3, 2, 120, dict(S=3, note="lenet (C5 architecture), M=4, S=3"))

    torch.manual_seed(0)
    u7 = torch.randn(6, 1, 28, 28, generator=gen)
    z7 = torch.tensor([0.0, 2.0, 4.0, 6.0, 8.0, 5.0])
    model = make_lenet(mc_samples=2, init_sd=0.05)
    perturb(model, gen, 0.2, -3.5, -2.0, 0.0)
    v7 = 0.3 * torch.randn(6, generator=gen)
    run_hyper("l2_lenet_hyper", "lenet", model, PSVIAV, u7, z7, v7, 60000, 1e-3, 2, 130,
              dict(S=2, f="exp_alpha_softmax", alpha=0.1, note="lenet hyper, PSVIAV"),
              alpha=0.1)


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
