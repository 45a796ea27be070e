"""psvi.hypergrad on the GPU: the reference's PSVI.hyper_step body run
through this package's hypergrad API.

``_reference_hyper_step`` is the call sequence of the reference's
PSVI.hyper_step (psvi/inference/psvi_classes.py:602-687): a functional copy of
the network (``monkeypatch``), T steps of hypergrad's ``DifferentiableAdam``
(``create_graph=False``) on ``inner_elbo(model=fmodel, params=p,
hyperopt=True)``, then ``CG_normaleq`` (or ``fixed_point``, stochastic) with a
``GradientDescent`` fixed-point map of step linsys_lr, the u / v Adam steps, the
outer loss at the new hparams and the copy of the solution into the model --
with the reference's own draws replayed in call order.  It must reproduce the
reference's whole hyper_step (y* fixtures) and agree with this package's
PSVI.hyper_step."""
import pytest
import torch
import torch.nn as nn

from golden_util import fixture_names, l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu


def _reference_hyper_step(self, xbatch, ybatch, K=30, linsys_lr=1e-4,
                          hypergrad_approx="CG_normaleq"):
    from psvi.hypergrad import CG_normaleq, DifferentiableAdam, GradientDescent, fixed_point
    from psvi.robust_higher import monkeypatch

    T = self.inner_it
    inner_opt_kwargs = {"step_size": self.optim_net.param_groups[0]["lr"]}
    fmodel = monkeypatch(self.model, copy_initial_weights=True)
    self.optim_u.zero_grad()
    if self.learn_v:
        self.optim_v.zero_grad()

    def inner_loop(hparams, params, optim, n_steps, create_graph=False):
        hist = [optim.get_opt_params(params)]
        for _ in range(n_steps):
            hist.append(optim(hist[-1], hparams, create_graph=create_graph))
        return hist

    def inner_loss_function(p, hp, hyperopt=True):
        if self.learn_v:
            self.u, self.v = hp[0], hp[1]
        else:
            self.u = hp[0]
        return self.inner_elbo(model=fmodel, params=p, hyperopt=hyperopt)

    def outer_loss_function(p, hp):
        if self.learn_v:
            self.u, self.v = hp[0], hp[1]
        else:
            self.u = hp[0]
        return self.psvi_elbo(xbatch, ybatch, model=fmodel, params=p, hyperopt=True)

    inner_opt = DifferentiableAdam(inner_loss_function, **inner_opt_kwargs)
    params = [p.detach().clone().requires_grad_(True) for p in fmodel.parameters()]
    hp = [self.u] + [self.v] if self.learn_v else [self.u]
    hist = inner_loop(hp, params, inner_opt, T)
    last_param = hist[-1][:len(params)]
    linear_opt = GradientDescent(loss_f=inner_loss_function, step_size=linsys_lr)
    if hypergrad_approx == "fixed_point":
        fixed_point(last_param, hp, K=K, fp_map=linear_opt, outer_loss=outer_loss_function,
                    stochastic=True)
    else:
        CG_normaleq(last_param, hp, K=K, fp_map=linear_opt, outer_loss=outer_loss_function,
                    set_grad=True)
    self.optim_u.step()
    if self.learn_v:
        self.optim_v.step()
        if not self.parameterised:
            with torch.no_grad():
                torch.clamp_(self.v, min=0.0)
    ll = outer_loss_function(last_param, [self.u] + [self.v])
    nn.utils.vector_to_parameters(nn.utils.parameters_to_vector(last_param),
                                  self.model.parameters())
    return ll.item()


def _psvi(f):
    from psvi.inference import PSVILearnV
    from test_host_api import build_model

    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    u = torch.tensor(f["u0"], device="cuda").requires_grad_(True)
    ps = PSVILearnV(u=u, z=torch.tensor(f["z"], device="cuda"), N=cfg["N"], model=model,
                    mc_samples=cfg["S"], device_id=0, inner_it=cfg["T"])
    ps.device = torch.device("cuda")
    ps.register_elbos = False
    ps.v = torch.tensor(f["v0"], device="cuda").requires_grad_(True)
    ps.setup_optimizers(lr0net=cfg["lr0net"], lr0u=cfg["lr0u"], lr0v=cfg["lr0v"])
    return ps, model


def _draws(f):
    """The reference's draws in call order: T inner, the outer objective at
    the inner solution, the solver's inner draws, the final outer loss."""
    T = f["cfg"]["T"]
    ei = [torch.tensor(e, device="cuda") for e in f["eps_inner"]]
    eo = [torch.tensor(e, device="cuda") for e in f["eps_outer"]]
    return ei[:T] + [eo[0]] + ei[T:] + eo[1:]


@pytest.mark.parametrize("name", fixture_names("y"))
def test_reference_hyper_step_body_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    ps, model = _psvi(f)
    ps.replay_eps(_draws(f))
    xb, yb = torch.tensor(f["xb"], device="cuda"), torch.tensor(f["yb"], device="cuda")
    ll = _reference_hyper_step(ps, xb, yb, K=cfg["K"], linsys_lr=cfg["linsys_lr"],
                               hypergrad_approx=cfg.get("approx", "CG_normaleq"))
    assert ps._eps_feed is not None and next(ps._eps_feed, None) is None, "draws left over"
    p = nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy()
    assert l2rel(p, f["params"]) < 1e-5
    ug, vg = ps.u.grad.cpu().numpy(), ps.v.grad.cpu().numpy()
    print(f"{name}: u_grad l2rel {l2rel(ug, f['u_grad']):.2e}, v_grad {l2rel(vg, f['v_grad']):.2e}, "
          f"ll rel {rel(ll, f['ll']):.2e}")
    assert l2rel(ug, f["u_grad"]) < 1e-4
    assert l2rel(vg, f["v_grad"]) < 1e-4
    assert rel(ll, f["ll"]) < 1e-5


def test_reference_body_equals_package_hyper_step():
    """The reference's body on psvi.hypergrad and PSVI.hyper_step give the
    same hypergradients on the same draws."""
    f = load_fixture("y1_fn2_tiny")
    cfg = f["cfg"]
    xb, yb = torch.tensor(f["xb"], device="cuda"), torch.tensor(f["yb"], device="cuda")
    a, _ = _psvi(f)
    a.replay_eps(_draws(f))
    la = _reference_hyper_step(a, xb, yb, K=cfg["K"], linsys_lr=cfg["linsys_lr"])
    b, _ = _psvi(f)
    lb = b.hyper_step(xb, yb, K=cfg["K"], linsys_lr=cfg["linsys_lr"],
                      eps_inner=[torch.tensor(e, device="cuda") for e in f["eps_inner"]],
                      eps_outer=[torch.tensor(e, device="cuda") for e in f["eps_outer"]])
    # two fp32 inner loops (per-step gradient + Adam kernel vs the fused step)
    # and CG orders: both sit within 1e-4 of the reference's fixture
    assert rel(la, lb) < 1e-6
    assert l2rel(a.u.grad.cpu().numpy(), b.u.grad.cpu().numpy()) < 2e-4
    assert l2rel(a.v.grad.cpu().numpy(), b.v.grad.cpu().numpy()) < 2e-4


def test_gd_step_node_is_i_minus_lr_hessian():
    """GradientDescent's HIP node: torch.autograd.grad(w_mapped, params, v) =
    v - lr H v and the jvp (two fresh draws, the second differentiated) equal
    psvi_hvp on the same draws."""
    from psvi.hypergrad import GradientDescent, jvp
    from psvi.robust_higher import monkeypatch
    from psvi.runtime import randn_

    f = load_fixture("y2_fn_deep")
    ps, model = _psvi(f)
    plan = ps._plan(model)
    draws = [randn_(torch.empty(plan.eps_count, device="cuda"), 40 + i) for i in range(3)]
    ps.replay_eps(draws)
    fmodel = monkeypatch(model)
    params = [p.detach().clone().requires_grad_(True) for p in fmodel.parameters()]
    lr = 1e-2
    fp = GradientDescent(lambda p, hp: ps.inner_elbo(model=fmodel, params=p, hyperopt=True), lr)
    w_mapped = fp(params, [ps.u, ps.v])
    v = [torch.randn_like(p) for p in params]
    jt = torch.autograd.grad(w_mapped, params, grad_outputs=v, retain_graph=True)
    pv = nn.utils.parameters_to_vector(params).detach()
    vv = torch.cat([x.reshape(-1) for x in v])
    u, z, w = ps._data(plan)
    hv0, _, _ = plan.hvp(u, z, w, draws[0], pv, vv, mixed=False)
    got = torch.cat([x.reshape(-1) for x in jt])
    assert torch.allclose(got, vv - lr * hv0, rtol=1e-5, atol=1e-6)
    jv = jvp(lambda p: fp(p, [ps.u, ps.v]), params, v)
    hv2, _, _ = plan.hvp(u, z, w, draws[2], pv, vv, mixed=False)
    assert torch.allclose(torch.cat([x.reshape(-1) for x in jv]), vv - lr * hv2, rtol=1e-5,
                          atol=1e-6)
    # the mixed products reach u and v through the node
    gu, gv = torch.autograd.grad(w_mapped, [ps.u, ps.v], grad_outputs=v)
    _, du, dw = plan.hvp(u, z, w, draws[0], pv, vv, mixed=True)
    assert torch.allclose(gu, (-lr * du).reshape(gu.shape), rtol=1e-5, atol=1e-7)
    wgt = ps.N * torch.softmax(ps.v, 0)             # PSVILearnV's N f(v)
    wv = torch.autograd.grad(wgt, ps.v, grad_outputs=(-lr * dw).to(wgt.dtype))[0]
    assert torch.allclose(gv, wv, rtol=1e-5, atol=1e-7)
