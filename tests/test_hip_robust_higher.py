"""psvi.robust_higher (innerloop_ctx / DifferentiableAdam.step) on the GPU.

``_reference_nested_step`` is the call sequence of the reference's
PSVI.nested_step (psvi/inference/psvi_classes.py:541-560, 584-600): optimiser
zero_grads, ``innerloop_ctx(self.model, self.optim_net)``, inner_it times
``diffopt.step(self.inner_elbo(model=fmodel))`` with the elbo log, then
``self.psvi_elbo(xbatch, ybatch, model=fmodel).backward()``, the u / v Adam
steps and the copy of the fast weights into the model -- driven through this
package's PSVI methods, with the reference's own draws replayed (replay_eps).
It must reproduce the reference's whole nested_step (n* fixtures) and agree
with this package's hand-written reverse pass (PSVI.nested_step)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from golden_util import fixture_names, l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu


def _reference_nested_step(self, xbatch, ybatch):
    from psvi.robust_higher import innerloop_ctx

    self.optim_u.zero_grad()
    self.optim_net.zero_grad()
    if self.learn_v:
        self.optim_v.zero_grad()
    with innerloop_ctx(self.model, self.optim_net) as (fmodel, diffopt):
        for in_it in range(self.inner_it):
            mfvi_loss = self.inner_elbo(model=fmodel)
            with torch.no_grad():
                if self.register_elbos and in_it % self.log_every == 0:
                    self.elbos.append((1, -mfvi_loss.item()))
            diffopt.step(mfvi_loss)
        psvi_loss = self.psvi_elbo(xbatch, ybatch, model=fmodel)
        with torch.no_grad():
            if self.register_elbos:
                self.elbos.append((0, -psvi_loss.item()))
        psvi_loss.backward()
    self.optim_u.step()
    if self.learn_v:
        self.optim_v.step()
        if not self.parameterised:
            with torch.no_grad():
                torch.clamp_(self.v, min=0.0)
    nn.utils.vector_to_parameters(nn.utils.parameters_to_vector(list(fmodel.parameters())),
                                  self.model.parameters())
    return psvi_loss


def _psvi(f):
    from psvi.inference import PSVILearnV
    from test_host_api import build_model

    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    u = torch.tensor(f["u0"], device="cuda").requires_grad_(True)
    ps = PSVILearnV(u=u, z=torch.tensor(f["z"], device="cuda"), N=cfg["N"], model=model,
                    mc_samples=cfg["S"], device_id=0, inner_it=cfg["T"])
    ps.device = torch.device("cuda")
    ps.v = torch.tensor(f["v0"], device="cuda").requires_grad_(True)
    ps.setup_optimizers(lr0net=cfg["lr0net"], lr0u=cfg["lr0u"], lr0v=cfg["lr0v"])
    return ps, model


@pytest.mark.parametrize("name", fixture_names("n"))
def test_reference_nested_step_body_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    ps, model = _psvi(f)
    ps.replay_eps([torch.tensor(e, device="cuda") for e in f["eps_inner"]] +
                  [torch.tensor(e, device="cuda") for e in f["eps_outer"]])
    loss = _reference_nested_step(ps, torch.tensor(f["xb"], device="cuda"),
                                  torch.tensor(f["yb"], device="cuda"))
    assert rel(loss.item(), f["loss"]) < 1e-5
    p = nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy()
    assert l2rel(p, f["params"]) < 1e-5
    for key in ("u_grad", "v_grad"):
        got = (ps.u if key == "u_grad" else ps.v).grad.cpu().numpy()
        own = l2rel(f[key + "_fp32"], f[key])   # bar as tests/test_host_api_gpu.py
        print(f"{name}: {key} l2rel {l2rel(got, f[key]):.2e} (reference fp32: {own:.2e})")
        assert l2rel(got, f[key]) < max(1e-4, 4 * own)
    assert [e[0] for e in ps.elbos][-1] == 0


def test_functional_unroll_equals_hand_reverse_pass():
    """The autograd-composed reverse pass (robust_higher) and PSVI.nested_step's
    hand-written one give the same hypergradients on the same draws."""
    f = load_fixture("n2_fn_deep")
    ei = [torch.tensor(e, device="cuda") for e in f["eps_inner"]]
    eo = [torch.tensor(e, device="cuda") for e in f["eps_outer"]]
    xb, yb = torch.tensor(f["xb"], device="cuda"), torch.tensor(f["yb"], device="cuda")
    a, _ = _psvi(f)
    a.replay_eps(ei + eo)
    la = _reference_nested_step(a, xb, yb)
    b, _ = _psvi(f)
    lb = b.nested_step(xb, yb, eps_inner=ei, eps_outer=eo)
    assert rel(la.item(), lb.item()) < 1e-6
    assert l2rel(a.u.grad.cpu().numpy(), b.u.grad.cpu().numpy()) < 1e-5
    assert l2rel(a.v.grad.cpu().numpy(), b.v.grad.cpu().numpy()) < 1e-5


def test_inner_elbo_backward_reaches_u_and_v():
    """inner_elbo's autograd reaches u and v like the reference's: the row
    gradients of the weighted NLL (the KL does not depend on the rows),
    against a float64 torch autograd restatement of the mean-field network
    (tests/test_sharded_outer_gloo.py's stand-in) on the same draw."""
    from psvi.runtime import randn_
    from test_sharded_outer_gloo import _AutogradMFPlan

    f = load_fixture("n2_fn_deep")
    cfg = f["cfg"]
    ps, model = _psvi(f)
    plan = ps._plan(model)
    e = randn_(torch.empty(plan.eps_count, device="cuda"), 3)
    ps.inner_elbo(eps=e).backward()
    ref = _AutogradMFPlan([tuple(l) for l in cfg["layers"]], cfg["S"], cfg["prior_sd"])
    X = torch.tensor(f["u0"], dtype=torch.float64).requires_grad_()
    v = torch.tensor(f["v0"], dtype=torch.float64).requires_grad_()
    pseudo, _, _ = ref._terms(X.shape[0], X, torch.tensor(f["z"]).long(),
                              cfg["N"] * torch.softmax(v, 0), e.double().cpu(),
                              torch.tensor(f["params0"], dtype=torch.float64))
    pseudo.sum().backward()
    assert l2rel(ps.u.grad.cpu().numpy(), X.grad.numpy()) < 1e-5
    assert l2rel(ps.v.grad.cpu().numpy(), v.grad.numpy()) < 1e-5
