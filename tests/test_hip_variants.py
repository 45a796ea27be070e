"""The PSVI plugin variants on the GPU, through the reference-shaped API,
against whole outer steps of the reference's own classes (tests/golden/v*.npz,
tools/gen_golden_variants.py): PSVIAV and PSVIAFixedU (alpha learned by its
own Adam), PSVIFixedU and PSVIAFixedU (u frozen), PSVI_Ablated (the ablated
outer objective, psvi_outer_ablated_elbo_grad) and PSVI_No_IW (single-sample
training).  Where the reference itself fails, the same exception type."""
import numpy as np
import pytest
import torch

from golden_util import fixture_names, l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu


def make(name):
    import psvi.inference as PI
    from test_host_api import build_model

    f = load_fixture(name)
    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    u = torch.tensor(f["u0"], device="cuda").requires_grad_(True)
    z = torch.tensor(f["z"], device="cuda")
    ps = getattr(PI, cfg["cls"])(u=u, z=z, N=cfg["N"], model=model, mc_samples=cfg["S"],
                                 device_id=0, inner_it=cfg["T"], lr0alpha=cfg["lr0alpha"])
    ps.device = torch.device("cuda")
    ps.v = torch.tensor(f["v0"], device="cuda").requires_grad_(True)
    if cfg.get("alpha0") is not None:
        ps.alpha = torch.tensor([cfg["alpha0"]], device="cuda").requires_grad_(True)
    ps.setup_optimizers(lr0net=cfg["lr0net"], lr0u=cfg["lr0u"], lr0v=cfg["lr0v"])
    ps.scheduler_optim_net = None
    return f, cfg, model, ps


def run(f, cfg, ps):
    xb = torch.tensor(f["xb"], device="cuda")
    yb = torch.tensor(f["yb"], device="cuda")
    ei = [torch.tensor(e, device="cuda") for e in f.get("eps_inner", [])]
    eo = [torch.tensor(e, device="cuda") for e in f.get("eps_outer", [])]
    if cfg["trainer"] == "psvi_elbo":
        loss = ps.psvi_elbo(xb, yb, eps=eo[0] if eo else None)
        loss.backward()
        return loss.item()
    if cfg["trainer"] == "nested":
        return ps.nested_step(xb, yb, eps_inner=ei, eps_outer=eo).item()
    return ps.hyper_step(xb, yb, K=cfg["K"], linsys_lr=cfg["linsys_lr"], eps_inner=ei,
                         eps_outer=eo, hypergrad_approx=cfg["approx"])


@pytest.mark.parametrize("name", fixture_names("v"))
def test_variant_step_matches_reference(name):
    f, cfg, model, ps = make(name)
    if "raises" in cfg:
        exc = {"IndexError": IndexError, "AttributeError": AttributeError}[cfg["raises"]]
        with pytest.raises(exc):
            run(f, cfg, ps)
        return
    out = run(f, cfg, ps)
    print(f"{name}: out {out:.6f} (reference {float(f['out']):.6f})")
    assert rel(out, f["out"]) < 1e-5
    p = torch.nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy()
    if cfg["trainer"] == "psvi_elbo":
        g = torch.cat([q.grad.reshape(-1) for q in model.parameters()]).cpu().numpy()
        assert l2rel(g, f["grad_params"]) < 1e-4
        assert ps.u.grad is None or float(ps.u.grad.abs().max()) == 0.0
        return
    assert l2rel(p, f["params"]) < 1e-5
    hp = [("v_grad", ps.v, "v", cfg["lr0v"])]
    if "u_grad" in f:
        hp.append(("u_grad", ps.u, "u", cfg["lr0u"]))
    else:  # u frozen: no gradient, no step
        assert ps.u.grad is None
        assert np.array_equal(ps.u.detach().cpu().numpy(), f["u0"])
        assert not ps.u.requires_grad
    if "alpha_grad" in f:
        hp.append(("alpha_grad", ps.alpha, "alpha", cfg["lr0alpha"]))
    for key, t, vkey, lr in hp:
        got = t.grad.detach().cpu().numpy()
        own = l2rel(f[key + "_fp32"], f[key]) if key + "_fp32" in f else 0.0
        e = l2rel(got, f[key])
        print(f"  {key}: l2rel {e:.2e} (reference fp32 {own:.2e})")
        assert e < max(1e-4, 4 * own), key
        big = np.abs(f[key]) > 1e-2 * np.abs(f[key]).max()
        assert np.abs(t.detach().cpu().numpy() - f[vkey])[big].max() < 1e-3 * lr, vkey


def test_ablated_outer_kernel_matches_oracle():
    """psvi_outer_ablated_elbo_grad at random states against the oracle, both
    mean-field and LeNet, S = 1 included."""
    import psvi_oracle as O
    from golden_util import LENET_PLAN_LAYERS
    from psvi.runtime import InnerLoopPlan

    rng = np.random.default_rng(5)
    for fam, layers, S, Nx, D, C in (("mf", [(5, 7), (7, 3)], 6, 9, 5, 3),
                                      ("mf", [(2, 2)], 1, 16, 2, 2),
                                      ("mf", [(12, 30), (30, 30), (30, 4)], 64, 200, 12, 4),
                                      ("lenet", LENET_PLAN_LAYERS, 3, 5, 784, 10)):
        fam_plan = {"mf": "meanfield", "lenet": "lenet"}[fam]
        plan = InnerLoopPlan(fam_plan, layers, S, Nx)
        if fam == "lenet":
            from test_hip_lenet import _random_state
            params = _random_state(rng, S, 1)[0]
        else:
            params = rng.normal(0, 0.3, plan.param_count).astype(np.float32)
            po = 0
            for din, dout in layers:
                n = din * dout + dout
                params[po + n:po + 2 * n] = rng.uniform(-4, -1, n)
                po += 2 * n
        eps = rng.standard_normal(plan.eps_count).astype(np.float32)
        xb = rng.normal(0, 1, (Nx, D)).astype(np.float32)
        yb = rng.integers(0, C, Nx).astype(np.int32)
        N = 800
        w = np.full(Nx, N / Nx, np.float32)
        t = lambda a, d=torch.float32: torch.tensor(a, dtype=d, device="cuda")
        out = plan.outer_ablated_elbo_grad(t(xb), t(yb, torch.int32), t(w), t(eps), t(params))
        loss, g, _, _ = O.outer_elbo_grad(fam, layers, params, xb, yb, w, 0, eps, S,
                                          mode="ablated")
        assert rel(out["loss"].item(), loss) < 1e-6, (fam, out["loss"].item(), loss)
        assert l2rel(out["grad"].cpu().numpy(), g) < 1e-5, fam


def test_ablated_rejects_fullcov_plan():
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime._lib import PsviError

    plan = InnerLoopPlan("fullcov", [(4, 3), (3, 2)], 4, 8)
    z = torch.zeros(8, dtype=torch.int32, device="cuda")
    with pytest.raises(PsviError):
        plan.outer_ablated_elbo_grad(torch.zeros(8, 4, device="cuda"), z,
                                     torch.ones(8, device="cuda"),
                                     torch.zeros(plan.eps_count, device="cuda"),
                                     torch.zeros(plan.param_count, device="cuda"))
