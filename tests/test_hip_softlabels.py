"""Soft labels (learn_z) and the truncated nested step on the GPU, against the
reference's own runs (tests/golden/w*, tools/gen_golden_softlabels.py: float64
with fp32 draws, the draws replayed here in call order).

* w01 PSVILearnV.nested_step and w02 PSVIAFixedU.nested_step (LeNet, the
  reference's psvi_alpha_fixed_u learn_z configuration) with learn_z: the
  soft-label inner and outer objectives as expanded rows, the hypergradient of
  z (and v, alpha, u) through psvi.robust_higher's unroll, optim_z stepped;
* w03 nested_step(truncated=True): the non-differentiable torch.optim.Adam
  warm start whose gradients accumulate into the network, u and v;
* w04 psvi_elbo and w05 inner_elbo with learn_z and their backward into z,
  u, v and the parameters.
Bar: values 1e-5 relative, gradients 1e-4 l2-relative or four times the
reference's own fp32 deviation on the same draws (unrolled steps)."""
import numpy as np
import pytest
import torch

from golden_util import fixture_names, l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu


def _setup(f, world=1, rank=0, comm=None):
    import psvi.inference as I
    from test_host_api import build_model

    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    dev = torch.device("cuda")
    u = torch.tensor(f["u0"], device=dev).requires_grad_(True)
    z = torch.tensor(f["z0"], device=dev)
    ps = getattr(I, cfg["cls"])(u=u, z=z, N=cfg["N"], model=model, mc_samples=cfg["S"],
                                device_id=0, inner_it=cfg["T"], learn_z=cfg["learn_z"],
                                lr0alpha=cfg["lr0alpha"], nc=cfg["C"], world=world, rank=rank,
                                comm=comm)
    ps.device = dev
    ps.register_elbos = False
    ps.v = torch.tensor(f["v0"], device=dev).requires_grad_(True)
    if cfg.get("alpha0") is not None:
        ps.alpha = torch.tensor([cfg["alpha0"]], device=dev).requires_grad_(True)
        ps.f = lambda *x: torch.exp(ps.alpha) * torch.softmax(x[0], x[1])
    ps.setup_optimizers(lr0net=cfg["lr0net"], lr0u=cfg["lr0u"], lr0v=cfg["lr0v"],
                        lr0z=cfg["lr0z"])
    if cfg.get("alpha0") is not None:
        ps.optim_alpha = torch.optim.Adam([ps.alpha], cfg["lr0alpha"])
    draws = [torch.tensor(e, device=dev) for e in f.get("eps_inner", [])] + \
            [torch.tensor(e, device=dev) for e in f.get("eps_outer", [])]
    ps.replay_eps(draws)
    return ps, model


@pytest.mark.parametrize("name", fixture_names("w"))
def test_softlabels_and_truncated_match_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    ps, model = _setup(f)
    xb = torch.tensor(f["xb"], device="cuda")
    yb = torch.tensor(f["yb"], device="cuda")
    tr = cfg["trainer"]
    if tr == "psvi_elbo":
        loss = ps.psvi_elbo(xb, yb)
        loss.backward()
    elif tr == "inner_elbo":
        loss = ps.inner_elbo()
        loss.backward()
    else:
        loss = ps.nested_step(xb, yb, truncated=(tr == "truncated"), K=cfg["K"])
    assert rel(loss.item(), float(f["out"])) < 1e-5, (loss.item(), float(f["out"]))
    p = torch.nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy()
    assert l2rel(p, f["params"]) < 1e-5
    if "grad_params" in f:
        g = torch.cat([q.grad.reshape(-1) for q in model.parameters()]).cpu().numpy()
        assert l2rel(g, f["grad_params"]) < 1e-4
    for key, t in (("u_grad", ps.u), ("v_grad", ps.v), ("z_grad", ps.z),
                   ("alpha_grad", getattr(ps, "alpha", None))):
        if key not in f:
            continue
        got = t.grad.detach().cpu().numpy().reshape(f[key].shape)
        own = l2rel(f[key + "_fp32"], f[key]) if key + "_fp32" in f else 0.0
        err = l2rel(got, f[key])
        print(f"{name}: {key} l2rel {err:.2e} (reference fp32 {own:.2e})")
        assert err < max(1e-4, 4 * own), (name, key, err)
    if cfg["learn_z"] and tr in ("nested", "truncated"):
        # optim_z's first step moves z by -lr sign(grad): compared wherever the
        # reference's gradient is not within its own fp32 rounding of zero
        g = f["z_grad"]
        big = np.abs(g) > 4 * np.abs(f["z_grad_fp32"] - g) + 1e-2 * np.abs(g).max()
        dz = np.abs(ps.z.detach().cpu().numpy() - f["z"])[big]
        assert dz.max() < 1e-3 * cfg["lr0z"] + 1e-6


@pytest.mark.parametrize("name,world", [("w04_learnz_psvi_elbo_fn2", 2), ("w04_learnz_psvi_elbo_fn2", 3)])
def test_softlabels_samples_sharded_match_reference(name, world):
    """learn_z with the samples split over ranks (ranks as threads of one
    process, all_reduce through a barrier): the soft-label outer objective on
    ShardedOuter (psvi_classes.py:445-486) -- loss and gradients into z, u, v
    and the parameters -- on every rank against the reference's own run.
    (A nested step cannot run on thread ranks: its unrolled backward calls the
    sample-sharded HVP's all_reduce from inside autograd, and the ranks'
    backward passes share one autograd device thread.)"""
    from test_hip_sharded_trainer import _run_ranks

    f = load_fixture(name)
    cfg = f["cfg"]

    def rank_fn(r, comm):
        ps, model = _setup(f, world, r, comm)
        xb = torch.tensor(f["xb"], device="cuda")
        yb = torch.tensor(f["yb"], device="cuda")
        if cfg["trainer"] == "psvi_elbo":
            loss = ps.psvi_elbo(xb, yb)
            loss.backward()
        else:
            loss = ps.nested_step(xb, yb, K=cfg["K"])
        out = dict(loss=loss.item(),
                   params=torch.nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy())
        if "grad_params" in f:
            out["grad_params"] = torch.cat([q.grad.reshape(-1) for q in model.parameters()]).cpu().numpy()
        for key, t in (("u_grad", ps.u), ("v_grad", ps.v), ("z_grad", ps.z)):
            if key in f:
                out[key] = t.grad.detach().cpu().numpy().reshape(f[key].shape)
        return out

    for g in _run_ranks(world, rank_fn):
        assert rel(g["loss"], float(f["out"])) < 1e-5, (g["loss"], float(f["out"]))
        assert l2rel(g["params"], f["params"]) < 1e-5
        if "grad_params" in g:
            assert l2rel(g["grad_params"], f["grad_params"]) < 1e-4
        for key in ("u_grad", "v_grad", "z_grad"):
            if key in g:
                own = l2rel(f[key + "_fp32"], f[key]) if key + "_fp32" in f else 0.0
                assert l2rel(g[key], f[key]) < max(1e-4, 4 * own), (name, key, l2rel(g[key], f[key]))
