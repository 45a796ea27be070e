"""Host-side mirror of the reference API (psvi.models / psvi.inference) on CPU:
parameter layout, model specs, coreset weights and KL closed forms.  The HIP
calls behind inner_elbo / inner_loop are exercised in test_host_api_gpu.py."""
import numpy as np
import pytest
import torch
import torch.distributions as dist
import torch.nn as nn

import psvi_oracle as O
from golden_util import family_of, fixture_names, load_fixture


def build_model(cfg, params0):
    """The reference module stack a fixture was generated from, at params0."""
    from psvi.models import VILinear, VILinearMultivariateNormal, make_lenet

    if cfg["family"] == "lenet":
        net = make_lenet(mc_samples=cfg["S"])
        with torch.no_grad():
            nn.utils.vector_to_parameters(torch.tensor(params0, dtype=torch.float32),
                                          net.parameters())
        return net
    cls = VILinear if family_of(cfg) == "meanfield" else VILinearMultivariateNormal
    mods = []
    for i, (a, b) in enumerate(cfg["layers"]):
        mods.append(cls(a, b, mc_samples=cfg["S"], prior_sd=cfg["prior_sd"]))
        if i + 1 < len(cfg["layers"]):
            mods.append(nn.ReLU())
    net = nn.Sequential(*mods)
    with torch.no_grad():
        nn.utils.vector_to_parameters(torch.tensor(params0, dtype=torch.float32),
                                      net.parameters())
    return net


def fixture_model(name):
    f = load_fixture(name)
    return f, build_model(f["cfg"], f["params0"])


def make_psvi(f, model, device="cpu"):
    from psvi.inference import PSVIAV, PSVILearnV

    cfg = f["cfg"]
    cls = PSVIAV if cfg["f"] == "exp_alpha_softmax" else PSVILearnV
    u = torch.tensor(f["u"], dtype=torch.float32, device=device)
    z = torch.tensor(f["z"], dtype=torch.float32, device=device)
    ps = cls(u=u, z=z, N=cfg["N"], model=model, mc_samples=cfg["S"], lr0net=cfg["lr"],
             device_id=0 if device == "cuda" else None)
    ps.device = torch.device(device)
    with torch.no_grad():
        ps.v = torch.tensor(f["v"], dtype=torch.float32, device=device)
        if cfg["f"] == "exp_alpha_softmax":
            ps.alpha = torch.tensor([cfg["alpha"]], dtype=torch.float32, device=device)
    return ps


def test_builders_match_reference_layout():
    from psvi.models import make_fc2net, make_fcnet, make_logreg, model_spec
    from psvi.runtime import InnerLoopPlan

    net = make_fc2net(64, 40, 2, mc_samples=128, init_sd=1e-6)
    assert [n for n, _ in net.named_parameters()][:3] == ["lin0.mean", "lin0._sd", "lin0._corr"]
    fam, layers, prior, S = model_spec(net)
    assert (fam, layers, prior, S) == ("fullcov", [(64, 40), (40, 40), (40, 2)], 1.0, 128)
    plan = InnerLoopPlan(fam, layers, S, 100)
    assert sum(p.numel() for p in net.parameters()) == plan.param_count == 4_730_326
    # init: mean 0, corr 0, sd = softplus^-1(init_sd)
    assert torch.all(net[0].mean == 0) and torch.all(net[0]._corr == 0)
    assert torch.allclose(torch.nn.functional.softplus(net[0]._sd), torch.full((2600,), 1e-6))

    net = make_fcnet(2, 100, 4, n_layers=1, mc_samples=32)
    assert [n for n, _ in net.named_parameters()] == [
        "lin0.weight", "lin0.bias", "lin0._weight_sd", "lin0._bias_sd",
        "classifier.weight", "classifier.bias", "classifier._weight_sd", "classifier._bias_sd"]
    fam, layers, prior, S = model_spec(net)
    assert sum(p.numel() for p in net.parameters()) == \
        InnerLoopPlan(fam, layers, S, 50).param_count == 1408
    assert model_spec(make_logreg(2, 2, mc_samples=4))[1] == [(2, 2)]
    assert model_spec(make_logreg(2, 2, fullcov=True, mc_samples=4))[0] == "fullcov"


def test_model_spec_rejects_unsupported_stacks():
    from psvi.models import VILinear, VILinearMultivariateNormal, model_spec

    with pytest.raises(ValueError):
        model_spec(nn.Sequential(VILinear(2, 3), nn.Tanh(), VILinear(3, 2)))
    with pytest.raises(ValueError):
        model_spec(nn.Sequential(VILinear(2, 3), nn.ReLU(), VILinearMultivariateNormal(3, 2)))
    with pytest.raises(ValueError):
        model_spec(nn.Sequential(VILinear(2, 3), nn.ReLU()))
    with pytest.raises(ValueError):
        model_spec(nn.Sequential(nn.Linear(2, 3)))


@pytest.mark.parametrize("name", fixture_names())
def test_fixture_params_roundtrip_and_weights(name):
    f, model = fixture_model(name)
    vec = nn.utils.parameters_to_vector(model.parameters()).detach().numpy()
    assert np.array_equal(vec, f["params0"].astype(np.float32))
    ps = make_psvi(f, model)
    w = ps.coreset_weights().numpy()
    assert np.allclose(w, f["w"], rtol=1e-6, atol=0), (w[:4], f["w"][:4])


@pytest.mark.parametrize("name", fixture_names())
def test_module_kl_matches_oracle_closed_form(name):
    f, model = fixture_model(name)
    cfg = f["cfg"]
    kl = float(sum(m.kl().detach() for m in model if not isinstance(m, nn.ReLU)))
    # the oracle's ELBO minus its data term is the KL; evaluate with w = 0
    fn = O.mf_elbo_grad if cfg["family"] == "mf" else O.mvn_elbo_grad
    val, _ = fn(cfg["layers"], f["params0"], f["u"], f["z"], np.zeros_like(f["w"]),
                f["eps"][0], cfg["S"], prior_sd=cfg["prior_sd"])
    assert abs(kl - val) <= 1e-4 * max(1.0, abs(val)), (kl, val)


def test_fullcov_kl_closed_form_equals_torch_triangular_solve():
    from psvi.models import VILinearMultivariateNormal

    torch.manual_seed(0)
    layer = VILinearMultivariateNormal(3, 2, prior_sd=0.7, init_sd=0.3).double()
    with torch.no_grad():
        layer.mean.normal_()
        layer._sd.normal_()
        layer._corr.normal_(std=0.2)
    ref = dist.kl_divergence(layer.param_dist, layer.prior_dist)
    assert torch.allclose(layer.kl(), ref, rtol=1e-10), (layer.kl(), ref)


def test_inner_loop_refuses_cpu_tensors():
    """No CPU fallback: without a HIP device the product path raises."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    f, model = fixture_model("g3r_fn2_tiny_rand")
    ps = make_psvi(f, model)
    with pytest.raises(ValueError, match="device tensor"):
        ps.inner_elbo(eps=torch.zeros(10))
    with pytest.raises(ValueError, match="device tensor"):
        ps.inner_loop(T=1)


def test_second_order_entry_points_raise():
    f, model = fixture_model("g1_logreg_c1")
    ps = make_psvi(f, model)
    def soft_hyper():
        ps.learn_z = True       # the reference's hyper_step raises for learn_z (619-620)
        try:
            ps.hyper_step(None, None)
        finally:
            ps.learn_z = False

    for fn in (soft_hyper,
               lambda: ps.run_psvi(init_args="custom"),
               lambda: ps.hyper_step(None, None, hypergrad_approx="neumann")):
        with pytest.raises(NotImplementedError):
            fn()


def test_outer_objective_has_no_cpu_fallback():
    """psvi_elbo runs on the HIP library only: host tensors (or a missing
    device / library) raise instead of computing anywhere else."""
    from psvi.runtime._lib import PsviError

    f, model = fixture_model("g1_logreg_c1")
    ps = make_psvi(f, model)
    xb, yb = torch.randn(8, 2), torch.zeros(8)
    with pytest.raises((ValueError, PsviError)):
        ps.psvi_elbo(xb, yb)


def test_make_lenet_layout_and_spec():
    """make_lenet (neural_net.py:334-359): parameter order = the library's
    layout, model_spec -> family "lenet"; the last layer keeps mc_samples=1."""
    from psvi.models import LENET_LAYERS, make_lenet, model_spec, set_mc_samples

    net = make_lenet(mc_samples=4, init_sd=0.05)
    names = [n for n, _ in net.named_parameters()]
    assert names[:4] == ["0.weight", "0.bias", "0._weight_sd", "0._bias_sd"]
    assert sum(p.numel() for p in net.parameters()) == O.lenet_param_count()
    assert model_spec(net) == ("lenet", LENET_LAYERS, 1.0, 4)
    assert net[11].mc_samples == 1
    f = load_fixture("l1_lenet_tiny")
    with torch.no_grad():
        nn.utils.vector_to_parameters(torch.tensor(f["params0"]), net.parameters())
    assert np.array_equal(nn.utils.parameters_to_vector(net.parameters()).detach().numpy(),
                          f["params0"])
    set_mc_samples(net, 4)  # also sets the last layer: no longer make_lenet's model
    with pytest.raises(ValueError, match="shared sample"):
        model_spec(net)


def test_lenet_torch_forward_matches_oracle():
    """The host VIConv2d / BatchMaxPool2d modules (prediction path) compute the
    oracle's forward on the same weight draws."""
    from psvi.models import make_lenet

    f = load_fixture("l1_lenet_tiny")
    S = f["cfg"]["S"]
    net = make_lenet(mc_samples=S).double()
    with torch.no_grad():
        nn.utils.vector_to_parameters(torch.tensor(f["params0"], dtype=torch.float64),
                                      net.parameters())
    Xl = O.lenet_sample(f["params0"], f["eps"][0], S)
    logits_o, _ = O.lenet_forward(Xl, f["u"], S)
    draws = []
    for x, (nw, nb, bat, _) in zip(Xl, O.LENET_LAYERS):
        E = x["E"]
        draws += [E[:, :nw], E[:, nw:]]
    it = iter(draws)
    import psvi.models.neural_net as nnmod

    def fake_rsample(self):
        ew, eb = next(it), next(it)
        ew = torch.tensor(ew).reshape((self.mc_samples,) * (self.mc_samples > 1) + self.weight.shape)
        eb = torch.tensor(eb).reshape(((self.mc_samples, 1) if self.mc_samples > 1 else ())
                                      + self.bias.shape)
        return self.weight + self.weight_sd * ew, self.bias + self.bias_sd * eb

    orig = nnmod.VIMixin.rsample
    nnmod.VIMixin.rsample = fake_rsample
    try:
        logits = net(torch.tensor(f["u"], dtype=torch.float64)).detach().numpy()
    finally:
        nnmod.VIMixin.rsample = orig
    assert np.allclose(logits, logits_o, rtol=1e-10, atol=1e-10)


# ------------------------------------------------------------ plugin variants
def _variant(cls_name, S=4, M=6, C=3, D=2):
    import psvi.inference as PI
    from psvi.models import make_fcnet

    torch.manual_seed(0)
    model = make_fcnet(D, 5, C, n_layers=1, mc_samples=S)
    u = torch.randn(M, D).requires_grad_(True)
    z = torch.tensor([float(i % C) for i in range(M)])
    ps = getattr(PI, cls_name)(u=u, z=z, N=100, model=model, mc_samples=S, lr0alpha=0.05)
    ps.device = torch.device("cpu")
    return ps


def test_variant_switches_follow_the_reference_classes():
    import psvi.inference as PI

    assert PI.PSVIFixedU._learn_u is False and PI.PSVIAFixedU._learn_u is False
    assert PI.PSVI_Ablated._outer_mode == "ablated" and PI.PSVI_No_IW._outer_mode == "ablated"
    assert PI.PSVI_No_IW._noiw and not PI.PSVI_Ablated._noiw
    assert issubclass(PI.PSVIAFixedU, PI.PSVILearnV) and not issubclass(PI.PSVIAFixedU, PI.PSVIAV)
    ps = _variant("PSVI_No_IW", S=1)
    assert ps.mc_samples == 1
    for name in ("PSVIAV", "PSVIAFixedU"):
        ps = _variant(name)
        assert float(ps.alpha) == 0.0 and ps.alpha.requires_grad
        assert ps.optim_alpha.param_groups[0]["lr"] == 0.05
        ps.setup_optimizers()
        assert ps.optim_alpha.param_groups[0]["params"][0] is ps.alpha


def test_chain_w_gives_v_and_alpha_gradients():
    ps = _variant("PSVIAV")
    with torch.no_grad():
        ps.alpha.fill_(0.3)
        ps.v.copy_(torch.linspace(-1, 1, 6))
    dw = torch.randn(6, dtype=torch.float64)
    gv, ga = ps._chain_w(dw)
    v = ps.v.detach().double().requires_grad_(True)
    a = ps.alpha.detach().double().requires_grad_(True)
    (100 * torch.exp(a) * torch.softmax(v, 0) * dw).sum().backward()
    assert torch.allclose(gv.double(), v.grad, rtol=1e-5)
    assert torch.allclose(ga.double(), a.grad, rtol=1e-5)
    ps2 = _variant("PSVILearnV")
    gv2, ga2 = ps2._chain_w(dw)
    assert ga2 is None and gv2.shape == (6,)


def test_noiw_rows_reproduce_the_broadcast_objective():
    """PSVI_No_IW's single-sample inner objective (the reference's (M, M)
    broadcast of Categorical.log_prob) equals the standard objective over
    the M*C expanded rows _data builds."""
    from psvi.models import model_spec

    ps = _variant("PSVI_No_IW", S=1, M=7, C=3)
    with torch.no_grad():
        ps.v.copy_(torch.rand(7))
    fam, layers, _, _ = model_spec(ps.model)

    class P:
        M, in_features = 7 * 3, 2
    P.layers = layers
    u, z, w = ps._data(P)
    assert u.shape == (21, 2) and z.tolist() == [0, 1, 2] * 7
    logits = torch.randn(7, 3, dtype=torch.float64)
    wp = ps.coreset_weights().double()
    # reference: logits (M, 1, C) against z (M,) -> (M, M), matmul w, sum
    ref = -torch.distributions.Categorical(logits=logits.unsqueeze(1)).log_prob(ps.z.double())
    ref = ref.matmul(wp).sum()
    le = logits.repeat_interleave(3, 0)
    got = (-torch.distributions.Categorical(logits=le).log_prob(z.double()) * w.double()).sum()
    assert torch.allclose(got, ref, rtol=1e-6)
    du, dw = ps._fold(P, torch.ones(21, 2), torch.arange(21.0))
    assert du.shape == (7, 2) and torch.all(du == 3)
    byclass = torch.arange(21.0).reshape(7, 3).sum(0)
    assert torch.equal(dw, byclass[ps.z.long()])


def test_minibatch_labels_out_of_range_raise():
    """psvi_elbo / the trainers take class ids in [0, C) as the reference's
    Categorical.log_prob does: ids outside that range (1-based, -1, or
    non-integral floats) raise ValueError instead of being clamped onto
    another class.  Outside a trainer the flag is read at the call; inside one
    it is read once per outer step (before the hyperparameters move)."""
    ps = _variant("PSVILearnV", M=6, C=3)
    x = torch.randn(5, 2)
    for bad in (torch.tensor([0, 1, 2, 3, 1]), torch.tensor([-1, 0, 1, 2, 0]),
                torch.tensor([0.0, 1.5, 2.0, 1.0, 0.0])):
        with pytest.raises(ValueError, match=r"\[0, 3\)"):
            ps._outer_rows(x, bad, 3)
    xb, yb, wd = ps._outer_rows(x, torch.tensor([0, 1, 2, 2, 1]), 3)
    assert yb.dtype == torch.int32 and yb.tolist() == [0, 1, 2, 2, 1]
    assert torch.allclose(wd, torch.full((5,), ps.N / 5.0))
    # deferred inside a trainer step: no read until the step ends, then it raises
    with pytest.raises(ValueError, match=r"\[0, 3\)"):
        with ps._outer_step():
            ps._outer_rows(x, torch.tensor([0, 1, 4, 2, 1]), 3)
            ps._outer_rows(x, torch.tensor([0, 1, 2, 2, 1]), 3)   # flag stays set
            assert ps._label_flag is not None
    assert ps._label_flag is None
    with ps._outer_step():                                        # a clean step
        ps._outer_rows(x, torch.tensor([2, 1, 0, 2, 1]), 3)
    assert ps._label_flag is None


def test_replay_feed_does_not_outlive_a_trainer_step():
    """A replay feed left unconsumed by a trainer step is dropped when the
    step ends (never served to later objective calls)."""
    ps = _variant("PSVILearnV", M=6, C=3)
    ps.replay_eps([torch.zeros(3), torch.ones(3)])
    with ps._outer_step():
        assert ps._eps_feed is not None
    assert ps._eps_feed is None


def test_plan_keys_carry_prior_sd():
    """Plans are cached per (family, layers, S, M, prior_sd): two models that
    differ only in prior_sd never share one (the soft-label outer plan too)."""
    import inspect

    from psvi.inference import psvi_classes as PC

    src = inspect.getsource(PC.PSVI._soft_psvi_elbo)
    assert '"soft-outer", fam, tuple(layers), S, R0 * C, model_spec(model)[2]' in src
    src = inspect.getsource(PC.PSVI._row_grad_fn)
    # the rows plan is built on first use inside the backward, not per objective
    assert src.index("def fn()") < src.index("self._new_plan(")
