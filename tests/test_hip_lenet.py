"""LeNet (make_lenet, config C5) on the HIP path vs the reference fixtures and
the fp64 oracle (oracle/psvi_oracle.py lenet_*).

* l1 (higher Adam) / l2 (hypergrad Adam): the reference's own eps, ELBO per
  step, the step-1 gradient and the T-step Adam trajectory;
* oracle parity on random states at ragged sizes (M not a multiple of the
  image chunk, S odd);
* at C5's size (S=256, M=500): bitwise run-to-run determinism, and the
  sample-sharded phases (world 2) summing to the single-rank accumulator.
Tolerance (north star): ELBO and gradient within 1e-4 relative."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import adam_kind, assert_grad_close, fixture_names, l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
LENET = [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]


def _t(x, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(x), dtype=dtype, device=DEV)


def _plan(S, M, world=1, rank=0):
    from psvi.runtime import InnerLoopPlan

    return InnerLoopPlan("lenet", LENET, S, M, world=world, rank=rank)


def _random_state(rng, S, M):
    P = O.lenet_param_count()
    params = np.empty(P)
    po = 0
    for nw, nb, _, _ in O.LENET_LAYERS:
        n = nw + nb
        params[po:po + n] = 0.15 * rng.normal(size=n)
        params[po + n:po + 2 * n] = rng.uniform(-4.0, -2.0, size=n)
        po += 2 * n
    u = rng.normal(size=(M, 1, 28, 28))
    z = rng.integers(0, 10, size=M)
    w = rng.uniform(0.2, 3.0, size=M)
    eps = rng.normal(size=O.lenet_eps_count(S))
    return params.astype(np.float32), u.astype(np.float32), z, w.astype(np.float32), \
        eps.astype(np.float32)


@pytest.mark.parametrize("name", fixture_names("l"))
def test_lenet_fixture_elbo_grad_and_trajectory(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    S, M, T = cfg["S"], cfg["M"], cfg["T"]
    plan = _plan(S, M)
    assert plan.param_count == f["params0"].size and plan.eps_count == f["eps"].shape[1]
    u, z, w = _t(f["u"]), _t(f["z"].astype(np.int32), torch.int32), _t(f["w"])
    elbo, grad = plan.elbo_grad(u, z, w, _t(f["eps"][0]), _t(f["params0"]))
    val, g = O.lenet_elbo_grad(f["params0"], f["u"], f["z"], f["w"], f["eps"][0], S)
    assert rel(elbo.item(), val) < 1e-5 and rel(elbo.item(), f["elbo"][0]) < 1e-5
    assert_grad_close(grad.cpu().numpy(), g, what=name, ref_fp32=f["grad0"])
    params = _t(f["params0"])
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    elbos = plan.inner_loop(u, z, w, params, m, v, T, cfg["lr"], kind=adam_kind(cfg),
                            eps=_t(f["eps"]))
    o_elbo, _, o_traj, o_m, o_v = O.lenet_inner_loop(
        f["params0"], f["u"], f["z"], f["w"], f["eps"], S, cfg["lr"], adam_kind(cfg))
    assert rel(elbos.cpu().numpy(), o_elbo) < 1e-5
    assert rel(elbos.cpu().numpy(), f["elbo"]) < 1e-5
    p = params.cpu().numpy()
    assert np.abs(p - o_traj[-1]).max() < 0.5 * cfg["lr"]
    assert l2rel(p, o_traj[-1]) < 1e-5 and l2rel(p, f["params"][-1]) < 1e-5
    assert l2rel(m.cpu().numpy(), o_m) < 1e-3 and l2rel(v.cpu().numpy(), o_v) < 1e-3


@pytest.mark.parametrize("S,M", [(2, 1), (3, 7), (5, 37)])
def test_lenet_random_states_match_oracle(S, M):
    rng = np.random.default_rng(S * 100 + M)
    params, u, z, w, eps = _random_state(rng, S, M)
    plan = _plan(S, M)
    elbo, grad = plan.elbo_grad(_t(u), _t(z.astype(np.int32), torch.int32), _t(w), _t(eps),
                                _t(params))
    val, g = O.lenet_elbo_grad(params, u, z, w, eps, S)
    assert rel(elbo.item(), val) < 1e-5, (elbo.item(), val)
    assert_grad_close(grad.cpu().numpy(), g, what=f"S{S}M{M}")
    # without the KL term the conv and head gradients are the data term alone
    e0, g0 = plan.elbo_grad(_t(u), _t(z.astype(np.int32), torch.int32), _t(w), _t(eps),
                            _t(params), include_kl=False)
    assert e0.item() < elbo.item()
    n_conv = 2 * (156 + 2416)
    assert torch.equal(g0[:n_conv], grad[:n_conv])  # no KL on the conv layers


def _c5_inputs(S=256, M=500, seed=5):
    rng = np.random.default_rng(seed)
    params, u, z, w, _ = _random_state(rng, 2, M)
    from psvi.runtime import randn_

    eps = torch.empty(O.lenet_eps_count(S), device=DEV)
    randn_(eps, seed=seed, offset=0)
    return (_t(params), _t(u), _t(z.astype(np.int32), torch.int32), _t(w * 120.0), eps)


def test_lenet_c5_deterministic_and_finite():
    S, M = 256, 500
    params, u, z, w, eps = _c5_inputs(S, M)
    plan = _plan(S, M)
    e1, g1 = plan.elbo_grad(u, z, w, eps, params)
    e2, g2 = plan.elbo_grad(u, z, w, eps, params)
    assert torch.isfinite(g1).all() and np.isfinite(e1.item())
    assert torch.equal(g1, g2)  # fixed-order reductions; the nll sum is fp64
    assert rel(e1.item(), e2.item()) < 1e-12


def test_lenet_sample_sharded_phases_sum_to_single():
    """world 2: each rank accumulates [sum dW | sum dW eps] over its samples;
    their sum (the all-reduce) equals the single-rank accumulator."""
    S, M = 256, 500
    params, u, z, w, eps = _c5_inputs(S, M, seed=7)
    single = _plan(S, M)
    acc1 = torch.empty(single.acc_count, device=DEV)
    nll1 = torch.zeros(1, dtype=torch.float64, device=DEV)
    single.mf_accumulate(u, z, w, eps, params, acc1, nll1)
    acc2 = torch.zeros_like(acc1)
    nll2 = torch.zeros(1, dtype=torch.float64, device=DEV)
    for r in range(2):
        pr = _plan(S, M, world=2, rank=r)
        assert pr.s_local == S // 2 and pr.s_offset == r * (S // 2)
        a = torch.empty(pr.acc_count, device=DEV)
        pr.mf_accumulate(u, z, w, eps, params, a, nll2)
        acc2 += a
    assert rel(nll2.item(), nll1.item()) < 1e-6
    assert l2rel(acc2.cpu().numpy(), acc1.cpu().numpy()) < 1e-5
