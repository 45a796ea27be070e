"""Sample-sharded outer objective: ShardedOuter's two passes
(psvi_outer_elbo_grad per-sample terms on each rank's own samples, then
psvi_outer_elbo_grad_coef with the global softmax coefficients) composed over
emulated ranks in one process, against the world-1 psvi_outer_elbo_grad and
the reference's own PSVI.psvi_elbo numbers (tests/golden/o*.npz).

Tolerance (north star): loss within 1e-5 relative of the reference, gradients
within 1e-4 relative; against world 1 only the fp32 summation order differs."""
import numpy as np
import pytest
import torch

from golden_util import (assert_grad_close, family_of, fixture_names, l2rel, load_fixture,
                         plan_layers, rel)
from test_hip_outer import _random_case, _run, _t
from test_oracle_outer import outer_inputs

pytestmark = pytest.mark.gpu


def _sharded(family, layers, S, X, z, w, n_pseudo, eps, params, world, prior_sd=1.0):
    from psvi.runtime.sharded import ShardedOuter, outer_coefficients

    args = (n_pseudo, _t(X), _t(z.astype(np.int32), torch.int32), _t(w))
    e, p = _t(eps), _t(params)
    ranks = [ShardedOuter(family, layers, S, X.shape[0], world, r, prior_sd=prior_sd)
             for r in range(world)]
    terms, el = [], []
    for so in ranks:                                  # pass 1 on every rank
        e_loc, t = so.local_terms(*args, e, p)
        terms.append(t)
        el.append(e_loc)
    loss, cp, cd, ck = outer_coefficients(torch.cat(terms))  # the all-reduced (S, 3)
    out = {"loss": loss.item()}
    for so, e_loc in zip(ranks, el):                  # pass 2 + the gradient all-reduce
        g = so.local_grads(*args, e_loc, p, cp, cd, ck)
        for k, v in g.items():
            out[k] = out.get(k, 0) + v.double().cpu().numpy()
    return out


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", fixture_names("o"))
def test_sharded_outer_matches_reference(name, world):
    f = load_fixture(name)
    cfg = f["cfg"]
    if cfg["S"] < world:
        pytest.skip("fewer samples than ranks")
    X, z, w, M = outer_inputs(f)
    fam, layers = family_of(cfg), plan_layers(cfg)
    out = _sharded(fam, layers, cfg["S"], X, z, w, M, f["eps"], f["params0"], world,
                   cfg["prior_sd"])
    _, one = _run(fam, layers, cfg["S"], X, z, w, M, f["eps"], f["params0"], cfg["prior_sd"])
    assert rel(out["loss"], f["loss"]) < 1e-5, (out["loss"], float(f["loss"]))
    assert rel(out["loss"], one["loss"][0]) < 1e-9
    assert_grad_close(out["grad"], f["grad_params"], what=name + " params")
    assert_grad_close(out["grad_u"].reshape(f["grad_u"].shape), f["grad_u"], what=name + " u")
    for k in ("grad", "grad_u", "grad_w"):
        assert l2rel(out[k].reshape(-1), one[k].reshape(-1)) < 1e-5, k


@pytest.mark.parametrize("case", [
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100, 128, 8),   # C4: C3 sharded 8 ways
    ("meanfield", [(2, 100), (100, 4)], 32, 50, 128, 5),            # ragged split (7,7,6,6,6)
    ("lenet", None, 16, 20, 12, 3),
])
def test_sharded_outer_fullsize(case):
    family, layers, S, M, Nx, world = case
    if family == "lenet":
        from golden_util import LENET_PLAN_LAYERS
        from psvi.models import make_lenet

        layers = LENET_PLAN_LAYERS
        torch.manual_seed(3)
        net = make_lenet(mc_samples=S, init_sd=0.05)
        params = torch.nn.utils.parameters_to_vector(net.parameters()).detach().numpy()
        rng = np.random.default_rng(5)
        from psvi.runtime import InnerLoopPlan

        n_eps = InnerLoopPlan(family, layers, S, M + Nx).eps_count
        eps = rng.standard_normal(n_eps).astype(np.float32)
        X = rng.standard_normal((M + Nx, 784)).astype(np.float32)
        z = rng.integers(0, 10, M + Nx)
        w = np.concatenate([np.full(M, 3.0), np.full(Nx, 60.0 / Nx)]).astype(np.float32)
    else:
        params, eps, X, z, w = _random_case(family, layers, S, M, Nx, seed=S + M)
    out = _sharded(family, layers, S, X, z, w, M, eps, params, world)
    _, one = _run(family, layers, S, X, z, w, M, eps, params)
    assert rel(out["loss"], one["loss"][0]) < 1e-9
    for k in ("grad", "grad_u", "grad_w"):
        assert l2rel(out[k].reshape(-1), one[k].reshape(-1)) < 1e-5, k


def test_coef_entry_validation():
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime._lib import PsviError

    f = load_fixture("o4_fn2_tiny")
    cfg = f["cfg"]
    X, z, w, M = outer_inputs(f)
    plan = InnerLoopPlan("fullcov", cfg["layers"], cfg["S"], X.shape[0])
    coef = torch.zeros(3 * cfg["S"] + 1, device="cuda")
    args = (_t(X), _t(z.astype(np.int32), torch.int32), _t(w), _t(f["eps"]), _t(f["params0"]))
    g = plan.outer_grad_coef(M, *args, coef)          # zero coefficients -> zero gradients
    torch.cuda.synchronize()
    assert all(float(v.abs().max()) == 0.0 for v in g.values())
    with pytest.raises(PsviError):
        plan.outer_grad_coef(X.shape[0] + 1, *args, coef)


class _ThreadComm:
    """all_reduce among threads standing in for ranks (the TorchDistComm API)."""

    def __init__(self, world):
        import threading

        self.slots = [None] * world
        self.bar = threading.Barrier(world)

    def bind(self, rank):
        outer = self

        class _Rank:
            def all_reduce(self, t):
                outer.slots[rank] = t.clone()
                outer.bar.wait()
                total = sum(outer.slots[r] for r in range(len(outer.slots)))
                outer.bar.wait()
                t.copy_(total)

        return _Rank()


def test_sharded_outer_elbo_grad_threads():
    """ShardedOuter.elbo_grad end to end with its collectives (ranks as threads)."""
    import threading

    from psvi.runtime.sharded import ShardedOuter

    f = load_fixture("o5_fn2_mid_av")
    cfg = f["cfg"]
    X, z, w, M = outer_inputs(f)
    fam, layers, world = family_of(cfg), plan_layers(cfg), 3
    args = (M, _t(X), _t(z.astype(np.int32), torch.int32), _t(w), _t(f["eps"]),
            _t(f["params0"]))
    comm = _ThreadComm(world)
    ranks = [ShardedOuter(fam, layers, cfg["S"], X.shape[0], world, r, cfg["prior_sd"],
                          comm=comm.bind(r)) for r in range(world)]
    res, errs = [None] * world, []

    def run(r):
        try:
            res[r] = ranks[r].elbo_grad(*args)
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not errs, errs
    _, one = _run(fam, layers, cfg["S"], X, z, w, M, f["eps"], f["params0"], cfg["prior_sd"])
    for r in range(world):
        assert rel(res[r]["loss"].item(), f["loss"]) < 1e-5
        for k in ("grad", "grad_u", "grad_w"):
            assert l2rel(res[r][k].cpu().numpy().reshape(-1), one[k].reshape(-1)) < 1e-5, k
