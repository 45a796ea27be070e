"""Outer objective on the HIP path (psvi_outer_elbo_grad through the C ABI) vs
the reference's own PSVI.psvi_elbo numbers (tests/golden/o*.npz, float64
reference run with fp32 draws) and vs the float64 oracle at full size.

Tolerance (north star): loss and gradients within 1e-4 relative."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import (assert_grad_close, family_of, fixture_names, l2rel, load_fixture,
                         plan_layers, rel)
from test_oracle_outer import f_jacobian_T, outer_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(x, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(x), dtype=dtype, device=DEV)


def _run(family, layers, S, X, z, w, n_pseudo, eps, params, prior_sd=1.0):
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan(family, layers, S, X.shape[0], prior_sd=prior_sd)
    out = plan.outer_elbo_grad(n_pseudo, _t(X), _t(z.astype(np.int32), torch.int32), _t(w),
                               _t(eps), _t(params), sample_stats=True)
    torch.cuda.synchronize()
    return plan, {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("name", fixture_names("o"))
def test_outer_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    X, z, w, M = outer_inputs(f)
    _, out = _run(family_of(cfg), plan_layers(cfg), cfg["S"], X, z, w, M, f["eps"],
                  f["params0"], cfg["prior_sd"])
    assert rel(out["loss"][0], f["loss"]) < 1e-5, (out["loss"][0], float(f["loss"]))
    assert_grad_close(out["grad"], f["grad_params"], what=name + " params")
    assert_grad_close(out["grad_u"].reshape(f["grad_u"].shape), f["grad_u"], what=name + " u")
    gv, ga = f_jacobian_T(cfg, f["v"], out["grad_w"].astype(np.float64), cfg.get("alpha"))
    assert l2rel(gv, f["grad_v"]) < 1e-4
    if cfg["f"] == "exp_alpha_softmax":
        assert rel(ga, f["grad_alpha"]) < 1e-4
    W = out["samples"][:, 3]
    assert abs(W.sum() - 1.0) < 1e-9 and (W >= 0).all()


def _random_case(family, layers, S, M, Nx, seed, N=800, mu=0.15, rho=(-5.0, -4.0), corr=2e-4):
    rng = np.random.default_rng(seed)
    D, C = layers[0][0], layers[-1][1]
    parts, eps = [], []
    for din, dout in layers:
        n = din * dout + dout
        if family == "meanfield":
            parts += [mu * rng.standard_normal(n), rng.uniform(*rho, n)]
            eps += [rng.standard_normal(S * n)]
        else:
            nc = (n - 1) * (n - 2) // 2
            parts += [mu * rng.standard_normal(n), rng.uniform(*rho, n),
                      corr * rng.standard_normal(nc)]
            eps += [rng.standard_normal(S * n)]
    params = np.concatenate(parts).astype(np.float32)
    eps = np.concatenate(eps).astype(np.float32)
    X = rng.standard_normal((M + Nx, D)).astype(np.float32)
    z = rng.integers(0, C, M + Nx)
    v = 0.2 * rng.standard_normal(M)
    w = np.concatenate([O.coreset_weights(v, N, "softmax"), np.full(Nx, N / Nx)])
    return params, eps, X, z, w


@pytest.mark.parametrize("case", [
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100, 128),   # C3 (+ a 128-row data batch)
    ("meanfield", [(2, 100), (100, 4)], 32, 50, 128),            # C2
    ("fullcov", [(16, 8), (8, 8), (8, 2)], 16, 300, 200),        # pseudopoint chunks
])
def test_outer_fullsize_vs_oracle(case):
    family, layers, S, M, Nx = case
    params, eps, X, z, w = _random_case(family, layers, S, M, Nx, seed=S + M)
    _, out = _run(family, layers, S, X, z, w, M, eps, params)
    fam = "mf" if family == "meanfield" else "mvn"
    loss, gp, gu, gw = O.outer_elbo_grad(fam, layers, params, X, z, w, M, eps, S)
    assert rel(out["loss"][0], loss) < 1e-4, (out["loss"][0], loss)
    assert l2rel(out["grad"], gp) < 1e-4
    assert l2rel(out["grad_u"], gu) < 1e-4
    assert l2rel(out["grad_w"], gw) < 1e-4


def test_outer_value_only_and_validation():
    f = load_fixture("o4_fn2_tiny")
    cfg = f["cfg"]
    X, z, w, M = outer_inputs(f)
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime._lib import PsviError

    plan = InnerLoopPlan("fullcov", cfg["layers"], cfg["S"], X.shape[0])
    out = plan.outer_elbo_grad(M, _t(X), _t(z.astype(np.int32), torch.int32), _t(w),
                               _t(f["eps"]), _t(f["params0"]), grad=False, grad_w=False)
    assert set(out) == {"loss"}
    assert rel(out["loss"].item(), f["loss"]) < 1e-5
    with pytest.raises(PsviError):
        plan.outer_elbo_grad(X.shape[0] + 1, _t(X), _t(z.astype(np.int32), torch.int32),
                             _t(w), _t(f["eps"]), _t(f["params0"]))
