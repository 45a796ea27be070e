"""Pin the LeNet oracle (oracle/psvi_oracle.py, lenet_*) against the reference's
own make_lenet inner loop (tools/gen_golden.py, fixtures l*): ELBO, gradient
and the Adam trajectory; plus a finite-difference check of the hand-derived
conv / pool backward at a size the reference fixtures do not cover."""
import numpy as np
import pytest

import psvi_oracle as O
from golden_util import adam_kind, assert_grad_close, fixture_names, l2rel, load_fixture, rel

NAMES = fixture_names("l")


def test_lenet_fixtures_present():
    assert {"l1_lenet_tiny", "l2_lenet_hyper"} <= set(NAMES)


def test_lenet_layout_counts():
    assert O.lenet_param_count() == 123_412          # SURVEY K13 (C5 P)
    assert O.lenet_eps_count(256) == 256 * 60_856 + 850
    for name in NAMES:
        f = load_fixture(name)
        assert f["params0"].size == O.lenet_param_count()
        assert f["eps"].shape[1] == O.lenet_eps_count(f["cfg"]["S"])


@pytest.mark.parametrize("name", NAMES)
def test_lenet_oracle_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    elbos, grads, traj, m, v = O.lenet_inner_loop(
        f["params0"], f["u"], f["z"], f["w"], f["eps"], cfg["S"], cfg["lr"], adam_kind(cfg))
    assert rel(elbos, f["elbo"]) < 1e-6, (elbos, f["elbo"])
    assert_grad_close(grads[0], f["grad0"], l2tol=1e-4, atol_frac=1e-3, what=name)
    p = np.array(traj)
    assert np.abs(p - f["params"]).max() < 0.3 * cfg["lr"]
    assert l2rel(p, f["params"]) < 1e-5
    assert l2rel(m, f["adam_m"]) < 2e-4 and l2rel(v, f["adam_v"]) < 2e-4


def test_lenet_gradient_finite_difference():
    """Central differences on a random subset of every layer's mu / rho
    (S=2, M=2, an all-positive and a mixed-sign input)."""
    rng = np.random.default_rng(3)
    S, M = 2, 2
    P = O.lenet_param_count()
    params = np.empty(P)
    po = 0
    for nw, nb, _, _ in O.LENET_LAYERS:
        n = nw + nb
        params[po:po + n] = 0.2 * rng.normal(size=n)
        params[po + n:po + 2 * n] = rng.uniform(-3.5, -2.0, size=n)
        po += 2 * n
    u = np.stack([np.abs(rng.normal(size=(1, 28, 28))), rng.normal(size=(1, 28, 28))])
    z = np.array([3.0, 8.0])
    w = np.array([2.5, 0.7])
    eps = rng.normal(size=O.lenet_eps_count(S))
    val, g = O.lenet_elbo_grad(params, u, z, w, eps, S)
    po = 0
    h = 1e-5
    for nw, nb, _, _ in O.LENET_LAYERS:
        n = nw + nb
        for base in (po, po + n):
            for i in rng.choice(n, size=4, replace=False):
                e = np.zeros(P)
                e[base + i] = h
                fp, _ = O.lenet_elbo_grad(params + e, u, z, w, eps, S)
                fm, _ = O.lenet_elbo_grad(params - e, u, z, w, eps, S)
                fd = (fp - fm) / (2 * h)
                assert abs(fd - g[base + i]) <= 1e-5 * max(1.0, abs(fd)), (base, i, fd, g[base + i])
        po += 2 * n


def test_route_margins_flag_the_c5_tie_row():
    """golden_util.lenet_route_margins (the C5 d/du outlier check): pseudo-image
    153 of the C5 rank case sits on a conv1 max-pool tie (relative gap ~1e-7:
    fp32 and fp64 can pick different window positions); typical rows sit
    orders of magnitude further from any tie or kink."""
    from golden_util import c5_lenet_case, lenet_route_margins

    m = lenet_route_margins(c5_lenet_case(), [153, 0, 1, 10, 499])
    assert m[0] < 1e-6
    assert (m[1:] > 1e-6).all(), m
