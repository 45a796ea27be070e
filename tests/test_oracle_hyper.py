"""Pin the second-order oracle (inner_hvp, hyper_step in oracle/psvi_oracle.py)
against the reference's own double backward and PSVI.hyper_step
(tests/golden/h*.npz, y*.npz from tools/gen_golden_hyper.py; float64 reference
run, fp32 draws)."""
import numpy as np
import pytest

import psvi_oracle as O
from golden_util import fixture_names, l2rel, load_fixture, rel


def softmax_T(v, dw, N):
    e = np.exp(v - v.max())
    sm = e / e.sum()
    gs = N * dw
    return sm * (gs - (gs * sm).sum())


def test_hyper_fixture_set():
    assert {"h1_fn2_tiny", "h2_fn_deep", "h3_fn_shallow", "h4_logreg_fullcov"} <= \
        set(fixture_names("h"))
    assert {"y1_fn2_tiny", "y2_fn_deep"} <= set(fixture_names("y"))


@pytest.mark.parametrize("name", fixture_names("h"))
def test_hvp_oracle_matches_reference_double_backward(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    val, g, hv, du, dw = O.inner_hvp(cfg["family"], cfg["layers"], f["params0"], f["u"], f["z"],
                                     f["w"], f["eps"], cfg["S"], f["vec"], cfg["prior_sd"])
    assert rel(val, f["elbo"]) < 1e-10
    assert l2rel(g, f["grad"]) < 1e-9
    assert l2rel(hv, f["hv"]) < 1e-8
    assert l2rel(du, f["d_u"]) < 1e-8
    assert l2rel(softmax_T(f["v"].astype(np.float64), dw, cfg["N"]), f["d_v"]) < 1e-8


@pytest.mark.parametrize("name", fixture_names("y"))
def test_hyper_step_oracle_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    out = O.hyper_step(cfg["family"], cfg["layers"], f["params0"], f["u0"], f["z"], f["v0"],
                       cfg["N"], f["xb"], f["yb"], f["eps_inner"], f["eps_outer"], cfg["S"],
                       cfg["T"], cfg["K"], cfg["lr0net"], cfg["lr0u"], cfg["lr0v"],
                       cfg["linsys_lr"], approx=cfg.get("approx", "CG_normaleq"))
    assert l2rel(out["params"], f["params"]) < 1e-9
    assert l2rel(out["u_grad"], f["u_grad"]) < 1e-7
    assert l2rel(out["v_grad"], f["v_grad"]) < 1e-7
    assert l2rel(out["u"], f["u"]) < 1e-9 and l2rel(out["v"], f["v"]) < 1e-9
    assert rel(out["ll"], f["ll"]) < 1e-9


@pytest.mark.parametrize("name", fixture_names("n"))
def test_nested_step_oracle_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    out = O.nested_step(cfg["family"], cfg["layers"], f["params0"], f["u0"], f["z"], f["v0"],
                        cfg["N"], f["xb"], f["yb"], f["eps_inner"], f["eps_outer"], cfg["S"],
                        cfg["T"], cfg["lr0net"], cfg["lr0u"], cfg["lr0v"])
    assert rel(out["loss"], f["loss"]) < 1e-10
    assert l2rel(out["params"], f["params"]) < 1e-10
    assert l2rel(out["u_grad"], f["u_grad"]) < 1e-8, l2rel(out["u_grad"], f["u_grad"])
    assert l2rel(out["v_grad"], f["v_grad"]) < 1e-8
    assert l2rel(out["u"], f["u"]) < 1e-10 and l2rel(out["v"], f["v"]) < 1e-10
