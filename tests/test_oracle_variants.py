"""The float64 oracle's PSVI plugin variants (PSVIAV, PSVIFixedU, PSVIAFixedU,
PSVI_Ablated, PSVI_No_IW) against whole outer steps of the reference's own
classes (tests/golden/v*.npz, tools/gen_golden_variants.py)."""
import numpy as np
import pytest

import psvi_oracle as O
from golden_util import fixture_names, l2rel, load_fixture, rel

VARIANTS = {
    "PSVIAV": dict(f="exp_alpha_softmax"),
    "PSVIFixedU": dict(fixed_u=True),
    "PSVIAFixedU": dict(f="exp_alpha_softmax", fixed_u=True),
    "PSVI_Ablated": dict(outer="ablated"),
    "PSVI_No_IW": dict(outer="ablated", noiw=True),
}


def variant_of(cfg):
    kw = dict(VARIANTS[cfg["cls"]])
    kw["alpha"] = cfg.get("alpha0")
    kw["lr0alpha"] = cfg["lr0alpha"]
    return O.Variant(**kw)


def run_oracle(f):
    cfg = f["cfg"]
    var = variant_of(cfg)
    layers = [tuple(x) for x in cfg["layers"]]
    if cfg["trainer"] == "psvi_elbo":
        return O._outer(var, cfg["family"], layers, f["params0"], f["u0"].astype(np.float64),
                        f["z"], None, f["xb"], f["yb"], cfg["N"], f.get("eps_outer", [None])[0], cfg["S"],
                        cfg["prior_sd"])
    common = (cfg["family"], layers, f["params0"], f["u0"], f["z"], f["v0"], cfg["N"], f["xb"],
              f["yb"], f.get("eps_inner", []), f.get("eps_outer", []), cfg["S"], cfg["T"])
    if cfg["trainer"] == "nested":
        return O.nested_step(*common, cfg["lr0net"], cfg["lr0u"], cfg["lr0v"], variant=var)
    return O.hyper_step(*common, cfg["K"], cfg["lr0net"], cfg["lr0u"], cfg["lr0v"],
                        linsys_lr=cfg["linsys_lr"], approx=cfg["approx"], variant=var)


def test_variant_fixture_set():
    names = fixture_names("v")
    assert len(names) >= 14
    classes = {load_fixture(n)["cfg"]["cls"] for n in names}
    assert classes == set(VARIANTS)


@pytest.mark.parametrize("name", fixture_names("v"))
def test_oracle_variant_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    if "raises" in cfg:  # the reference's own failure, reproduced
        exc = {"IndexError": IndexError, "AttributeError": AttributeError}[cfg["raises"]]
        with pytest.raises(exc):
            run_oracle(f)
        return
    out = run_oracle(f)
    if cfg["trainer"] == "psvi_elbo":
        loss, g, gu, gw = out
        assert rel(loss, f["out"]) < 1e-9
        assert l2rel(g, f["grad_params"]) < 1e-8
        assert "u_grad" not in f or np.abs(f["u_grad"]).max() == 0
        return
    key = "loss" if cfg["trainer"] == "nested" else "ll"
    assert rel(out[key], f["out"]) < 1e-8, (out[key], float(f["out"]))
    assert l2rel(out["params"], f["params"]) < 1e-9
    for k in ("u_grad", "v_grad", "alpha_grad"):
        if k in f:
            assert l2rel(out[k], f[k]) < 1e-6, (k, l2rel(out[k], f[k]))
        elif k != "alpha_grad":
            assert out[k] is None, k  # u frozen: the reference leaves u.grad None
    assert l2rel(out["u"], f["u"]) < 1e-9
    assert l2rel(out["v"], f["v"]) < 1e-9
    if "alpha" in f:
        assert rel(out["alpha"], f["alpha"]) < 1e-9
        assert rel(out["alpha"], cfg["alpha0"]) > 0  # alpha moved (optim_alpha stepped)
    if cfg["cls"] in ("PSVIFixedU", "PSVIAFixedU"):
        assert np.array_equal(f["u"].astype(np.float32), f["u0"])
