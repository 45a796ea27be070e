"""MFVI baselines (run_mfvi / run_mfvi_subset, baselines.py:824-1062): the
oracle replays the reference's own runs (tools/gen_golden_mfvi.py, fixtures
b*): per-iteration ELBO, predictive accuracy and NLL."""
import numpy as np
import pytest

import psvi_oracle as O
from golden_util import fixture_names, load_fixture

NAMES = fixture_names("b")


def mfvi_layers(cfg):
    D, H, C = cfg["D"], cfg["n_hidden"], cfg["nc"]
    if cfg["arch"] in ("logistic_regression", "logistic_regression_fullcov"):
        return "mf" if cfg["arch"] == "logistic_regression" else "mvn", [(D, C)]
    fam = "mf" if cfg["arch"] == "fn" else "mvn"
    return fam, [(D, H), (H, H), (H, C)]   # make_fcnet / make_fc2net: 2 hidden layers


def subset(f, cfg):
    """pseudo_subsample_init (psvi/inference/utils.py:33-50) on the fixture's data."""
    import torch

    x, y = torch.tensor(f["x"]), torch.tensor(f["y"])
    torch.manual_seed(0)
    N = x.shape[0]
    us, zs, cnt = [], [], 0
    M, nc = cfg["num_pseudo"], cfg["nc"]
    for c in range(nc):
        idx = torch.arange(N)[y == c]
        k = M // nc if c < nc - 1 else M - cnt
        us.append(x[idx[torch.randperm(len(idx))[:k]]])
        zs.append(c * torch.ones(k))
        cnt += M // nc
    return torch.cat(us).numpy(), torch.cat(zs).numpy()


def test_mfvi_fixtures_present():
    assert {"b1_mfvi_fn", "b2_mfvi_fn2", "b3_mfvi_subset_logreg"} <= set(NAMES)


@pytest.mark.parametrize("name", NAMES)
def test_mfvi_oracle_replays_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    fam, layers = mfvi_layers(cfg)
    if cfg["fn"] == "run_mfvi":
        x, y, scale, last = f["x"], f["y"], 1.0, True
    else:
        x, y = subset(f, cfg)
        scale, last = cfg["n_train"] / cfg["num_pseudo"], False
    elbos, accs, nlls, _ = O.mfvi_run(fam, layers, f["params0"], x, y, f["xt"], f["yt"],
                                      f["draws"], cfg["S"], cfg["iters"], cfg["log_every"],
                                      cfg["lr"], scale, eval_last=last)
    assert np.allclose(elbos, f["elbos"], rtol=1e-5), (elbos, f["elbos"])
    assert np.array_equal(np.round(accs * len(f["yt"])), np.round(f["accs"] * len(f["yt"])))
    assert np.allclose(nlls, f["nlls"], rtol=1e-5)


@pytest.mark.parametrize("name", NAMES)
def test_host_set_up_model_reproduces_reference_init(name):
    """run_mfvi seeds torch and builds the model first (baselines.py:853-857):
    the host set_up_model gives the reference's initial parameters."""
    import random

    import torch

    from psvi.inference.baselines import set_up_model

    f = load_fixture(name)
    cfg = f["cfg"]
    random.seed(0), np.random.seed(0), torch.manual_seed(0)
    net = set_up_model(architecture=cfg["arch"], D=cfg["D"], n_hidden=cfg["n_hidden"],
                       nc=cfg["nc"], mc_samples=cfg["S"], init_sd=cfg["init_sd"])
    p = torch.nn.utils.parameters_to_vector(net.parameters()).detach().numpy()
    assert np.array_equal(p, f["params0"])


def test_host_subset_init_matches_oracle_helper():
    import torch

    from psvi.inference.baselines import pseudo_subsample_init

    f = load_fixture("b3_mfvi_subset_logreg")
    cfg = f["cfg"]
    u, z = pseudo_subsample_init(torch.tensor(f["x"]), torch.tensor(f["y"]),
                                 num_pseudo=cfg["num_pseudo"], nc=cfg["nc"], seed=0)
    u2, z2 = subset(f, cfg)
    assert np.array_equal(u.detach().numpy(), u2) and np.array_equal(z.numpy(), z2)


def test_mfvi_without_device_raises():
    import torch

    from psvi.inference.baselines import run_mfvi

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="HIP device"):
        run_mfvi(architecture="fn", D=2, n_hidden=4, nc=2)
