"""Importance-weighted predictive evaluation on the HIP path (psvi_evaluate /
PSVI.evaluate / pred_on_grid) vs the reference's own PSVI.evaluate numbers
(tests/golden/e*.npz) and vs the float64 oracle at C3 size."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import family_of, fixture_names, l2rel, load_fixture, rel
from test_oracle_outer import eval_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(x, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(x), dtype=dtype, device=DEV)


@pytest.mark.parametrize("name", fixture_names("e"))
def test_psvi_evaluate_matches_reference(name):
    from psvi.inference import PSVIAV, PSVILearnV
    from test_host_api import build_model

    f = load_fixture(name)
    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    cls = PSVIAV if cfg["f"] == "exp_alpha_softmax" else PSVILearnV
    ps = cls(u=_t(f["u"]), z=_t(f["z"]), N=cfg["N"], model=model, mc_samples=cfg["S"],
             device_id=0)
    ps.device = torch.device(DEV)
    ps.v = _t(f["v"])
    if cls is PSVIAV:
        ps.alpha = _t([cfg["alpha"]])
    ps.test_loader = [(_t(f["xt"]), _t(f["yt"]))]
    for tag, corr in (("", True), ("_nc", False)):
        acc, nll, went, ness, vent = ps.evaluate(correction=corr, eps=[_t(f["eps" + tag])])
        Nt = cfg["Nt"]
        print(f"{name}{tag}: acc {acc.item():.4f} ({float(f['acc' + tag]):.4f}) nll {nll.item():.5f} "
              f"({float(f['nll' + tag]):.5f}) ness {ness.item():.4f} ({float(f['ness' + tag]):.4f})")
        assert abs(acc.item() - float(f["acc" + tag])) <= 1.0 / Nt + 1e-6  # argmax ties
        assert rel(nll.item(), f["nll" + tag]) < 1e-4
        assert abs(went.item() - float(f["went" + tag])) < 1e-4 * max(1.0, abs(float(f["went" + tag])))
        assert rel(ness.item(), f["ness" + tag]) < 1e-4
        assert rel(vent.item(), f["vent" + tag]) < 1e-6
    if cls is PSVIAV:
        assert len(ps.results["alpha"]) == 2


def test_evaluate_c3_vs_oracle():
    """C3 model (fn2 64-40-40-2, S=128) with 100 pseudopoints and 1000 test rows."""
    from psvi.runtime import InnerLoopPlan

    rng = np.random.default_rng(5)
    layers, S, M, Nt = [(64, 40), (40, 40), (40, 2)], 128, 100, 1000
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.15 * rng.standard_normal(n), rng.uniform(-5, -4, n),
                  2e-4 * rng.standard_normal((n - 1) * (n - 2) // 2)]
    params = np.concatenate(parts).astype(np.float32)
    eps = rng.standard_normal(S * 4322).astype(np.float32)
    X = rng.standard_normal((M + Nt, 64)).astype(np.float32)
    z = rng.integers(0, 2, M + Nt)
    w = np.concatenate([O.coreset_weights(0.1 * rng.standard_normal(M), 800), np.zeros(Nt)])
    plan = InnerLoopPlan("fullcov", layers, S, M + Nt)
    for corr in (True, False):
        st, pr = plan.evaluate(M, _t(X), _t(z.astype(np.int32), torch.int32), _t(w), _t(eps),
                               _t(params), correction=corr, probs=True)
        st = st.cpu().numpy()
        c, nll, ent, ness, probs = O.evaluate_batch("mvn", layers, params, X, z, w, M, eps, S,
                                                     corr)
        assert l2rel(pr.cpu().numpy(), probs) < 1e-4
        assert abs(st[2] - c) <= 3  # argmax near-ties may flip in fp32
        assert rel(st[3], nll) < 1e-4
        assert rel(st[1], ness) < 1e-4


def test_pred_on_grid_shape_and_normalisation():
    from psvi.inference import PSVILearnV
    from psvi.models import make_logreg

    torch.manual_seed(0)
    model = make_logreg(2, 3, mc_samples=8, init_sd=0.1).cuda()
    ps = PSVILearnV(u=torch.randn(9, 2, device=DEV), z=(torch.arange(9, device=DEV) % 3).float(),
                    N=800, model=model, mc_samples=8, device_id=0)
    ps.device = torch.device(DEV)
    p = ps.pred_on_grid(n_test_per_dim=40)
    assert p.shape == (1600, 3)
    assert torch.allclose(p.sum(-1), torch.ones(1600, device=DEV), atol=1e-5)


@pytest.mark.parametrize("name", fixture_names("p"))
def test_pred_on_grid_matches_reference(name):
    """PSVI.pred_on_grid through psvi_evaluate against the reference's own
    pred_on_grid (tests/golden/p*.npz, tools/gen_golden_grid.py), with and
    without the importance-weight correction (fp32 path against the float64
    reference run: 1e-5 absolute on probabilities)."""
    from psvi.inference import PSVIAV, PSVILearnV
    from test_host_api import build_model

    f = load_fixture(name)
    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    cls = PSVIAV if cfg["f"] == "exp_alpha_softmax" else PSVILearnV
    ps = cls(u=_t(f["u"]), z=_t(f["z"]), N=cfg["N"], model=model, mc_samples=cfg["S"],
             device_id=0)
    ps.device = torch.device(DEV)
    ps.v = _t(f["v"])
    if cls is PSVIAV:
        ps.alpha = _t([cfg["alpha"]])
    n = cfg["n_test_per_dim"]
    for tag, corr in (("", True), ("_nc", False)):
        p = ps.pred_on_grid(n_test_per_dim=n, correction=corr, eps=_t(f["eps" + tag]))
        ref = f["probs" + tag]
        assert p.shape == ref.shape
        err = float(np.abs(p.cpu().numpy() - ref).max())
        print(f"{name}{tag}: max |p - ref| {err:.2e}")
        assert err < 1e-5
