"""Hessian-vector products on the HIP path (psvi_hvp through the C ABI) vs the
reference's own double backward (tests/golden/h*.npz) and vs the float64
R-op oracle at full size.  Tolerance: 1e-4 relative (l2), as the north star's
gradient bar; HIP fp32 vs float64."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import family_of, fixture_names, l2rel, load_fixture, plan_layers
from test_oracle_hyper import softmax_T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(x, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(x), dtype=dtype, device=DEV)


def _hvp(family, layers, S, u, z, w, eps, params, vec):
    """psvi_hvp with its mixed products, and H vec alone (mixed=False: for
    LeNet no d/du kernel after the tangent backward) -- both returned so each
    launch path is checked."""
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan(family, layers, S, u.shape[0])
    args = (_t(u), _t(z.astype(np.int32), torch.int32), _t(w), _t(eps), _t(params), _t(vec))
    hv, du, dw = plan.hvp(*args)
    hv0, du0, dw0 = plan.hvp(*args, mixed=False)
    assert du0 is None and dw0 is None
    torch.cuda.synchronize()
    return hv.cpu().numpy(), du.cpu().numpy(), dw.cpu().numpy(), hv0.cpu().numpy()


@pytest.mark.parametrize("name", fixture_names("h"))
def test_hvp_matches_reference_double_backward(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    hv, du, dw, hv0 = _hvp(family_of(cfg), plan_layers(cfg), cfg["S"], f["u"], f["z"], f["w"],
                           f["eps"], f["params0"], f["vec"])
    assert l2rel(hv, f["hv"]) < 1e-4, l2rel(hv, f["hv"])
    assert l2rel(hv0, f["hv"]) < 1e-4, l2rel(hv0, f["hv"])
    assert l2rel(du, f["d_u"]) < 1e-4, l2rel(du, f["d_u"])
    assert l2rel(softmax_T(f["v"].astype(np.float64), dw.astype(np.float64), cfg["N"]),
                 f["d_v"]) < 1e-4


@pytest.mark.parametrize("case", [
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100),   # C3
    ("meanfield", [(2, 100), (100, 4)], 32, 50),            # C2
    ("meanfield", [(5, 7), (7, 7), (7, 3)], 6, 70),         # row chunks
])
def test_hvp_fullsize_vs_oracle(case):
    family, layers, S, M = case
    rng = np.random.default_rng(S + M)
    fam = "mf" if family == "meanfield" else "mvn"
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.15 * rng.standard_normal(n), rng.uniform(-5, -4, n)]
        if fam == "mvn":
            parts += [2e-4 * rng.standard_normal((n - 1) * (n - 2) // 2)]
    params = np.concatenate(parts).astype(np.float32)
    eps_n = sum(S * (i * o + o) for i, o in layers)
    eps = rng.standard_normal(eps_n).astype(np.float32)
    u = rng.standard_normal((M, layers[0][0])).astype(np.float32)
    z = rng.integers(0, layers[-1][1], M)
    w = O.coreset_weights(0.2 * rng.standard_normal(M), 800, "softmax").astype(np.float32)
    vec = rng.standard_normal(params.size).astype(np.float32)
    hv, du, dw, hv0 = _hvp(family, layers, S, u, z, w, eps, params, vec)
    _, _, hv_o, du_o, dw_o = O.inner_hvp(fam, layers, params, u, z, w, eps, S, vec)
    assert l2rel(hv, hv_o) < 1e-4, l2rel(hv, hv_o)
    assert l2rel(hv0, hv_o) < 1e-4, l2rel(hv0, hv_o)
    assert l2rel(du, du_o) < 1e-4, l2rel(du, du_o)
    assert l2rel(dw, dw_o) < 1e-4, l2rel(dw, dw_o)




@pytest.mark.parametrize("family,layers,S,M", [
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100),   # C3: 50-row blocks
    ("fullcov", [(33, 17), (17, 5)], 6, 37),                # ragged: 19 / 18 rows, K not a 16-multiple
    ("fullcov", [(7, 5), (5, 3)], 4, 3),                    # 2 / 1 rows
    ("fullcov", [(33, 17), (17, 5)], 300, 11),              # three sample passes, the last ragged
    ("meanfield", [(2, 100), (100, 4)], 32, 50),            # C2
    ("meanfield", [(5, 7), (7, 7), (7, 3)], 6, 70),
])
def test_hvp_kernel_forms_agree(family, layers, S, M):
    """The matrix-core R-op (net_rop_mfma_kernel, the default where a row block
    fits the LDS) against the VALU kernel (PSVI_DBG_ROP_VALU A/B), and the
    full-cov J^T G_dot on the bf16-piece K-split kernel's gradient mode (the
    default) against the chunked fp32 kernel (PSVI_DBG_KSTREAM_OFF A/B), and
    the sample pair (x and its tangent) on the paired bf16-piece launch (the
    default) against the fp32 item grid (PSVI_DBG_FWD_PAIR_BF 0): H vec
    and both mixed products within 1e-5 relative (l2) -- fp32 sums in another
    order -- and the default result bitwise run to run."""
    from psvi.runtime import InnerLoopPlan

    rng = np.random.default_rng(S * 7 + M)
    fam = "mf" if family == "meanfield" else "mvn"
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.15 * rng.standard_normal(n), rng.uniform(-5, -4, n)]
        if fam == "mvn":
            parts += [2e-4 * rng.standard_normal((n - 1) * (n - 2) // 2)]
    params = np.concatenate(parts).astype(np.float32)
    eps = rng.standard_normal(sum(S * (i * o + o) for i, o in layers)).astype(np.float32)
    u = rng.standard_normal((M, layers[0][0])).astype(np.float32)
    z = rng.integers(0, layers[-1][1], M).astype(np.int32)
    w = (1.0 + rng.random(M)).astype(np.float32)
    vec = rng.standard_normal(params.size).astype(np.float32)
    plan = InnerLoopPlan(family, layers, S, M)
    args = (_t(u), _t(z, torch.int32), _t(w), _t(eps), _t(params), _t(vec))

    def run():
        return [t.cpu().numpy() for t in plan.hvp(*args)]

    a, b = run(), run()
    alt = []
    # the VALU R-op; the chunked gradient-mode update; (full-cov) the sample
    # pair on the fp32 item grid instead of the paired bf16-piece launch
    forms = [(29, 1, 0), (19, 1, 0)]
    if family == "fullcov":
        forms.append((31, 0, 1))
    for key, val, dflt in forms:
        plan.lib.psvi_debug_set(key, val)
        try:
            alt.append(run())
        finally:
            plan.lib.psvi_debug_set(key, dflt)
    for i, (x, y) in enumerate(zip(a, b)):
        assert np.isfinite(x).all()
        assert np.array_equal(x, y)
        for f, r in zip(forms, alt):
            assert l2rel(x, r[i]) < 1e-5, (f, l2rel(x, r[i]))
