"""The K-split streaming update (mvn_kstream_kernel): the full-cov Adam update
at K = S > 128 -- every rank of the row-sharded step (a rank's rows take all S
samples) and C4 on one GPU.  Checked, on seeded synthetic G / eps / state,
against the float64 oracle's update phase (psvi_oracle.mvn_grad_from_G + the
reference's Adam: psvi/models/neural_net.py:452-476 reparameterisation
gradient, robust_higher/optim.py:339-367 / hypergrad/diff_optimizers.py:
197-213 Adam), against the chunked kernel (PSVI_DBG_KSTREAM_OFF A/B), and for
run-to-run bitwise reproducibility: a split tile's partials are added in pass
order whichever contributor arrives last.  The default kernel forms dL from
bf16 pieces (fp32-faithful); its errors are held within twice those of the fp32
MFMA kernel (PSVI_DBG_KSTREAM_BF_OFF A/B).  Tolerances: parameters and Adam
state within 1e-6 relative (l2) of the oracle -- fp32 summation over K = S
samples of an fp64 reference; the Adam moments, which carry the gradient's
summation error unscaled, within 1e-5 -- and likewise of the chunked kernel."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import l2rel, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
FN2 = [(64, 40), (40, 40), (40, 2)]


def _state(layers, S, seed):
    rng = np.random.default_rng(seed)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
                  (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
    p = np.concatenate(parts).astype(np.float32)
    m = (1e-3 * rng.standard_normal(p.size)).astype(np.float32)
    v = (1e-6 * rng.random(p.size)).astype(np.float32)
    n_tot = sum(i * o + o for i, o in layers)
    G = (0.05 * rng.standard_normal((S, n_tot))).astype(np.float32)
    eps = rng.standard_normal(S * n_tot).astype(np.float32)
    return p, m, v, G, eps


def _run(plan, G_full, eps, p, m, v, step, kind, info, ks_off=0, bf_off=0):
    """One update phase of this plan's rank: g_shard = the rank's columns of
    G_full in x-shard order; returns (params, m, v, kl) as numpy."""
    from psvi.runtime.sharded import layer_rows

    t = lambda x: torch.tensor(x, dtype=torch.float32, device=DEV)
    woff = np.concatenate([[0], np.cumsum([i * o + o for i, o in plan.layers])]).astype(int)
    S = plan.S
    gs = np.zeros((S, info["rows"]), np.float32)
    for l in range(len(plan.layers)):
        rows, cols = layer_rows(info, l)
        gs[:, cols] = G_full[:, woff[l] + rows]
    pd, md, vd = t(p), t(m), t(v)
    kl = torch.zeros(1, dtype=torch.float64, device=DEV)
    plan.lib.psvi_debug_set(19, ks_off)
    plan.lib.psvi_debug_set(27, bf_off)
    try:
        plan.mvn_update(t(eps), t(gs.ravel()), pd, md, vd, step=step, lr=1e-3, kind=kind, kl_out=kl)
        torch.cuda.synchronize()
    finally:
        plan.lib.psvi_debug_set(19, 0)
        plan.lib.psvi_debug_set(27, 0)
    return pd.cpu().numpy(), md.cpu().numpy(), vd.cpu().numpy(), kl.item()


def _owned(plan, info):
    po, mask = 0, np.zeros(plan.param_count, bool)
    offs = [0]
    for din, dout in plan.layers:
        n = din * dout + dout
        offs.append(offs[-1] + 2 * n + (n - 1) * (n - 2) // 2)
    for (l, lo, cnt, _) in info["runs"]:
        din, dout = plan.layers[l]
        n = din * dout + dout
        hi = lo + cnt
        o = offs[l]
        mask[o + lo:o + hi] = True
        mask[o + n + lo:o + n + hi] = True
        clo, chi = min(lo, n - 1), min(hi, n - 1)
        mask[o + 2 * n + clo * (clo - 1) // 2:o + 2 * n + chi * (chi - 1) // 2] = True
    return mask


@pytest.mark.parametrize("W,S,kind", [(1, 256, "higher"), (1, 1024, "hypergrad"), (1, 300, "higher"),
                                      (8, 1024, "higher"), (4, 512, "hypergrad"), (2, 256, "higher")])
def test_kstream_update_matches_oracle_and_chunked(W, S, kind):
    from psvi.runtime import InnerLoopPlan

    p, m, v, G, eps = _state(FN2, S, 7 + W + S)
    step = 3
    g = O.mvn_grad_from_G(FN2, p, G, eps, S)
    pn_o, mn_o, vn_o = O.adam(kind, p.astype(np.float64), g, m.astype(np.float64),
                              v.astype(np.float64), step, 1e-3)
    ranks = range(W) if W <= 2 else (0, W // 2, W - 1)
    for r in ranks:
        plan = InnerLoopPlan("fullcov", FN2, S, 100, world=W, rank=r)
        info = plan.shard_info(r)
        own = _owned(plan, info)
        a = _run(plan, G, eps, p, m, v, step, kind, info)
        b = _run(plan, G, eps, p, m, v, step, kind, info)
        c = _run(plan, G, eps, p, m, v, step, kind, info, ks_off=1)
        f = _run(plan, G, eps, p, m, v, step, kind, info, bf_off=1)
        for x, y in zip(a[:3], b[:3]):   # bitwise run to run
            assert np.array_equal(x, y)
        for x, xf, ref, nm, tol in zip(a[:3], f[:3], (pn_o, mn_o, vn_o), ("params", "m", "v"),
                                       (1e-6, 1e-5, 1e-5)):
            e_bf = l2rel(x[own], ref[own])
            assert e_bf < tol, (W, r, nm, e_bf)
            assert np.array_equal(x[~own], (p, m, v)[("params", "m", "v").index(nm)][~own])
            # the default bf16-piece dL against the fp32 kernel (PSVI_DBG_KSTREAM_BF_OFF):
            # each held to the oracle, the bf16-piece error within twice the fp32 one
            assert e_bf <= 2 * l2rel(xf[own], ref[own]) + 1e-7, (W, r, nm, e_bf)
        for x, y, nm, tol in zip(a[:3], c[:3], ("params", "m", "v"), (1e-6, 1e-5, 1e-5)):
            assert l2rel(x[own], y[own]) < tol, (W, r, nm)
        assert rel(a[3], c[3]) < 1e-6


def test_kstream_world8_ranks_cover_the_update():
    """The 8 ranks' K-split updates, each applied to its own rows, assemble the
    world-1 K-split update of all rows (same G, eps, state)."""
    from psvi.runtime import InnerLoopPlan

    S, W = 1024, 8
    p, m, v, G, eps = _state(FN2, S, 99)
    one = InnerLoopPlan("fullcov", FN2, S, 100)
    a1 = _run(one, G, eps, p, m, v, 2, "higher", one.shard_info(0))
    full = [np.zeros_like(p) for _ in range(3)]
    cover = np.zeros(p.size, int)
    kl = 0.0
    for r in range(W):
        plan = InnerLoopPlan("fullcov", FN2, S, 100, world=W, rank=r)
        info = plan.shard_info(r)
        own = _owned(plan, info)
        res = _run(plan, G, eps, p, m, v, 2, "higher", info)
        for k in range(3):
            full[k][own] = res[k][own]
        cover += own
        kl += res[3]
    assert (cover == 1).all()
    for k, tol in zip(range(3), (1e-6, 1e-5, 1e-5)):
        assert l2rel(full[k], a1[k]) < tol
    assert rel(kl, a1[3]) < 1e-6


@pytest.mark.parametrize("W,S", [(1, 1024), (1, 300), (8, 1024), (3, 257), (2, 256)])
def test_segmented_sample_matches_oracle(W, S):
    """The segmented sample (mvn_fwd_seg_kernel + the (row block, pass) reduce,
    K = S > 128): each rank's rows of x = mean + L eps for all S samples against
    the float64 oracle (1e-6 relative, l2) and against the item-grid kernel
    (PSVI_DBG_FWD_SEG_OFF A/B) and the fp32 segmented kernel
    (PSVI_DBG_FWD_SEG_BF_OFF A/B: the default is the bf16-piece one); ragged S
    leaves a partial last pass."""
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime.sharded import layer_rows

    p, _, _, _, eps = _state(FN2, S, 11 + W + S)
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=DEV)
    dp, de = t(p), t(eps)
    woff = np.concatenate([[0], np.cumsum([i * o + o for i, o in FN2])]).astype(int)
    Xo = np.zeros((S, woff[-1]))
    po = eo = 0
    for l, (din, dout) in enumerate(FN2):
        n = din * dout + dout
        nc = (n - 1) * (n - 2) // 2
        L = O.mvn_dense_L(p[po + n:po + 2 * n], p[po + 2 * n:po + 2 * n + nc], n)
        E = eps[eo:eo + S * n].reshape(S, n).astype(np.float64)
        Xo[:, woff[l]:woff[l + 1]] = p[po:po + n][None].astype(np.float64) + E @ L.T
        po += 2 * n + nc
        eo += S * n
    ranks = range(W) if W <= 3 else (0, W - 1)
    for r in ranks:
        plan = InnerLoopPlan("fullcov", FN2, S, 100, world=W, rank=r)
        info = plan.shard_info(r)
        xs = torch.full((plan.xshard_count,), float("nan"), device=DEV)
        plan.mvn_sample(de, dp, xs)
        xa = xs.clone()
        plan.lib.psvi_debug_set(22, 1)
        try:
            xs.fill_(float("nan"))
            plan.mvn_sample(de, dp, xs)
            torch.cuda.synchronize()
        finally:
            plan.lib.psvi_debug_set(22, 0)
        xf = xs.clone()
        plan.lib.psvi_debug_set(26, 1)
        try:
            xf.fill_(float("nan"))
            plan.mvn_sample(de, dp, xf)
            torch.cuda.synchronize()
        finally:
            plan.lib.psvi_debug_set(26, 0)
        X = xa.view(S, -1).cpu().numpy().astype(np.float64)
        Xb = xs.view(S, -1).cpu().numpy().astype(np.float64)
        Xf = xf.view(S, -1).cpu().numpy().astype(np.float64)
        assert np.isfinite(X).all()
        assert l2rel(X, Xb) < 1e-6
        assert l2rel(X, Xf) < 1e-6
        for l in range(len(FN2)):
            rows, cols = layer_rows(info, l)
            if len(rows):
                e_bf = l2rel(X[:, cols], Xo[:, woff[l] + rows])
                assert e_bf < 1e-6, (W, r, l)
                # fp32-faithful: the bf16-piece error within twice the fp32 kernel's
                assert e_bf <= 2 * l2rel(Xf[:, cols], Xo[:, woff[l] + rows]) + 1e-8, (W, r, l)
