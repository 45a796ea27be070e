"""Fixture loading + comparison helpers shared by the parity tests."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names(prefix="g"):
    """Inner-loop fixtures (tools/gen_golden.py) start with "g", outer-objective
    fixtures (tools/gen_golden_outer.py) with "o"."""
    return sorted(os.path.basename(f)[:-4]
                  for f in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load_fixture(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    cfg = json.loads(str(d["config"]))
    if "layers" in cfg:
        cfg["layers"] = [tuple(x) for x in cfg["layers"]]
    out = {k: d[k] for k in d.files if k != "config"}
    out["cfg"] = cfg
    return out


def family_of(cfg):
    return {"mf": "meanfield", "mvn": "fullcov", "lenet": "lenet"}[cfg["family"]]


LENET_PLAN_LAYERS = [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]


def plan_layers(cfg):
    """The InnerLoopPlan layer table of a fixture (LeNet fixtures list only
    their VILinear layers in cfg["layers"])."""
    return LENET_PLAN_LAYERS if cfg["family"] == "lenet" else cfg["layers"]


def adam_kind(cfg):
    return "higher" if cfg["adam"] == "higher" else "hypergrad"


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def l2rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def assert_grad_close(g, gref, l2tol=1e-4, rtol=1e-3, atol_frac=1e-4, what="grad",
                      ref_fp32=None):
    """north-star tolerance: gradient within 1e-4 relative (l2), and every
    element within rtol plus atol_frac of the largest gradient entry -- or, where
    the reference's own fp32 gradient (ref_fp32) deviates more from the fp64
    oracle (sums of cancelling terms), within four times that deviation."""
    g = np.asarray(g, np.float64)
    gref = np.asarray(gref, np.float64)
    e = l2rel(g, gref)
    assert e <= l2tol, f"{what}: l2-relative error {e:.3e} > {l2tol:.0e}"
    tol = rtol * np.abs(gref) + atol_frac * np.abs(gref).max()
    if ref_fp32 is not None:
        tol = np.maximum(tol, 4.0 * np.abs(np.asarray(ref_fp32, np.float64) - gref))
    bad = np.abs(g - gref) > tol
    assert not bad.any(), (f"{what}: {int(bad.sum())} elements out of tolerance, "
                           f"worst idx {int(np.argmax(np.abs(g - gref)))}")


# ---------------------------------------------------------------------------
# C5 (make_lenet, S = 256, M = 500) parity case: one rank's share of a world-8
# sample split, regenerated from a seed (the oracle's outputs are the fixture
# tests/golden/c5_lenet_rank.npz, tools/gen_oracle_c5.py)
C5 = dict(S=256, M=500, world=8, rank=3, Nx=64, N=60000, seed=2026)


def c5_lenet_case(seed=C5["seed"]):
    """Seeded C5 inputs: params at a trained-like scale, M MNIST-shaped
    pseudo-images with coreset weights N f(v), a data batch of Nx rows, the
    rank's noise (its S / world samples per batched layer, plus the shared
    last-layer draw), outer coefficients and an HVP direction."""
    import psvi_oracle as O

    rng = np.random.default_rng(seed)
    S, M, Nx = C5["S"], C5["M"], C5["Nx"]
    s_cnt = S // C5["world"]
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
    v = rng.normal(size=M)
    w = C5["N"] * np.exp(v) / np.exp(v).sum()
    xb = rng.normal(size=(Nx, 1, 28, 28))
    yb = rng.integers(0, 10, size=Nx)
    eps_loc = rng.normal(size=O.lenet_eps_count(s_cnt))
    # coefficients of the form outer_coefficients produces: W_s the softmax
    # weight (this rank holds 32 of 256 samples: sum ~ 1/8), ck_s = W_s (a_s -
    # abar) - 1/S, cp_s = -W_s - ck_s, cd_s = W_s
    r = rng.normal(size=(3, s_cnt))
    W = np.exp(0.3 * r[0])
    W /= 8.0 * W.sum()
    ck = W * r[1] - 1.0 / S
    coef = np.stack([-W - ck, W, ck])
    vec = rng.normal(size=P) * 1e-2
    f32 = lambda a: np.asarray(a, np.float32)
    return dict(params=f32(params), u=f32(u), z=z.astype(np.int32), w=f32(w), xb=f32(xb),
                yb=yb.astype(np.int32), eps_loc=f32(eps_loc), cp=coef[0], cd=coef[1],
                ck=coef[2], vec=f32(vec), s_cnt=s_cnt, s_off=C5["rank"] * s_cnt)


def c5_global_eps(case, fill=np.nan):
    """The global (S = 256) eps in the reference draw order with the rank's
    samples (and the shared last-layer draw) from the case and every other
    sample's noise = fill: a plan that reads outside its shard sees NaN."""
    import psvi_oracle as O

    S, s_off, s_cnt = C5["S"], case["s_off"], case["s_cnt"]
    out = np.full(O.lenet_eps_count(S), fill, np.float32)
    go = lo = 0
    for nw, nb, bat, _ in O.LENET_LAYERS:
        if not bat:
            out[go:go + nw + nb] = case["eps_loc"][lo:lo + nw + nb]
            go += nw + nb
            lo += nw + nb
            continue
        for k in (nw, nb):
            g = out[go:go + S * k].reshape(S, k)
            g[s_off:s_off + s_cnt] = case["eps_loc"][lo:lo + s_cnt * k].reshape(s_cnt, k)
            go += S * k
            lo += s_cnt * k
    assert go == out.size and lo == case["eps_loc"].size
    return out


def lenet_route_margins(case, rows, S=None):
    """Smallest route margin of each pseudo-image row over the case's samples
    (float64 forward of the oracle, psvi_oracle.lenet_forward): per conv layer
    the gap between a max-pool window's two largest relu'd values (a pool tie)
    and the magnitude of the window's maximum pre-activation (the relu kink),
    and per hidden linear layer the pre-activations' magnitude -- each relative
    to the layer's mean |pre-activation|.  A row whose margin is at fp32's
    rounding reach (~1e-6) can route its gradient differently in fp32 and fp64
    (another window position, or a unit on the other side of the kink)."""
    import psvi_oracle as O

    S = case["s_cnt"] if S is None else S
    rows = list(rows)
    Xl = O.lenet_sample(case["params"], case["eps_loc"], S)
    u = np.asarray(case["u"], np.float64).reshape(-1, 1, 28, 28)[rows]
    _, cache = O.lenet_forward(Xl, u, S)
    a1 = O._conv(cache["x0"], cache["W1"], Xl[0]["X"][:, 150:], 2)
    a2 = O._conv(cache["p1"], cache["W2"], Xl[1]["X"][:, 2400:], 0)
    best = np.full(len(rows), np.inf)
    for a in (a1, a2):
        s_, m_, c_, h_, w_ = a.shape
        win = a.reshape(s_, m_, c_, h_ // 2, 2, w_ // 2, 2).transpose(0, 1, 2, 3, 5, 4, 6)
        win = win.reshape(s_, m_, -1, 4)
        srt = np.sort(np.maximum(win, 0.0), -1)
        scale = np.abs(a).mean()
        tie = np.where(srt[..., 3] > 0, srt[..., 3] - srt[..., 2], np.inf) / scale
        kink = np.abs(np.sort(win, -1)[..., 3]) / scale
        best = np.minimum(best, np.minimum(tie, kink).min(axis=(0, 2)))
    hs = cache["hs"]
    for l, off in ((0, 48000), (1, 10080)):
        a = np.einsum("smi,soi->smo", hs[l], cache["Wf"][l]) + Xl[2 + l]["X"][:, off:][:, None, :]
        best = np.minimum(best, (np.abs(a) / np.abs(a).mean()).min(axis=(0, 2)))
    return best
