"""HIP path (libpsvi_hip.so through its C ABI) vs the CPU oracle.

* every golden fixture: T = 3 fused inner steps with the reference's own eps
  (ELBO per step, Adam trajectory) and the step-1 gradient via psvi_elbo_grad;
* world = 1 phase API == fused step;
* world = 2, 3 sharded phases, exchanged in-process on one GPU == world = 1.
Tolerance (north star): ELBO and gradient within 1e-4 relative; HIP fp32 vs
oracle fp64."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import (adam_kind, assert_grad_close, family_of, fixture_names, l2rel, plan_layers,
                         load_fixture, rel)

pytestmark = pytest.mark.gpu
NAMES = fixture_names()
DEV = "cuda"


def _t(x, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(x), dtype=dtype, device=DEV)


def _setup(f):
    from psvi.runtime import InnerLoopPlan

    cfg = f["cfg"]
    plan = InnerLoopPlan(family_of(cfg), cfg["layers"], cfg["S"], cfg["M"])
    u, z, w = _t(f["u"]), _t(f["z"].astype(np.int32), torch.int32), _t(f["w"])
    return cfg, plan, u, z, w


@pytest.mark.parametrize("name", NAMES)
def test_elbo_grad_matches_oracle(name):
    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    elbo, grad = plan.elbo_grad(u, z, w, _t(f["eps"][0]), _t(f["params0"]))
    fn = O.mf_elbo_grad if cfg["family"] == "mf" else O.mvn_elbo_grad
    val, g = fn(cfg["layers"], f["params0"], f["u"], f["z"], f["w"], f["eps"][0], cfg["S"])
    assert rel(elbo.item(), val) < 1e-5, (elbo.item(), val)
    if name == "g4_fn2_mid":
        # reference init: the classifier-bias gradient is an exact cancellation
        # whose fp32 value (ours and the reference's) is rounding noise
        assert l2rel(grad.cpu().numpy(), g) < 1e-4
    else:
        assert_grad_close(grad.cpu().numpy(), g, what=name, ref_fp32=f["grad0"])
    # and the reference's own numbers
    assert rel(elbo.item(), f["elbo"][0]) < 1e-5


@pytest.mark.parametrize("name", NAMES)
def test_inner_loop_trajectory(name):
    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    params = _t(f["params0"])
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    ws = plan.workspace()
    o_elbo, _, o_traj, o_m, o_v = O.run_inner_loop(
        cfg["family"], cfg["layers"], f["params0"], f["u"], f["z"], f["w"], f["eps"], cfg["S"],
        cfg["lr"], adam_kind(cfg))
    for t in range(cfg["T"]):
        elbo = plan.inner_step(u, z, w, _t(f["eps"][t]), params, m, v, step=t + 1,
                               lr=cfg["lr"], kind=adam_kind(cfg), ws=ws)
        assert rel(elbo.item(), o_elbo[t]) < 1e-5, (t, elbo.item(), o_elbo[t])
        assert rel(elbo.item(), f["elbo"][t]) < 1e-5
        p = params.cpu().numpy()
        # Adam maps entries whose true gradient is below fp32 resolution to
        # +-lr either way; everything else must track the fp64 trajectory.
        assert np.abs(p - o_traj[t]).max() < 0.5 * cfg["lr"], t
        assert l2rel(p, o_traj[t]) < 1e-5, t
        assert l2rel(p, f["params"][t]) < 1e-5, t
    if name != "g4_fn2_mid":
        assert l2rel(m.cpu().numpy(), o_m) < 1e-3
        assert l2rel(v.cpu().numpy(), o_v) < 1e-3


@pytest.mark.parametrize("name", ["g2r_fn_c2_rand_av", "g3r_fn2_tiny_rand", "g5_logreg_fullcov"])
def test_phases_equal_fused_step(name):
    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    eps = _t(f["eps"][0])
    p1 = _t(f["params0"])
    m1, v1 = torch.zeros_like(p1), torch.zeros_like(p1)
    e1 = plan.inner_step(u, z, w, eps, p1, m1, v1, step=1, lr=cfg["lr"])
    p2 = _t(f["params0"])
    m2, v2 = torch.zeros_like(p2), torch.zeros_like(p2)
    if plan.family == "meanfield":
        acc = torch.empty(plan.acc_count, device=DEV)
        e2 = torch.zeros(1, dtype=torch.float64, device=DEV)
        plan.mf_accumulate(u, z, w, eps, p2, acc, e2)
        plan.mf_update(acc, p2, m2, v2, step=1, lr=cfg["lr"], kl_out=e2)
    else:
        xs = torch.empty(plan.xshard_count, device=DEV)
        gs = torch.empty(plan.xshard_count, device=DEV)
        nll = torch.zeros(1, dtype=torch.float64, device=DEV)
        plan.mvn_sample(eps, p2, xs)
        gs.zero_()
        plan.mvn_net(u, z, w, xs, gs, nll)
        kl = torch.zeros(1, dtype=torch.float64, device=DEV)
        plan.mvn_update(eps, gs, p2, m2, v2, step=1, lr=cfg["lr"], kl_out=kl)
        e2 = nll + kl
    assert rel(e2.item(), e1.item()) < 1e-6
    if plan.family == "meanfield":
        # the same fixed-order slot sums in the accumulate and the fused update
        assert torch.equal(p1, p2) and torch.equal(m1, m2) and torch.equal(v1, v2)
    d = (p1 - p2).abs()
    assert d.max().item() < 0.5 * cfg["lr"] and l2rel(p2.cpu().numpy(), p1.cpu().numpy()) < 1e-6


def _emulated_sharded_step(loops, u, z, w, eps, params, ms, vs, step, lr, kind):
    """Run one sharded step for all ranks in-process, doing the two
    all_to_all exchanges with plain device copies."""
    W = len(loops)
    for r in range(W):
        loops[r].phase_sample(eps, params[r])

    def offs(splits):
        return np.concatenate([[0], np.cumsum(splits)]).astype(int)

    for r in range(W):
        parts = []
        for p in range(W):
            o = offs(loops[p].x_in)
            parts.append(loops[p].x_shard[o[r]:o[r + 1]])
        loops[r].x_recv.copy_(torch.cat(parts))
    for r in range(W):
        loops[r].phase_net(u, z, w)
    for p in range(W):
        parts = []
        for q in range(W):
            o = offs(loops[q].g_in)
            parts.append(loops[q].g_send[o[p]:o[p + 1]])
        loops[p].g_shard.copy_(torch.cat(parts))
    for r in range(W):
        loops[r].phase_update(eps, params[r], ms[r], vs[r], step, lr, kind)
    return sum(l.parts.sum().item() for l in loops)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["g3r_fn2_tiny_rand", "g4h_fn2_mid_hyper"])
def test_sharded_fullcov_equals_single(name, world):
    from psvi.runtime.sharded import ShardedInnerLoop

    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    kind = adam_kind(cfg)
    p1 = _t(f["params0"])
    m1, v1 = torch.zeros_like(p1), torch.zeros_like(p1)
    loops = [ShardedInnerLoop("fullcov", cfg["layers"], cfg["S"], cfg["M"], world, r)
             for r in range(world)]
    ps = [_t(f["params0"]) for _ in range(world)]
    ms = [torch.zeros_like(p1) for _ in range(world)]
    vs = [torch.zeros_like(p1) for _ in range(world)]
    for t in range(cfg["T"]):
        eps = _t(f["eps"][t])
        e1 = plan.inner_step(u, z, w, eps, p1, m1, v1, step=t + 1, lr=cfg["lr"], kind=kind)
        e2 = _emulated_sharded_step(loops, u, z, w, eps, ps, ms, vs, t + 1, cfg["lr"], kind)
        assert rel(e2, e1.item()) < 1e-5
    masks = [l.owned_mask() for l in loops]
    total = torch.stack(masks).sum(0)
    assert int(total.min()) == 1 and int(total.max()) == 1, "row shards must partition params"
    full = sum(ps[r] * masks[r] for r in range(world))
    assert torch.allclose(full, p1, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("name", ["g3r_fn2_tiny_rand", "g4h_fn2_mid_hyper", "g5_logreg_fullcov"])
def test_net_draw_equals_separate(name, world):
    """psvi_mvn_phase_net_draw (the sharded loop's network phase with the next
    step's eps drawn by the same launch) == psvi_mvn_phase_net + psvi_randn,
    bitwise: gradients, NLL and every drawn normal, for every rank's plan."""
    from psvi.runtime import randn_
    from psvi.runtime.sharded import ShardedInnerLoop

    f = load_fixture(name)
    cfg, _, u, z, w = _setup(f)
    for r in range(world):
        plan = ShardedInnerLoop("fullcov", cfg["layers"], cfg["S"], cfg["M"], world, r).plan
        g = torch.Generator().manual_seed(5 + r)
        xs = torch.randn(plan.xrecv_count, generator=g).to(DEV)
        n = plan.eps_count
        for off in (0, 4 * n + 8):
            outs = []
            for fused in (False, True):
                gs = torch.full((plan.xrecv_count,), float("nan"), device=DEV)
                nll = torch.zeros(1, dtype=torch.float64, device=DEV)
                e = torch.full((n,), float("nan"), device=DEV)
                if fused:
                    plan.mvn_net(u, z, w, xs, gs, nll, draw=(e, 31, off))
                else:
                    plan.mvn_net(u, z, w, xs, gs, nll)
                    randn_(e, 31, off)
                outs.append((gs, nll, e))
            for a, b in zip(*outs):
                assert torch.equal(a, b), (name, world, r, off)
            assert torch.isfinite(outs[1][2]).all()


def test_net_draw_rank_without_samples():
    """S < world: ranks 4 and 5 of a world-6 plan of S = 4 own rows but no
    samples; their network launch has nothing to compute and must still draw
    the next step's eps (every rank's update reads the same global draw)."""
    from psvi.runtime import randn_
    from psvi.runtime.sharded import ShardedInnerLoop

    f = load_fixture("g5_logreg_fullcov")
    cfg, _, u, z, w = _setup(f)
    assert cfg["S"] == 4
    for r in range(6):
        plan = ShardedInnerLoop("fullcov", cfg["layers"], cfg["S"], cfg["M"], 6, r).plan
        n = plan.eps_count
        xs = torch.randn(max(plan.xrecv_count, 1)).to(DEV)[:plan.xrecv_count]
        gs = torch.zeros(plan.xrecv_count, device=DEV)
        nll = torch.zeros(1, dtype=torch.float64, device=DEV)
        e = torch.full((n,), float("nan"), device=DEV)
        ref = torch.empty(n, device=DEV)
        plan.mvn_net(u, z, w, xs, gs, nll, draw=(e, 7, 4 * n))
        randn_(ref, 7, 4 * n)
        assert torch.equal(e, ref), r
        if r >= 4:
            assert float(nll.item()) == 0.0


def test_net_draw_rejects_bad_draw_args():
    """The fused draw's contract: offset a multiple of 4, eps_out 16-byte
    aligned (vector stores) -- refused with EINVAL, nothing launched."""
    from psvi.runtime import PsviError
    from psvi.runtime.sharded import ShardedInnerLoop

    f = load_fixture("g3r_fn2_tiny_rand")
    cfg, _, u, z, w = _setup(f)
    plan = ShardedInnerLoop("fullcov", cfg["layers"], cfg["S"], cfg["M"], 2, 0).plan
    xs = torch.zeros(plan.xrecv_count, device=DEV)
    gs = torch.zeros(plan.xrecv_count, device=DEV)
    nll = torch.zeros(1, dtype=torch.float64, device=DEV)
    e = torch.zeros(plan.eps_count + 4, device=DEV)
    with pytest.raises(PsviError, match="multiple of 4"):
        plan.mvn_net(u, z, w, xs, gs, nll, draw=(e, 1, 2))
    with pytest.raises(PsviError, match="16-byte"):
        plan.mvn_net(u, z, w, xs, gs, nll, draw=(e[1:], 1, 0))


def test_randn_moments_and_determinism():
    from psvi.runtime import randn_

    a = torch.empty(1 << 22, device=DEV)
    b = torch.empty(1 << 22, device=DEV)
    randn_(a, seed=1234, offset=0)
    randn_(b, seed=1234, offset=0)
    assert torch.equal(a, b)
    assert torch.isfinite(a).all()
    assert abs(a.mean().item()) < 3e-3 and abs(a.std().item() - 1) < 3e-3
    # N(0,1) shape: tail probabilities and the fourth moment
    for k, p in ((1.0, 0.3173105), (2.0, 0.0455003), (3.0, 0.0026998)):
        frac = (a.abs() > k).float().mean().item()
        assert abs(frac - p) < 5 * (p * (1 - p) / a.numel()) ** 0.5 + 1e-5, (k, frac)
    assert abs((a.double() ** 4).mean().item() - 3.0) < 0.02
    c = torch.empty(1 << 22, device=DEV)
    randn_(c, seed=1235, offset=0)
    assert not torch.equal(a, c)
    # counter-based: a shifted offset reproduces the tail of the stream
    d = torch.empty((1 << 22) - 1024, device=DEV)
    randn_(d, seed=1234, offset=1024)
    assert torch.equal(d, a[1024:])


@pytest.mark.parametrize("name", [n for n in NAMES if load_fixture(n)["cfg"]["family"] == "mvn"])
def test_fused_update_sample_equals_separate(name):
    """psvi_mvn_phase_update_sample == update, then sample from the new params."""
    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    eps0, eps1 = _t(f["eps"][0]), _t(f["eps"][1])
    p1 = _t(f["params0"])
    xs = torch.empty(plan.xshard_count, device=DEV)
    gs = torch.empty(plan.xshard_count, device=DEV)
    nll = torch.zeros(1, dtype=torch.float64, device=DEV)
    plan.mvn_sample(eps0, p1, xs)
    plan.mvn_net(u, z, w, xs, gs, nll)
    p2 = p1.clone()
    m1, v1 = torch.zeros_like(p1), torch.zeros_like(p1)
    m2, v2 = torch.zeros_like(p1), torch.zeros_like(p1)
    k1 = torch.zeros(1, dtype=torch.float64, device=DEV)
    k2 = torch.zeros(1, dtype=torch.float64, device=DEV)
    plan.mvn_update(eps0, gs, p1, m1, v1, step=1, lr=cfg["lr"], kl_out=k1)
    x1 = torch.empty_like(xs)
    plan.mvn_sample(eps1, p1, x1)
    x2 = torch.full_like(xs, float("nan"))
    plan.mvn_update(eps0, gs, p2, m2, v2, step=1, lr=cfg["lr"], kl_out=k2, eps_next=eps1,
                    x_next=x2)
    # the streaming kernel (S a multiple of 32) contracts the Adam arithmetic
    # differently from the packed one: equal to within a few ulp
    for a, b in ((p1, p2), (m1, m2), (v1, v2)):
        a, b = a.cpu().numpy().astype(np.float64), b.cpu().numpy()
        assert np.abs(a - b).max() <= 1e-7 * np.abs(b).max()
    assert rel(k1.item(), k2.item()) < 1e-12
    assert torch.isfinite(x2).all()
    assert l2rel(x2.cpu().numpy(), x1.cpu().numpy()) < 1e-6
    assert (x2 - x1).abs().max().item() <= 1e-5 * x1.abs().max().item()


@pytest.mark.parametrize("name", NAMES)
def test_inner_loop_api_matches_oracle(name):
    """psvi_inner_loop (T chained steps, fused next-step sampling) with the
    reference's eps == the oracle trajectory and the reference's ELBOs."""
    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    params = _t(f["params0"])
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    eps = _t(np.ascontiguousarray(f["eps"]).reshape(-1))
    elbos = plan.inner_loop(u, z, w, params, m, v, cfg["T"], cfg["lr"], adam_kind(cfg), eps=eps)
    o_elbo, _, o_traj, _, _ = O.run_inner_loop(
        cfg["family"], cfg["layers"], f["params0"], f["u"], f["z"], f["w"], f["eps"], cfg["S"],
        cfg["lr"], adam_kind(cfg))
    e = elbos.cpu().numpy()
    for t in range(cfg["T"]):
        assert rel(e[t], o_elbo[t]) < 1e-5 and rel(e[t], f["elbo"][t]) < 1e-5, t
    p = params.cpu().numpy()
    assert np.abs(p - o_traj[-1]).max() < 0.5 * cfg["lr"]
    assert l2rel(p, o_traj[-1]) < 1e-5 and l2rel(p, f["params"][-1]) < 1e-5


@pytest.mark.parametrize("family,layers,S,M", [
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100),
    ("fullcov", [(9, 5), (5, 3)], 40, 7),
    ("meanfield", [(2, 100), (100, 4)], 32, 50)])
def test_inner_loop_philox_equals_stepwise(family, layers, S, M):
    """Philox-drawn loop == the same draws fed step by step through psvi_inner_step.

    Full-cov: the first step is bitwise the same.  From the second on, the
    loop's fused update + next-step sample has summed x' in another fp32
    order than the stepwise sample, so x_1 differs in the last bits; where
    that moves a hidden pre-activation across the ReLU kink (a route flip)
    the gradient of that unit's rows changes by O(1), and Adam moves the
    affected coordinates by up to a step (lr) in either trajectory (measured
    at C3 for this seed: 508 of 4.73 M coordinates by more than 0.1 lr after
    two steps with one build of the network kernel, none with the previous
    one, and none with either on 8 other seeds -- it hangs on the last bits).
    Bar after two steps: the ELBOs to 1e-6; the parameters equal (to 0.1 lr)
    except on at most 0.1 % of the coordinates, and there by at most two
    steps."""
    from psvi.runtime import InnerLoopPlan, randn_

    plan = InnerLoopPlan(family, layers, S, M)
    g = torch.Generator().manual_seed(S + M)
    u = torch.randn(M, layers[0][0], generator=g).to(DEV)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).to(DEV)
    w = torch.full((M,), 8.0, device=DEV)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * torch.randn(n, generator=g), torch.full((n,), -3.0)]
        if family == "fullcov":
            parts.append(1e-3 * torch.randn((n - 1) * (n - 2) // 2, generator=g))
    p0 = torch.cat(parts).to(DEV)
    T, lr = 2, 1e-3
    pa, ma, va = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    ea = plan.inner_loop(u, z, w, pa, ma, va, T, lr, seed=7, offset=0)
    pb, mb, vb = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    eps = torch.empty(plan.eps_count, device=DEV)
    ws = plan.workspace()
    eb = []
    for t in range(T):
        randn_(eps, 7, t * plan.eps_stride)
        eb.append(plan.inner_step(u, z, w, eps, pb, mb, vb, step=t + 1, lr=lr, ws=ws).item())
        if t == 0:
            pb1 = pb.clone()
    ea = ea.cpu().numpy()
    p1, m1, v1 = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    plan.inner_loop(u, z, w, p1, m1, v1, 1, lr, seed=7, offset=0)
    assert torch.equal(p1, pb1)
    if family == "meanfield":  # no fused sample: the whole trajectory is bitwise the same
        assert torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb)
    d = (pa - pb).abs()
    moved = int((d > 0.1 * lr).sum())
    print(f"{family} S={S} M={M}: loop-step ELBO rel {np.abs(ea - eb) / np.abs(eb)}, params "
          f"l2rel {l2rel(pa.cpu().numpy(), pb.cpu().numpy()):.2e}, {moved} moved, max {float(d.max()):.2e}")
    assert np.allclose(ea, eb, rtol=1e-6, atol=0)
    assert moved <= 1e-3 * d.numel() and float(d.max()) <= 2 * lr + 1e-6


@pytest.mark.parametrize("layers,S", [([(64, 40), (40, 40), (40, 2)], 128),
                                      ([(9, 5), (5, 3)], 40), ([(8, 6), (6, 6), (6, 3)], 16)])
def test_tiled_state_roundtrip(layers, S):
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan("fullcov", layers, S, 10)
    assert plan.tiled_floats > 0
    g = torch.Generator().manual_seed(1)
    p, m, v = (torch.randn(plan.param_count, generator=g).to(DEV) for _ in range(3))
    ts = plan.tiled_state()
    plan.tiled_convert(p, m, v, ts, True)
    q, mq, vq = (torch.zeros_like(p) for _ in range(3))
    plan.tiled_convert(q, mq, vq, ts, False)
    po = 0
    for din, dout in layers:
        n = din * dout + dout
        nc = (n - 1) * (n - 2) // 2
        sl = slice(po + 2 * n, po + 2 * n + nc)
        for a, b in ((p, q), (m, mq), (v, vq)):
            assert torch.equal(a[sl], b[sl])
            assert torch.count_nonzero(b[po:po + 2 * n]) == 0  # mean / sd untouched
        po += 2 * n + nc
    # the tiled copy holds each corr entry exactly once, zeros elsewhere
    tf = plan.tiled_floats // 3
    assert torch.count_nonzero(ts[:tf]) == torch.count_nonzero(
        torch.cat([p[po2 + 2 * n2: po2 + 2 * n2 + (n2 - 1) * (n2 - 2) // 2]
                   for po2, n2 in _layer_offsets(layers)]))


def _layer_offsets(layers):
    po, out = 0, []
    for din, dout in layers:
        n = din * dout + dout
        out.append((po, n))
        po += 2 * n + (n - 1) * (n - 2) // 2
    return out


@pytest.mark.parametrize("name", [n for n in NAMES if load_fixture(n)["cfg"]["family"] == "mvn"])
@pytest.mark.parametrize("fused", [False, True])
def test_tiled_update_equals_packed(name, fused):
    f = load_fixture(name)
    cfg, plan, u, z, w = _setup(f)
    eps0, eps1 = _t(f["eps"][0]), _t(f["eps"][1])
    p1 = _t(f["params0"])
    xs = torch.empty(plan.xshard_count, device=DEV)
    gs = torch.empty(plan.xshard_count, device=DEV)
    nll = torch.zeros(1, dtype=torch.float64, device=DEV)
    plan.mvn_sample(eps0, p1, xs)
    plan.mvn_net(u, z, w, xs, gs, nll)
    p2 = p1.clone()
    m1, v1 = torch.zeros_like(p1), torch.zeros_like(p1)
    m2, v2 = torch.zeros_like(p1), torch.zeros_like(p1)
    k1 = torch.zeros(1, dtype=torch.float64, device=DEV)
    k2 = torch.zeros(1, dtype=torch.float64, device=DEV)
    x1, x2 = torch.empty_like(xs), torch.full_like(xs, float("nan"))
    kw = dict(eps_next=eps1, x_next=x1) if fused else {}
    plan.mvn_update(eps0, gs, p1, m1, v1, step=1, lr=cfg["lr"], kind=adam_kind(cfg), kl_out=k1, **kw)
    ts = plan.tiled_state()
    plan.tiled_convert(p2, m2, v2, ts, True)
    kw = dict(eps_next=eps1, x_next=x2) if fused else {}
    plan.mvn_update_tiled(eps0, gs, p2, m2, v2, ts, step=1, lr=cfg["lr"], kind=adam_kind(cfg),
                          kl_out=k2, **kw)
    plan.tiled_convert(p2, m2, v2, ts, False)
    # the streaming kernel (S a multiple of 32) contracts the Adam arithmetic
    # differently from the packed one: equal to within a few ulp
    for a, b in ((p1, p2), (m1, m2), (v1, v2)):
        a, b = a.cpu().numpy().astype(np.float64), b.cpu().numpy()
        assert np.abs(a - b).max() <= 1e-7 * np.abs(b).max()
    assert rel(k1.item(), k2.item()) < 1e-6  # fp32 per-thread partial sums, other order
    if fused:
        assert torch.isfinite(x2).all()
        assert l2rel(x2.cpu().numpy(), x1.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("name", ["g2r_fn_c2_rand_av", "g3r_fn2_tiny_rand", "l1_lenet_tiny"])
def test_inner_loop_checkpoint_resume(name):
    """Checkpoint / resume: the inner-loop state is caller-owned,
    so saving params and the Adam m, v with torch.save after k steps and
    resuming with step0 = k + 1 continues the same trajectory."""
    import io

    from psvi.runtime import InnerLoopPlan

    f = load_fixture(name)
    cfg = f["cfg"]
    plan = InnerLoopPlan(family_of(cfg), plan_layers(cfg), cfg["S"], cfg["M"])
    u, z, w = _t(f["u"]), _t(f["z"].astype(np.int32), torch.int32), _t(f["w"])
    T, kind, eps = cfg["T"], adam_kind(cfg), _t(f["eps"])
    p1 = _t(f["params0"])
    m1, v1 = torch.zeros_like(p1), torch.zeros_like(p1)
    e1 = plan.inner_loop(u, z, w, p1, m1, v1, T, cfg["lr"], kind=kind, eps=eps)
    p2 = _t(f["params0"])
    m2, v2 = torch.zeros_like(p2), torch.zeros_like(p2)
    k = 1
    ea = plan.inner_loop(u, z, w, p2, m2, v2, k, cfg["lr"], kind=kind,
                         eps=eps[:k].contiguous()).clone()
    buf = io.BytesIO()
    torch.save({"params": p2, "m": m2, "v": v2, "step": k}, buf)
    buf.seek(0)
    st = torch.load(buf, weights_only=True)  # a file this test wrote
    eb = plan.inner_loop(u, z, w, st["params"], st["m"], st["v"], T - k, cfg["lr"], kind=kind,
                         step0=st["step"] + 1, eps=eps[k:].contiguous())
    e2 = torch.cat([ea, eb]).cpu().numpy()
    assert rel(e2, e1.cpu().numpy()) < 1e-6
    for a, b in ((st["params"], p1), (st["m"], m1), (st["v"], v1)):
        assert l2rel(a.cpu().numpy(), b.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("layers,S,M", [
    ([(64, 40), (40, 40), (40, 2)], 1024, 200),   # C4 at one GPU: two pseudopoint chunks
    ([(64, 40), (40, 40), (40, 2)], 8, 200),      # few samples: many chunks per sample
])
def test_fullcov_step_bitwise_reproducible(layers, S, M):
    """Pseudopoint-chunked full-cov network: the chunks' partial dW go to
    per-chunk slots added in chunk order (no float atomics), so two identical
    inner steps give bitwise identical parameters, Adam state and ELBO."""
    from psvi.runtime import InnerLoopPlan, randn_

    plan = InnerLoopPlan("fullcov", layers, S, M)
    g = torch.Generator().manual_seed(S + M)
    u = torch.randn(M, layers[0][0], generator=g).to(DEV)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).to(DEV)
    w = torch.full((M,), 4.0, device=DEV)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * torch.randn(n, generator=g), torch.full((n,), -3.0),
                  1e-3 * torch.randn((n - 1) * (n - 2) // 2, generator=g)]
    p0 = torch.cat(parts).to(DEV)
    eps = torch.empty(plan.eps_count, device=DEV)
    randn_(eps, 5)
    out = []
    for _ in range(2):
        p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
        e = plan.inner_step(u, z, w, eps, p, m, v, step=1, lr=1e-3)
        out.append((e.item(), p, m, v))
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1:], out[1][1:]):
        assert torch.equal(a, b)
