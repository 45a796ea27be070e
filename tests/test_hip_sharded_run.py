"""GPU parity of ShardedInnerLoop.run() -- the exact per-rank schedule the
N > 1 bench times (reference semantics: T chained steps of
PSVI.inner_elbo + DifferentiableAdam, psvi/inference/psvi_classes.py:549-555,
psvi/models/neural_net.py:452-476).

run() composes, per step: the x exchange, the network launch that also draws
the next step's eps (psvi_mvn_phase_net_draw), the G exchange, and the update
fused with the next step's sample (psvi_mvn_phase_update_sample; the K-split
kernel at K = S > 128), the e_cur / e_nxt swap and the Philox offsets; the last
step samples nothing.  Here W ranks run as threads on one GPU; the two
all_to_alls are device copies of exactly the blocks each rank receives (the
TorchDistComm contract, check_exchange asserted), the all-reduces sums.  The
result must equal the world-1 psvi_inner_loop on the same seed and offset, and
the float64 oracle (oracle/psvi_oracle.py run_inner_loop) on those draws."""
import threading

import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import family_of, l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _DevComm:
    """all_to_all / all_reduce among thread-ranks sharing one GPU stream."""

    def __init__(self, world):
        self.world = world
        self.slots = [None] * world
        self.bar = threading.Barrier(world)

    def bind(self, rank):
        from psvi.runtime.sharded import check_exchange

        outer = self

        class _Rank:
            name = "device copies (thread ranks)"
            host_staged = False

            def all_to_all(self, out, inp, out_splits, in_splits):
                check_exchange(out, inp, out_splits, in_splits, outer.world)
                outer.slots[rank] = (inp, [int(x) for x in in_splits])
                outer.bar.wait()
                o = 0
                for q in range(outer.world):
                    src, sp = outer.slots[q]
                    lo = sum(sp[:rank])
                    n = int(out_splits[q])
                    assert sp[rank] == n, (q, rank, sp[rank], n)
                    out[o:o + n].copy_(src[lo:lo + n])
                    o += n
                outer.bar.wait()

            def all_reduce(self, t):
                outer.slots[rank] = t.clone()
                outer.bar.wait()
                total = sum(outer.slots[r] for r in range(outer.world))
                outer.bar.wait()
                t.copy_(total)

        return _Rank()


def _run_ranks(world, fn):
    comm = _DevComm(world)
    res, errs = [None] * world, []

    def run(r):
        try:
            res[r] = fn(r, comm.bind(r))
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not errs, errs
    return res


def _sharded_run(layers, S, M, world, u, z, w, p0, T, lr, kind, seed, offset):
    """run() on every thread-rank; returns (negative ELBO per step, params,
    m, v) after gather_params (identical on every rank)."""
    from psvi.runtime.sharded import ShardedInnerLoop

    def rank_fn(r, comm):
        loop = ShardedInnerLoop("fullcov", layers, S, M, world, r, comm=comm)
        p = p0.clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        parts = torch.zeros(T, 2, dtype=torch.float64, device=DEV)
        loop.run(u, z, w, p, m, v, T, lr, kind=kind, seed=seed, offset=offset,
                 elbo_parts=parts)
        neg = loop.reduce_elbo(parts)
        loop.gather_params(p, m, v)
        return neg, p, m, v

    res = _run_ranks(world, rank_fn)
    for r in range(1, world):
        for a, b in zip(res[0][1:], res[r][1:]):
            assert torch.equal(a, b), f"rank {r} differs after gather_params"
    return [x.cpu().numpy().astype(np.float64) for x in res[0]]


def _world1(layers, S, M, u, z, w, p0, T, lr, kind, seed, offset):
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan("fullcov", layers, S, M)
    p = p0.clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    e = plan.inner_loop(u, z, w, p, m, v, T, lr, kind=kind, seed=seed, offset=offset)
    return [x.cpu().numpy().astype(np.float64) for x in (e, p, m, v)], plan


CASES = [("g3r_fn2_tiny_rand", 2), ("g3r_fn2_tiny_rand", 3), ("g3r_fn2_tiny_rand", 8),
         ("g4h_fn2_mid_hyper", 2), ("g4h_fn2_mid_hyper", 3), ("g4h_fn2_mid_hyper", 8),
         ("g5_logreg_fullcov", 6)]   # S = 4 < world: ranks 4, 5 own rows but no samples


@pytest.mark.parametrize("name,world", CASES)
def test_run_matches_world1_and_oracle(name, world):
    from psvi.runtime import randn_

    f = load_fixture(name)
    cfg = f["cfg"]
    assert family_of(cfg) == "fullcov"
    layers, S, M, lr = cfg["layers"], cfg["S"], cfg["M"], cfg["lr"]
    kind = cfg["adam"]
    t = lambda x, d=torch.float32: torch.tensor(np.ascontiguousarray(x), dtype=d, device=DEV)
    u, z, w, p0 = t(f["u"]), t(f["z"].astype(np.int32), torch.int32), t(f["w"]), t(f["params0"])
    T, seed = 3, 4242
    (e1, p1, m1, v1), plan = _world1(layers, S, M, u, z, w, p0, T, lr, kind, seed, 0)
    offset = 8 * plan.eps_stride   # a non-zero start: step t at offset + t * stride
    (e1, p1, m1, v1), _ = _world1(layers, S, M, u, z, w, p0, T, lr, kind, seed, offset)
    eW, pW, mW, vW = _sharded_run(layers, S, M, world, u, z, w, p0, T, lr, kind, seed, offset)
    for k in range(T):
        assert rel(eW[k], e1[k]) < 1e-6, (k, eW[k], e1[k])
    assert l2rel(pW, p1) < 1e-6
    assert l2rel(mW, m1) < 1e-5 and l2rel(vW, v1) < 1e-5
    # the float64 oracle on the same Philox draws
    draws = []
    for k in range(T):
        e = torch.empty(plan.eps_count, device=DEV)
        randn_(e, seed, offset + k * plan.eps_stride)
        draws.append(e.cpu().numpy().astype(np.float64))
    o_e, _, o_traj, o_m, o_v = O.run_inner_loop("mvn", layers, f["params0"], f["u"], f["z"],
                                                f["w"], draws, S, lr, kind,
                                                prior_sd=cfg["prior_sd"])
    for k in range(T):
        assert rel(eW[k], o_e[k]) < 1e-5, (k, eW[k], o_e[k])
    assert l2rel(pW, o_traj[-1]) < 1e-6
    assert l2rel(mW, o_m) < 1e-4 and l2rel(vW, o_v) < 1e-4


@pytest.mark.parametrize("W,S,M", [(8, 1024, 200), (8, 1024, 100), (2, 256, 100)])
def test_run_full_size_matches_world1(W, S, M):
    """C4 (S = 1024, M = 200) and the weak headline's W = 8 / W = 2 shapes:
    run() over T = 3 steps against the world-1 psvi_inner_loop (same seed and
    offset).  The sharded sample splits its K sums along the row shards, so x
    differs from world 1 in the last bits and a sample sitting on a ReLU kink
    can take the other mask; Adam's first steps are ~ lr sign(g), so an entry
    whose gradient cancels to ~0 can then move by up to ~lr.  The bound: the
    ELBO per step within 1e-6, params / m within 1e-6 / 1e-4 (l2), and every
    entry within 0.1 lr per step."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_hip_fullsize import make_case

    layers = [(64, 40), (40, 40), (40, 2)]
    params, u, z, w, _ = make_case("fullcov", layers, S, M, 3)
    t = lambda x, d=torch.float32: torch.tensor(x, dtype=d, device=DEV)
    du, dz, dw, p0 = t(u), t(z, torch.int32), t(w), t(params)
    T, lr, seed, offset = 3, 1e-3, 99, 0
    (e1, p1, m1, v1), _ = _world1(layers, S, M, du, dz, dw, p0, T, lr, "higher", seed, offset)
    eW, pW, mW, vW = _sharded_run(layers, S, M, W, du, dz, dw, p0, T, lr, "higher", seed, offset)
    print(f"W={W} S={S} M={M}: elbo {eW} vs {e1}; params l2 {l2rel(pW, p1):.2e} "
          f"max {np.abs(pW - p1).max():.2e}")
    for k in range(T):
        assert rel(eW[k], e1[k]) < 1e-6, (k, eW[k], e1[k])
    assert l2rel(pW, p1) < 1e-6
    assert np.abs(pW - p1).max() < 0.1 * lr * T
    assert l2rel(mW, m1) < 1e-4
