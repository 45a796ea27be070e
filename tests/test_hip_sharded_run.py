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

            def all_to_all_list(self, outs, ins):
                # per-peer views; each rank copies on its current stream (a side
                # stream in run(overlap=True)) after the sources' producers
                from psvi.runtime.sharded import check_exchange_list
                check_exchange_list(outs, ins, outer.world)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
                outer.slots[rank] = (list(ins), ev)
                outer.bar.wait()
                for q in range(outer.world):
                    src, qev = outer.slots[q]
                    torch.cuda.current_stream().wait_event(qev)
                    assert src[rank].numel() == outs[q].numel(), (q, rank)
                    outs[q].copy_(src[rank])
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


def _sharded_run(layers, S, M, world, u, z, w, p0, T, lr, kind, seed, offset, overlap=False):
    """run() on every thread-rank; returns (negative ELBO per step, params,
    m, v) after gather_params (identical on every rank)."""
    from psvi.runtime.sharded import ShardedInnerLoop

    def rank_fn(r, comm):
        loop = ShardedInnerLoop("fullcov", layers, S, M, world, r, comm=comm)
        p = p0.clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        parts = torch.zeros(T, 2, dtype=torch.float64, device=DEV)
        loop.run(u, z, w, p, m, v, T, lr, kind=kind, seed=seed, offset=offset,
                 elbo_parts=parts, overlap=overlap)
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


def _chain_steps(layers, S, M, world, u, z, w, p0, T, lr, kind, seed, offset):
    """The same T steps through ShardedInnerLoop.step() (unfused phases:
    sample, x exchange, network, G exchange, update) on separate psvi_randn
    draws -- what run() must reproduce bit for bit."""
    from psvi.runtime import randn_
    from psvi.runtime.sharded import ShardedInnerLoop

    def rank_fn(r, comm):
        loop = ShardedInnerLoop("fullcov", layers, S, M, world, r, comm=comm)
        p = p0.clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        parts = torch.zeros(T, 2, dtype=torch.float64, device=DEV)
        e = torch.empty(loop.plan.eps_count, device=DEV)
        for k in range(T):
            randn_(e, seed, offset + k * loop.plan.eps_stride)
            loop.step(u, z, w, e, p, m, v, k + 1, lr, kind=kind, elbo_parts=parts[k])
        neg = loop.reduce_elbo(parts)
        loop.gather_params(p, m, v)
        return neg, p, m, v

    res = _run_ranks(world, rank_fn)
    return [x.cpu().numpy().astype(np.float64) for x in res[0]]


@pytest.mark.parametrize("W,S,M", [(8, 1024, 200), (8, 1024, 100), (2, 256, 100)])
def test_run_full_size(W, S, M):
    """C4 (S = 1024, M = 200) and the weak headline's W = 8 / W = 2 shapes.
    (1) run() over T = 3 steps == the unfused step() chain on psvi_randn draws,
    bit for bit (ELBO terms, params, m, v): the fused draw, the fused
    update + next sample, the eps swap and the offsets change nothing.
    (2) One step of run() against the world-1 psvi_inner_loop (same seed and
    offset): ELBO within 1e-6; params within 0.1 lr per entry except rare
    sign-flipped Adam steps (below), the rest within 1e-6 (l2).
    The sharded sample splits its K sums along the row shards, so x differs
    from world 1 in the last bits and a sample on a ReLU kink can take the
    other mask (test_hip_fullsize.py::test_row_sharded_full_size margin-checks
    those); over several steps such differences compound through Adam's
    ~ lr sign(g) steps, so multi-step trajectories are compared with the
    chain above, not with world 1."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_hip_fullsize import make_case

    layers = [(64, 40), (40, 40), (40, 2)]
    params, u, z, w, _ = make_case("fullcov", layers, S, M, 3)
    t = lambda x, d=torch.float32: torch.tensor(x, dtype=d, device=DEV)
    du, dz, dw, p0 = t(u), t(z, torch.int32), t(w), t(params)
    lr, seed, offset = 1e-3, 99, 0
    eW, pW, mW, vW = _sharded_run(layers, S, M, W, du, dz, dw, p0, 3, lr, "higher", seed, offset)
    eC, pC, mC, vC = _chain_steps(layers, S, M, W, du, dz, dw, p0, 3, lr, "higher", seed, offset)
    assert np.array_equal(eW, eC), (eW, eC)
    for a, b, n in ((pW, pC, "params"), (mW, mC, "m"), (vW, vC, "v")):
        assert np.array_equal(a, b), (n, np.abs(a - b).max())
    (e1, p1, m1, v1), _ = _world1(layers, S, M, du, dz, dw, p0, 1, lr, "higher", seed, offset)
    e8, p8, m8, v8 = _sharded_run(layers, S, M, W, du, dz, dw, p0, 1, lr, "higher", seed, offset)
    print(f"W={W} S={S} M={M}: elbo {e8[0]!r} vs {e1[0]!r}; params l2 {l2rel(p8, p1):.2e} "
          f"max {np.abs(p8 - p1).max():.2e}")
    assert rel(e8[0], e1[0]) < 1e-6
    # kink samples change G of that sample; a gradient entry that cancels to
    # ~0 over S can then flip the sign of its Adam step (~ lr sign(g)): such
    # entries move by at most 2 lr and must be rare, every other entry agrees
    d = np.abs(p8 - p1)
    off = d > 0.1 * lr
    print(f"  entries off by > 0.1 lr: {int(off.sum())} of {d.size}")
    assert off.sum() < 1e-3 * d.size and d.max() < 2.05 * lr
    assert l2rel(p8[~off], p1[~off]) < 1e-6


@pytest.mark.parametrize("W,S,M", [(8, 1024, 200), (2, 256, 100), (3, 768, 40), (3, 257, 40)])
def test_run_overlap_equals_plain(W, S, M):
    """run(overlap=True): the rank's samples in two halves, each exchange as
    two list all_to_alls of per-peer views on a side stream beside the other
    half's network (psvi_mvn_phase_net_part), the draw split between the two
    launches -- the same parameters, Adam state and draws as the plain
    schedule, bit for bit (the NLL's atomic adds come in another order).
    (3, 257, 40): a plan with per-chunk gradient slots (not looped), which
    takes the plain schedule.)"""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_hip_fullsize import make_case

    layers = [(64, 40), (40, 40), (40, 2)] if M >= 100 else [(12, 20), (20, 4)]
    params, u, z, w, _ = make_case("fullcov", layers, S, M, 5)
    t = lambda x, d=torch.float32: torch.tensor(x, dtype=d, device=DEV)
    du, dz, dw, p0 = t(u), t(z, torch.int32), t(w), t(params)
    eA, pA, mA, vA = _sharded_run(layers, S, M, W, du, dz, dw, p0, 3, 1e-3, "higher", 7, 0)
    eB, pB, mB, vB = _sharded_run(layers, S, M, W, du, dz, dw, p0, 3, 1e-3, "higher", 7, 0,
                                  overlap=True)
    for a, b, n in ((pA, pB, "params"), (mA, mB, "m"), (vA, vB, "v")):
        assert np.array_equal(a, b), (n, np.abs(a - b).max())
    for k in range(3):
        assert rel(eA[k], eB[k]) < 1e-12, (k, eA[k], eB[k])
