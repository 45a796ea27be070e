"""Host-side contracts that guard the multi-GPU path before anything runs on
RCCL (CPU): the all_to_all split/dtype/contiguity check every exchange passes
through (psvi.runtime.sharded.check_exchange), and the plan's bound on the
tiled corr / m / v state that the write-through buffer stores address with
one 32-bit descriptor (capi.cpp tiled_ok)."""
import pytest
import torch


def test_check_exchange_accepts_the_plan_splits():
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime.sharded import check_exchange

    layers, S, W = [(64, 40), (40, 40), (40, 2)], 256, 4
    infos = [InnerLoopPlan("fullcov", layers, S, 100, world=W, rank=0).shard_info(r)
             for r in range(W)]
    for r in range(W):
        me = infos[r]
        x_in = [q["s_count"] * me["rows"] for q in infos]
        x_out = [me["s_count"] * p["rows"] for p in infos]
        inp = torch.zeros(sum(x_in))
        out = torch.zeros(sum(x_out))
        check_exchange(out, inp, x_out, x_in, W)


@pytest.mark.parametrize("bad", ["sum", "count", "neg", "dtype", "contig"])
def test_check_exchange_rejects(bad):
    from psvi.runtime.sharded import check_exchange

    out, inp = torch.zeros(12), torch.zeros(12)
    so, si = [6, 6], [6, 6]
    if bad == "sum":
        si = [6, 5]
    elif bad == "count":
        so = [4, 4, 4]
    elif bad == "neg":
        so = [13, -1]
    elif bad == "dtype":
        inp = torch.zeros(12, dtype=torch.float64)
    elif bad == "contig":
        out = torch.zeros(12, 2)[:, 0]
    with pytest.raises(ValueError):
        check_exchange(out, inp, so, si, 2)


def test_tiled_state_stays_under_the_descriptor_bound():
    """Every full-cov plan the library accepts either keeps corr / m / v
    packed (tiled_floats == 0) or tiles them in < 2^31 bytes.  Today the
    per-sample network kernel's LDS bound keeps a layer below ~13 k rows (the
    widest accepted layers tile to < 0.5 x 2^31 bytes); the plan-side guard
    covers any future widening of that kernel."""
    from psvi.runtime import InnerLoopPlan, PsviError

    widest = 0
    for layers in ([(90, 140), (140, 2)], [(64, 40), (40, 40), (40, 2)], [(120, 100), (100, 2)],
                   [(64, 180), (180, 2)], [(200, 60), (60, 60), (60, 2)]):
        try:
            p = InnerLoopPlan("fullcov", layers, 128, 8)
        except PsviError:
            continue
        tb = 4 * p.tiled_floats
        assert tb == 0 or tb < 2 ** 31 - 16, (layers, tb)
        widest = max(widest, tb)
    assert widest > 0
