"""The network kernel's looped pseudopoint chunks (full-cov, M past the LDS:
C4's M = 200) against one workgroup per chunk with per-chunk slots and the
slot sum (PSVI_DBG_NET_MLOOP_OFF).  The looped form adds chunk c's weight
gradient to chunk 0's in chunk order -- the slot sum's order -- so every
gradient element must agree bit for bit; the weighted NLL (each thread's
fp32 share now spans every chunk before the fp64 sum) to 1e-7.  Reference op:
VILinearMultivariateNormal.forward + the weighted NLL backward
(/root/reference/psvi/models/neural_net.py:485-491,
psvi/inference/psvi_classes.py:496-505)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
MLOOP_OFF = 23  # PSVI_DBG_NET_MLOOP_OFF


def _net_once(plan, u, z, w, xs, off):
    g = torch.full((plan.xrecv_count,), float("nan"), device=DEV)
    nll = torch.zeros(1, dtype=torch.float64, device=DEV)
    assert plan.lib.psvi_debug_set(MLOOP_OFF, off) == 0
    try:
        plan.mvn_net(u, z, w, xs, g, nll)
        torch.cuda.synchronize()
    finally:
        plan.lib.psvi_debug_set(MLOOP_OFF, 0)
    return g, nll


@pytest.mark.parametrize("world,S,M,layers", [
    (8, 1024, 200, [(64, 40), (40, 40), (40, 2)]),   # C4 rank at W = 8 (several sources)
    (1, 1024, 200, [(64, 40), (40, 40), (40, 2)]),   # C4 on one GPU
    (2, 512, 333, [(64, 40), (40, 40), (40, 2)]),    # three chunks, ragged last
    (1, 300, 250, [(32, 48), (48, 24), (24, 3)]),    # other widths, C = 3
])
def test_looped_chunks_equal_slots(world, S, M, layers):
    from psvi.runtime.sharded import ShardedInnerLoop

    ranks = [0, world - 1] if world > 1 else [0]
    g = torch.Generator().manual_seed(M)
    u = torch.randn(M, layers[0][0], generator=g).to(DEV)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(DEV, torch.int32)
    w = (torch.rand(M, generator=g) * 8).to(DEV)
    for r in ranks:
        plan = ShardedInnerLoop("fullcov", layers, S, M, world, r).plan
        assert plan.lib.psvi_debug_set(MLOOP_OFF, 0) == 0
        xs = (0.3 * torch.randn(plan.xrecv_count, generator=g)).to(DEV)
        g1, n1 = _net_once(plan, u, z, w, xs, 0)
        g2, n2 = _net_once(plan, u, z, w, xs, 1)
        assert torch.isfinite(g1).all(), (world, r)
        assert torch.equal(g1, g2), (world, r, float((g1 - g2).abs().max()))
        assert abs(n1.item() - n2.item()) <= 1e-7 * abs(n2.item())  # fp32 per-thread parts
