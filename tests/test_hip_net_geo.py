"""The network kernel's compile-time fn2 geometry (NetGeo<1 / 2>: the 64 ->
40 -> 40 -> 2 stack of configs C3 / C4, 100-row pseudopoint chunks) against
its run-time geometry (PSVI_DBG_NET_GEO_OFF): the same arithmetic in the same
order, so the gradients and the NLL are bitwise equal -- one source rank and
several (the band table), one pseudopoint chunk and the looped chunks of M =
200.  Reference: VILinearMultivariateNormal.forward / the inner ELBO's
backward (psvi/models/neural_net.py:485-491, psvi/inference/
psvi_classes.py:488-511); the kernels themselves are held to the oracle by
test_hip_parity.py / test_hip_fullsize.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
GEO_OFF = 30  # PSVI_DBG_NET_GEO_OFF
FN2 = [(64, 40), (40, 40), (40, 2)]


def _net(plan, u, z, w, xs, draw, geo_off):
    lib = plan.lib
    assert lib.psvi_debug_set(GEO_OFF, int(geo_off)) == 0
    try:
        gs = torch.full((plan.xrecv_count,), float("nan"), device=DEV)
        nll = torch.zeros(1, dtype=torch.float64, device=DEV)
        if draw:
            e = torch.zeros(plan.eps_count, device=DEV)
            plan.mvn_net(u, z, w, xs, gs, nll, draw=(e, 7, 4 * plan.eps_stride))
        else:
            e = None
            plan.mvn_net(u, z, w, xs, gs, nll)
        torch.cuda.synchronize()
    finally:
        lib.psvi_debug_set(GEO_OFF, 0)
    return gs, nll, e


@pytest.mark.parametrize("S,M,world,rank,draw", [
    (128, 100, 1, 0, True),     # C3: two roles per sample, one chunk
    (256, 200, 1, 0, False),    # looped chunks (M = 200), one role
    (256, 100, 2, 1, True),     # several sources: the band table, two roles
    (1024, 200, 8, 3, False),   # C4 at W = 8: band table, two roles, looped chunks
    (128, 97, 1, 0, False),     # a ragged chunk (Mp = 112 still)
])
def test_fixed_geometry_equals_runtime(S, M, world, rank, draw):
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan("fullcov", FN2, S, M, world=world, rank=rank)
    g = torch.Generator().manual_seed(S + M + rank)
    u = torch.randn(M, 64, generator=g).to(DEV)
    z = torch.randint(0, 2, (M,), generator=g).to(torch.int32).to(DEV)
    w = (torch.rand(M, generator=g) * 10 + 1).to(DEV)
    xs = (0.2 * torch.randn(plan.xrecv_count, generator=g)).to(DEV)
    a = _net(plan, u, z, w, xs, draw, False)
    b = _net(plan, u, z, w, xs, draw, True)
    assert torch.isfinite(a[0]).all(), "a gradient element left unwritten"
    assert torch.equal(a[0], b[0])
    # (the NLL: one fp64 atomic add per workgroup, in arrival order)
    assert abs(a[1].item() - b[1].item()) <= 1e-12 * abs(b[1].item())
    if draw:
        assert torch.equal(a[2], b[2])
