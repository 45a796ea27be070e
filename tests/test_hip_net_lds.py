"""The network kernel's padding contract (kernels_net.hip header): every LDS
word a GEMM reads is written by the kernel itself (zero fill, loads,
epilogues) or multiplies a zero weight.  Checked by running the kernel after
another kernel left NaN / 1e30 in the LDS of every CU (a large torch GEMM on
NaN-filled operands stages its tiles there): the outputs must equal, bit for
bit, those of a run after a zero-filled GEMM.  Also the run-to-run
determinism of the gradients (plain stores, one writer per element; the
mean-field slots are summed in a fixed order)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pollute(fill):
    a = torch.full((4096, 4096), fill, device=DEV)
    (a @ a).sum()  # tiles of `fill` staged through the LDS of every CU
    torch.cuda.synchronize()


@pytest.mark.parametrize("layers,S,M", [
    ([(64, 40), (40, 40), (40, 2)], 128, 100),   # C3: two role workgroups per sample
    ([(64, 40), (40, 40), (40, 2)], 1024, 200),  # C4 shape: one workgroup per sample
    ([(9, 5), (5, 3)], 40, 7),
    ([(33, 17), (17, 5)], 6, 37)])               # odd widths: row overruns into padding
def test_fullcov_net_ignores_stale_lds(layers, S, M):
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan("fullcov", layers, S, M)
    g = torch.Generator().manual_seed(3)
    u = torch.randn(M, layers[0][0], generator=g).to(DEV)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).to(DEV)
    w = torch.full((M,), 8.0, device=DEV)
    xs = (0.1 * torch.randn(plan.xshard_count, generator=g)).to(DEV)
    outs = []
    for fill in (0.0, float("nan"), 1e30, 0.0):
        _pollute(fill)
        gs = torch.zeros(plan.xshard_count, device=DEV)
        nll = torch.zeros(1, dtype=torch.float64, device=DEV)
        plan.mvn_net(u, z, w, xs, gs, nll)
        torch.cuda.synchronize()
        outs.append((gs.cpu().numpy(), nll.item()))
    g0 = outs[0][0]
    assert np.isfinite(g0).all()
    for gk, nk in outs[1:]:
        assert np.array_equal(gk, g0)
        assert abs(nk - outs[0][1]) <= 1e-12 * abs(outs[0][1])  # fp64 atomics: order only


@pytest.mark.parametrize("layers,S,M", [([(2, 100), (100, 4)], 32, 50), ([(5, 7), (7, 3)], 8, 19)])
def test_meanfield_net_ignores_stale_lds(layers, S, M):
    from psvi.runtime import InnerLoopPlan, randn_

    plan = InnerLoopPlan("meanfield", layers, S, M)
    g = torch.Generator().manual_seed(4)
    u = torch.randn(M, layers[0][0], generator=g).to(DEV)
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).to(DEV)
    w = torch.full((M,), 8.0, device=DEV)
    params = (0.1 * torch.randn(plan.param_count, generator=g)).to(DEV)
    eps = randn_(torch.empty(plan.eps_count, device=DEV), 5)
    outs = []
    for fill in (0.0, float("nan"), 1e30):
        _pollute(fill)
        acc = torch.empty(plan.acc_count, device=DEV)
        nll = torch.zeros(1, dtype=torch.float64, device=DEV)
        plan.mf_accumulate(u, z, w, eps, params, acc, nll)
        torch.cuda.synchronize()
        outs.append(acc.cpu().numpy())
    assert np.isfinite(outs[0]).all()
    for a in outs[1:]:  # per-(sample, chunk) slots summed in a fixed order: bitwise
        assert np.array_equal(a, outs[0])


@pytest.mark.parametrize("fam,layers,S,M", [
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 128, 100),
    ("fullcov", [(64, 40), (40, 40), (40, 2)], 1024, 200),
    ("fullcov", [(9, 5), (5, 3)], 130, 129),
    ("meanfield", [(7, 33), (33, 5), (5, 3)], 130, 129),
    ("meanfield", [(7, 33), (33, 5), (5, 3)], 256, 129),
    ("meanfield", [(64, 64), (64, 10)], 16, 200)])
def test_net_reads_only_lds_it_wrote(fam, layers, S, M):
    """The network kernel with its whole LDS poisoned with NaN before use
    (diagnostics ablation bit 128) gives the same ELBO and gradient bit for
    bit: no word is read before the kernel writes it -- in particular the
    row chain's k-loops that run past a row's end into rows another wave owns
    (masked to zero in the last k-group).  LDS keeps whatever an earlier
    kernel left there, NaN included."""
    import torch

    from psvi.runtime import InnerLoopPlan

    g = torch.Generator().manual_seed(S + M)
    plan = InnerLoopPlan(fam, layers, S, M)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        if fam == "meanfield":
            parts += [0.3 * torch.randn(n, generator=g), -4 + 3 * torch.rand(n, generator=g)]
        else:
            parts += [0.1 * torch.randn(n, generator=g), -5 + 2 * torch.rand(n, generator=g),
                      (0.15 / n ** 0.5) * torch.randn((n - 1) * (n - 2) // 2, generator=g)]
    p = torch.cat(parts).cuda()
    u = torch.randn(M, layers[0][0], generator=g).cuda()
    z = torch.randint(0, layers[-1][1], (M,), generator=g).to(torch.int32).cuda()
    w = torch.full((M,), 3.0).cuda()
    eps = torch.randn(plan.eps_count, generator=g).cuda()
    out = []
    for abl in (0, 128, 0):
        plan.lib.psvi_debug_set(1, abl)
        try:
            e, gr = plan.elbo_grad(u, z, w, eps, p)
            torch.cuda.synchronize()
        finally:
            plan.lib.psvi_debug_set(1, 0)
        out.append((e.item(), gr.cpu()))
    for e, gr in out:
        assert e == e and torch.isfinite(gr).all()
        # the ELBO's fp64 partials are added with atomics in arrival order
        assert abs(e - out[0][0]) <= 1e-12 * abs(out[0][0])
        assert torch.equal(gr, out[0][1])
