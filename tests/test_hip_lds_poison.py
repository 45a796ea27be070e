"""Stale-LDS contract of the kernels beyond the network kernel
(test_hip_net_lds.py): every LDS word a kernel reads it wrote itself, or it
multiplies a zero.  Each entry point runs after another kernel left NaN /
1e30 in the LDS of every CU (a large torch GEMM on filled operands stages its
tiles there) and must give, bit for bit, what it gives after a zero-filled
one.  Covered: the bf16-piece streaming update (psvi_inner_loop, C3), the
K-split update and the segmented sample (S > 128, both the bf16-piece and the
fp32 kernels), the R-op / HVP kernels (full-cov and LeNet) and the LeNet
inner step.  The same k-contiguous over-read that the round-4 row chain
introduced (a GEMM's last k-group past a row's end) would show here as NaN."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
FN2 = [(64, 40), (40, 40), (40, 2)]
LENET = [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]


def _pollute(fill):
    a = torch.full((4096, 4096), fill, device=DEV)
    (a @ a).sum()  # tiles of `fill` staged through the LDS of every CU
    torch.cuda.synchronize()


def _same_after_pollution(fn, approx=()):
    """fn() -> list of numpy arrays; run after 0 / NaN / 1e30 / 0 pollution.
    Outputs at the indices `approx` are float64 accumulators summed by
    atomics (order only: 1e-12 relative), the rest must be bitwise equal."""
    outs = []
    for fill in (0.0, float("nan"), 1e30, 0.0):
        _pollute(fill)
        outs.append([np.asarray(x) for x in fn()])
        torch.cuda.synchronize()
    for o in outs[0]:
        assert np.isfinite(o).all()
    for k, o in enumerate(outs[1:], 1):
        for i, (a, b) in enumerate(zip(o, outs[0])):
            if i in approx:
                assert np.allclose(a, b, rtol=1e-12, atol=0), (k, i, a, b)
            else:
                assert np.array_equal(a, b), (k, i, np.nanmax(np.abs(a - b)))


def _fullcov_state(layers, seed):
    rng = np.random.default_rng(seed)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
                  (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
    return rng, torch.tensor(np.concatenate(parts).astype(np.float32), device=DEV)


@pytest.mark.parametrize("layers,S", [(FN2, 128), ([(7, 5), (5, 3)], 128), ([(30, 33), (33, 2)], 64)])
def test_inner_loop_ignores_stale_lds(layers, S):
    """psvi_inner_loop (tiled state: the bf16-piece streaming update at S = 128,
    the fp32 one at S = 64), Philox draws, 3 steps."""
    from psvi.runtime import InnerLoopPlan

    M = 24
    plan = InnerLoopPlan("fullcov", layers, S, M)
    rng, p0 = _fullcov_state(layers, 1)
    u = torch.tensor(rng.standard_normal((M, layers[0][0])).astype(np.float32), device=DEV)
    z = torch.tensor(rng.integers(0, layers[-1][1], M).astype(np.int32), device=DEV)
    w = torch.full((M,), 8.0, device=DEV)

    def run():
        p = p0.clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        e = plan.inner_loop(u, z, w, p, m, v, 3, 1e-3, seed=4)
        return [t.cpu().numpy() for t in (e, p, m, v)]

    _same_after_pollution(run, approx=(0,))


@pytest.mark.parametrize("W,S", [(1, 300), (8, 1024), (2, 256)])
@pytest.mark.parametrize("bf_off", [0, 1])
def test_kstream_and_segmented_sample_ignore_stale_lds(W, S, bf_off):
    """The update with the next sample at K = S > 128 (psvi_mvn_phase_update_sample:
    mvn_kstream_kernel + the segmented sample), bf16-piece (default) and fp32
    kernels, a rank of a world-W plan."""
    from psvi.runtime import InnerLoopPlan

    rng, p0 = _fullcov_state(FN2, 2)
    r = W - 1
    plan = InnerLoopPlan("fullcov", FN2, S, 100, world=W, rank=r)
    g = torch.tensor((0.05 * rng.standard_normal(plan.xshard_count)).astype(np.float32), device=DEV)
    eps = torch.tensor(rng.standard_normal(plan.eps_count).astype(np.float32), device=DEV)
    eps2 = torch.tensor(rng.standard_normal(plan.eps_count).astype(np.float32), device=DEV)
    plan.lib.psvi_debug_set(26, bf_off)
    plan.lib.psvi_debug_set(27, bf_off)
    try:
        def run():
            p = p0.clone()
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            x = torch.zeros(plan.xshard_count, device=DEV)
            kl = torch.zeros(1, dtype=torch.float64, device=DEV)
            plan.mvn_update(eps, g, p, m, v, step=2, lr=1e-3, kl_out=kl, eps_next=eps2, x_next=x)
            return [t.cpu().numpy() for t in (p, m, v, x)]

        _same_after_pollution(run)
    finally:
        plan.lib.psvi_debug_set(26, 0)
        plan.lib.psvi_debug_set(27, 0)


@pytest.mark.parametrize("layers,S,M", [(FN2, 128, 100), ([(33, 17), (17, 5)], 6, 37)])
def test_fullcov_hvp_ignores_stale_lds(layers, S, M):
    """psvi_hvp (the tangent sample, net_rop_kernel, the R-backward and its
    assembly) with the mixed products."""
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan("fullcov", layers, S, M)
    rng, p = _fullcov_state(layers, 3)
    u = torch.tensor(rng.standard_normal((M, layers[0][0])).astype(np.float32), device=DEV)
    z = torch.tensor(rng.integers(0, layers[-1][1], M).astype(np.int32), device=DEV)
    w = torch.full((M,), 8.0, device=DEV)
    eps = torch.tensor(rng.standard_normal(plan.eps_count).astype(np.float32), device=DEV)
    vec = torch.tensor((1e-2 * rng.standard_normal(plan.param_count)).astype(np.float32), device=DEV)

    def run():
        hv, du, dw = plan.hvp(u, z, w, eps, p, vec)
        return [t.cpu().numpy() for t in (hv, du, dw)]

    _same_after_pollution(run)


@pytest.mark.parametrize("S,M", [(4, 6), (3, 17)])
def test_lenet_step_and_hvp_ignore_stale_lds(S, M):
    """LeNet (the conv towers on MFMA, their backward, the tangent kernels):
    one inner step and one HVP."""
    from psvi.runtime import InnerLoopPlan

    plan = InnerLoopPlan("lenet", LENET, S, M)
    g = torch.Generator().manual_seed(5)
    u = torch.randn(M, 784, generator=g).to(DEV)
    z = torch.randint(0, 10, (M,), generator=g).to(torch.int32).to(DEV)
    w = torch.full((M,), 4.0, device=DEV)
    p0 = (0.05 * torch.randn(plan.param_count, generator=g)).to(DEV)
    eps = torch.randn(plan.eps_count, generator=g).to(DEV)
    vec = (1e-2 * torch.randn(plan.param_count, generator=g)).to(DEV)

    def run():
        p = p0.clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        e = plan.inner_step(u, z, w, eps, p, m, v, 1, 1e-3)
        hv, du, dw = plan.hvp(u, z, w, eps, p0, vec)
        return [t.cpu().numpy() for t in (e, p, hv, du, dw)]

    _same_after_pollution(run, approx=(0,))
