"""psvi.hypergrad's generic (torch autograd) paths on CPU: the hypergradient
approximations of the reference's psvi/hypergrad/hypergradients.py against
the closed-form implicit hypergradient of a quadratic bilevel problem, the
conjugate-gradient solver, and the differentiable optimisers' arithmetic
(diff_optimizers.py: hypergrad's Adam stores v + 1e-12)."""
import numpy as np
import pytest
import torch


def _problem(seed=0, n=6, k=3):
    g = torch.Generator().manual_seed(seed)
    Q = torch.randn(n, n, generator=g, dtype=torch.float64)
    A = Q @ Q.T / n + torch.eye(n, dtype=torch.float64)          # SPD, eigenvalues >= 1
    B = torch.randn(k, n, generator=g, dtype=torch.float64)
    c = torch.randn(n, generator=g, dtype=torch.float64)
    lam = torch.randn(k, generator=g, dtype=torch.float64).requires_grad_(True)

    def inner(params, hparams):
        w, = params
        return 0.5 * w @ A @ w - hparams[0] @ B @ w

    def outer(params, hparams):
        w, = params
        return 0.5 * ((w - c) ** 2).sum() + 0.05 * (hparams[0] ** 2).sum()

    w_star = torch.linalg.solve(A, B.T @ lam.detach())
    exact = 0.1 * lam.detach() + B @ torch.linalg.solve(A, w_star - c)
    return A, inner, outer, lam, w_star, exact


@pytest.mark.parametrize("method,K,tol", [("CG_normaleq", 6, 0.0), ("CG", 6, 0.0),
                                          ("fixed_point", 3000, 1e-14), ("neumann", 3000, 1e-14)])
def test_implicit_hypergradient_of_a_quadratic(method, K, tol):
    """CG / CG_normaleq: n = 6 iterations solve the 6 x 6 system exactly (with
    tol = 0: on reaching tol the reference's cg returns the iterate BEFORE
    the converged one, CG_torch.py:26-44); fixed_point / neumann: the series."""
    import psvi.hypergrad as H

    A, inner, outer, lam, w_star, exact = _problem()
    lr = 0.5 / float(torch.linalg.eigvalsh(A).max())
    fp = H.GradientDescent(inner, step_size=lr)
    fn = getattr(H, method)
    kw = {} if method in ("CG_normaleq", "neumann") else {"stochastic": False}
    grads = fn([w_star.clone()], [lam], K=K, fp_map=fp, outer_loss=outer, tol=tol, **kw)
    assert torch.allclose(grads[0].double(), exact, rtol=1e-6, atol=1e-8), (grads[0], exact)
    assert torch.allclose(lam.grad, exact, rtol=1e-6, atol=1e-8)


def test_reverse_unroll_and_reverse_agree():
    """reverse (recomputing each update map) equals reverse_unroll (backprop
    through the stored unroll) on the same gradient-descent trajectory."""
    import psvi.hypergrad as H

    A, inner, outer, lam, _, _ = _problem(1)
    lr = 0.3 / float(torch.linalg.eigvalsh(A).max())
    fp = H.GradientDescent(inner, step_size=lr)
    hist = [[torch.zeros(A.shape[0], dtype=torch.float64, requires_grad=True)]]
    for _ in range(20):
        hist.append(fp(hist[-1], [lam], create_graph=True))
    g_unroll = [g.clone() for g in H.reverse_unroll(hist[-1], [lam], outer, set_grad=False)]
    g_rev = H.reverse(hist, [lam], [fp] * 20, outer, set_grad=False)
    assert torch.allclose(g_unroll[0], g_rev[0], rtol=1e-10, atol=1e-12)


def test_cg_solves_spd_system_and_keeps_previous_iterate_on_convergence():
    from psvi.hypergrad.CG_torch import cg

    A, _, _, _, _, _ = _problem(2)
    b = torch.arange(1.0, A.shape[0] + 1, dtype=torch.float64)
    Ax = lambda xs: [A @ xs[0]]
    x = cg(Ax, [b], max_iter=6, epsilon=0.0)[0]          # n = 6: exact in n steps
    assert torch.allclose(A @ x, b, rtol=1e-9, atol=1e-9)
    # reaching epsilon returns the iterate before the one that did
    xe = cg(Ax, [b], max_iter=50, epsilon=1e-8)[0]
    prev = [cg(Ax, [b], max_iter=j, epsilon=0.0)[0] for j in range(1, 7)]
    assert any(torch.equal(xe, xp) for xp in prev[:-1])
    assert not torch.allclose(A @ xe, b, rtol=1e-9, atol=1e-9)
    x1 = cg(lambda xs: [A @ xs[0]], [b], max_iter=1, epsilon=0.0)[0]
    alpha = (b @ b) / (b @ A @ b)
    assert torch.allclose(x1, alpha * b)


def test_cg_after_convergence_stays_finite_and_calls_ax_like_the_reference():
    """max_iter >> n on a non-symmetric, indefinite A: once the residual test
    fires, the iterate is the reference's (the one before), nothing computed
    after convergence reaches it (no inf / NaN), and with sync_every = 1 Ax is
    called exactly as often as the reference's loop calls it (CG_torch.py:21-37:
    a stochastic Ax draws the same noise)."""
    from psvi.hypergrad.CG_torch import cg

    g = torch.Generator().manual_seed(11)
    n = 5
    A = torch.randn(n, n, generator=g, dtype=torch.float64)   # non-symmetric, indefinite
    b = torch.randn(n, generator=g, dtype=torch.float64)

    def ref_cg(Ax, b, max_iter, eps):
        x, r, p = torch.zeros_like(b), b.clone(), b.clone()
        calls = 0
        for _ in range(max_iter):
            Ap = Ax(p)
            calls += 1
            rTr = r @ r
            alpha = rTr / (p @ Ap)
            xn, rn = x + alpha * p, r - alpha * Ap
            if float(torch.norm(rn)) < eps:
                break
            p = rn + (rn @ rn) / rTr * p
            x, r = xn, rn
        return x, calls

    # an SPD system solved to round-off, then 200 more iterations
    S = A @ A.T + n * torch.eye(n, dtype=torch.float64)
    # S: converges in ~n iterations, then 190+ iterations of A(p) on a
    # vanishing residual (p.Ap -> 0: inf / NaN step lengths that must not
    # reach x); A with a residual test: the reference's break; A with eps 0:
    # no break, both run all iterations
    for M, eps in ((S, 1e-9), (A, 1e-6), (A, 0.0)):
        ncall = [0]

        def Ax(xs, M=M):
            ncall[0] += 1
            return [M @ xs[0]]

        x = cg(Ax, [b], max_iter=200, epsilon=eps)[0]
        xr, calls = ref_cg(lambda v, M=M: M @ v, b, 200, eps)
        # the reference's loop may itself break down on an indefinite A (p.Ap
        # = 0 before any residual test fires): then both agree on non-finite
        assert bool(torch.isfinite(x).all()) == bool(torch.isfinite(xr).all())
        if torch.isfinite(xr).all():
            assert torch.allclose(x, xr, rtol=1e-9, atol=1e-12)
        if eps > 0 and M is S:
            assert ncall[0] == calls < 200    # the reference's exit
        # a host read every 8 iterations: at most 7 Ax calls more, same x
        ncall[0] = 0
        x8 = cg(Ax, [b], max_iter=200, epsilon=eps, sync_every=8)[0]
        assert torch.allclose(x8, x, rtol=0, atol=0, equal_nan=True)
        if eps > 0 and M is S:
            assert calls <= ncall[0] < calls + 8


def test_hypergrad_adam_step_arithmetic():
    """adam_step (diff_optimizers.py:184-213): v stored with + 1e-12,
    w' = w - lr (m'/(1-b1^t)) / (sqrt(v'/(1-b2^t)) + eps); DifferentiableAdam
    carries [p, m, v] and advances its step count."""
    import psvi.hypergrad as H

    g = torch.Generator().manual_seed(3)
    w0 = torch.randn(5, generator=g, dtype=torch.float64).requires_grad_(True)
    target = torch.randn(5, generator=g, dtype=torch.float64)
    loss_f = lambda params, hp: ((params[0] - target) ** 2).sum()
    opt = H.DifferentiableAdam(loss_f, step_size=0.1)
    state = opt.get_opt_params([w0])
    assert len(state) == 3 and torch.equal(state[1], torch.zeros(5, dtype=torch.float64))
    p, m, v = w0.detach().numpy().copy(), np.zeros(5), np.zeros(5)
    for t in range(1, 4):
        state = opt(state, [], create_graph=False)
        grad = 2 * (p - target.numpy())
        m = 0.9 * m + 0.1 * grad
        v = 0.999 * v + 0.001 * grad ** 2 + 1e-12
        p = p - 0.1 * (m / (1 - 0.9 ** t)) / (np.sqrt(v / (1 - 0.999 ** t)) + 1e-8)
        assert np.allclose(state[0].detach().numpy(), p, rtol=1e-12, atol=1e-14)
        assert np.allclose(state[2].detach().numpy(), v, rtol=1e-12, atol=1e-20)
    assert opt.step_cnt == 4


def test_momentum_and_heavy_ball_steps():
    import psvi.hypergrad as H

    w = torch.tensor([1.0, -2.0], dtype=torch.float64, requires_grad=True)
    loss_f = lambda params, hp: (params[0] ** 2).sum()
    mom = H.Momentum(loss_f, step_size=0.1, momentum=0.5)
    st = mom([w, torch.tensor([0.2, 0.2], dtype=torch.float64)], [], create_graph=False)
    vel = 0.5 * torch.tensor([0.2, 0.2], dtype=torch.float64) + 2 * w.detach()
    assert torch.allclose(st[1], vel) and torch.allclose(st[0], w.detach() - 0.1 * vel)
    hb = H.HeavyBall(loss_f, step_size=0.1, momentum=0.5)
    prev = torch.tensor([0.5, -1.0], dtype=torch.float64)
    st = hb([w, prev], [], create_graph=False)
    assert torch.allclose(st[0], w.detach() - 0.2 * w.detach() + 0.5 * (w.detach() - prev))
    assert torch.equal(st[1], w)
