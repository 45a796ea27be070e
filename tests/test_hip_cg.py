"""The fused conjugate-gradient iteration of hyper_step (psvi_cg_*,
psvi.runtime.cg.DeviceCG) against the reference's cg loop
(psvi/hypergrad/CG_torch.py:21-43) on CG_normaleq's operator
(hypergradients.py:217-230: A(p) = vmj - J vmj, vmj = lr H_A p, J y = y - lr
H_B y), with explicit fp32 matrices standing in for the two Hessian-vector
products: the same products, the same number of operator calls, x within
float64 summation order; the iterate before the residual test fired when it
fires; nothing non-finite reaches x after convergence."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops(n, seed, indefinite=False):
    g = torch.Generator().manual_seed(seed)
    Q = torch.randn(n, n, generator=g, dtype=torch.float64)
    HA = (Q @ Q.T / n + torch.eye(n, dtype=torch.float64))
    HB = HA + 0.01 * torch.randn(n, n, generator=g, dtype=torch.float64)
    if indefinite:
        HA = HA - 1.5 * torch.eye(n, dtype=torch.float64)
    return HA.float().to(DEV), HB.float().to(DEV)


def _reference(HA, HB, b, lr, K, tol):
    """CG_torch.cg on A(p) = vmj - (vmj - lr H_B float(vmj)), vmj = lr H_A float(p)
    (the fp32 products promoted as psvi_classes' torch formulation did)."""
    calls = [0]

    def A(p):
        calls[0] += 1
        vmj = (HA @ p.float()).double() * lr
        return vmj - torch.sub(vmj, (HB @ vmj.float()).double(), alpha=lr)

    x, r, p = torch.zeros_like(b), b.clone(), b.clone()
    for _ in range(K):
        Ap = A(p)
        rTr = r @ r
        alpha = rTr / (p @ Ap)
        xn, rn = x + alpha * p, r - alpha * Ap
        if float(torch.norm(rn)) < tol:
            break
        p = rn + (rn @ rn) / rTr * p
        x, r = xn, rn
    return x, calls[0]


@pytest.mark.parametrize("n,K,tol,indef", [(3001, 12, 1e-10, False), (3001, 60, 1e-6, False),
                                           (777, 40, 1e-10, True)])
def test_device_cg_equals_reference_loop(n, K, tol, indef):
    from psvi.runtime.cg import DeviceCG

    HA, HB = _ops(n, n + K, indef)
    g = torch.Generator().manual_seed(1)
    b = torch.randn(n, generator=g, dtype=torch.float64).to(DEV)
    lr = 0.3
    xr, calls = _reference(HA, HB, b, lr, K, tol)
    ncall = [0]

    def hv_a(x32):
        ncall[0] += 1
        return HA @ x32

    def hv_b(x32):
        return HB @ x32

    cg = DeviceCG(n, DEV)
    x = cg.solve(hv_a, hv_b, b, lr, K, tol=tol, sync_every=1)
    torch.cuda.synchronize()
    assert ncall[0] == calls, (ncall[0], calls)   # the reference's exit: same operator calls
    assert torch.isfinite(x).all() == torch.isfinite(xr).all()
    if torch.isfinite(xr).all():
        err = float((x - xr).norm() / xr.norm())
        print(f"n {n} K {K} tol {tol}: {calls} operator calls, rel l2 {err:.2e}")
        # (an indefinite operator amplifies the dots' summation order over 40
        # iterations: the iterates agree to that conditioning only)
        assert err < (1e-4 if indef else 1e-9)
    # a host read every 4 iterations: the same x (frozen), up to 3 more calls
    ncall[0] = 0
    x4 = cg.solve(hv_a, hv_b, b, lr, K, tol=tol, sync_every=4)
    torch.cuda.synchronize()
    assert torch.allclose(x4, x, rtol=0, atol=0, equal_nan=True)
    assert calls <= ncall[0] < calls + 4 or ncall[0] == K


def test_device_cg_is_deterministic():
    from psvi.runtime.cg import DeviceCG

    n = 20001
    HA, HB = _ops(1000, 3)
    HA = torch.block_diag(*([HA] * 20 + [torch.ones(1, 1, device=DEV)]))
    HB = HA
    b = torch.randn(n, dtype=torch.float64, device=DEV)
    cg = DeviceCG(n, DEV)
    a = cg.solve(lambda v: HA @ v, lambda v: HB @ v, b, 0.5, 8)
    c = cg.solve(lambda v: HA @ v, lambda v: HB @ v, b, 0.5, 8)
    torch.cuda.synchronize()
    assert torch.equal(a, c)
