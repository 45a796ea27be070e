"""Conjugate gradient over lists of tensors (the solver behind
psvi.hypergrad.CG / CG_normaleq; reference: psvi/hypergrad/CG_torch.py:9-45).

``cg(Ax, b, max_iter, epsilon)`` runs at most ``max_iter`` iterations from
x = 0 and returns the last iterate before the residual norm fell below
``epsilon`` (the reference's convention: on convergence the returned x is the
one from the previous iteration)."""
import torch

__all__ = ["cg", "cat_list_to_tensor"]


def cat_list_to_tensor(list_tx):
    return torch.cat([t.reshape(-1) for t in list_tx])


def cg(Ax, b, max_iter=100, epsilon=1.0e-5):
    x = [torch.zeros_like(t) for t in b]
    r = [t.clone() for t in b]
    p = [t.clone() for t in r]
    for _ in range(max_iter):
        Ap = Ax(p)
        rr = torch.sum(cat_list_to_tensor(r) ** 2)
        alpha = rr / torch.sum(cat_list_to_tensor(p) * cat_list_to_tensor(Ap))
        x_new = [xi + alpha * pi for xi, pi in zip(x, p)]
        r_new = [ri - alpha * api for ri, api in zip(r, Ap)]
        rn = cat_list_to_tensor(r_new)
        if float(torch.linalg.vector_norm(rn)) < epsilon:
            break
        beta = torch.sum(rn * rn) / rr
        p = [ri + beta * pi for ri, pi in zip(r_new, p)]
        x, r = x_new, r_new
    return x
