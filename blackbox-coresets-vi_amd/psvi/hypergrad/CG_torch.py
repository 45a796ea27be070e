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
    """The reference's iteration on one flat buffer per vector (the lists Ax
    sees are views into it), with its stopping test kept on the device: once
    ||r_new|| < epsilon the iterate freezes (torch.where) -- the same x the
    reference's ``break`` returns -- so no iteration waits on a host read of
    the norm.  After convergence the remaining iterations still evaluate Ax
    (discarded); on a GPU the host otherwise idles the device once per
    iteration (the fused HVPs take ~0.13 ms, the round trip about as long)."""
    shapes = [t.shape for t in b]
    sizes = [t.numel() for t in b]

    def flat(ts):
        return cat_list_to_tensor(ts) if len(ts) > 1 else ts[0].reshape(-1)

    def views(v):
        return [c.view(sh) for c, sh in zip(torch.split(v, sizes), shapes)]

    # per iteration six passes over the vectors (two dots, four fused
    # x + a y): alpha / beta stay 0-dim device tensors; where the reference
    # breaks, the step length is zeroed instead (x and r keep their values;
    # p no longer enters them)
    r = flat(b).clone()
    x = torch.zeros_like(r)
    p = r.clone()
    rr = torch.dot(r, r)
    done = torch.zeros((), dtype=torch.bool, device=r.device)
    zero = torch.zeros((), dtype=r.dtype, device=r.device)
    for _ in range(max_iter):
        Ap = flat(Ax(views(p)))
        alpha = rr / torch.dot(p, Ap)
        rn = torch.dot(r_new := torch.addcmul(r, alpha, Ap, value=-1), r_new)
        done = done | (torch.sqrt(rn) < epsilon)
        a_eff = torch.where(done, zero, alpha)
        x = torch.addcmul(x, a_eff, p)
        r = torch.where(done, r, r_new)
        p = torch.addcmul(r, rn / rr, p)
        rr = torch.where(done, rr, rn)
    return views(x)
