"""Conjugate gradient over lists of tensors (the solver behind
psvi.hypergrad.CG / CG_normaleq; reference: psvi/hypergrad/CG_torch.py:9-45).

``cg(Ax, b, max_iter, epsilon)`` runs at most ``max_iter`` iterations from
x = 0 and returns the last iterate before the residual norm fell below
``epsilon`` (the reference's convention: on convergence the returned x is the
one from the previous iteration), after as many Ax calls as the reference
makes (``sync_every`` = 1)."""
import torch

__all__ = ["cg", "cat_list_to_tensor"]


def cat_list_to_tensor(list_tx):
    return torch.cat([t.reshape(-1) for t in list_tx])


def cg(Ax, b, max_iter=100, epsilon=1.0e-5, sync_every=1):
    """The reference's iteration on one flat buffer per vector (the lists Ax
    sees are views into it), with its stopping test evaluated on the device:
    once ||r_new|| < epsilon the iterate, the residual and the direction
    freeze (torch.where) -- x is the one the reference's ``break`` returns,
    and values computed after convergence (possibly inf / NaN: A need not be
    SPD) never reach it.  The host reads the flag every ``sync_every``
    iterations and leaves the loop once it is set; with the default 1 that is
    the reference's exit (the same number of Ax calls -- a stochastic Ax draws
    the same noise).  A larger value trades the host round trip per
    iteration (on a GPU the device otherwise idles once per iteration) for up
    to sync_every - 1 discarded Ax calls after convergence."""
    shapes = [t.shape for t in b]
    sizes = [t.numel() for t in b]

    def flat(ts):
        return cat_list_to_tensor(ts) if len(ts) > 1 else ts[0].reshape(-1)

    def views(v):
        return [c.view(sh) for c, sh in zip(torch.split(v, sizes), shapes)]

    # per iteration: two dots and the fused x + a y passes; alpha / beta stay
    # 0-dim device tensors; where the reference breaks, the step length is
    # zeroed (x keeps its value) and r, p, rr keep theirs
    r = flat(b).clone()
    x = torch.zeros_like(r)
    p = r.clone()
    rr = torch.dot(r, r)
    done = torch.zeros((), dtype=torch.bool, device=r.device)
    zero = torch.zeros((), dtype=r.dtype, device=r.device)
    sync_every = max(1, int(sync_every))
    for it in range(max_iter):
        Ap = flat(Ax(views(p)))
        alpha = rr / torch.dot(p, Ap)
        rn = torch.dot(r_new := torch.addcmul(r, alpha, Ap, value=-1), r_new)
        done = done | (torch.sqrt(rn) < epsilon)
        x = torch.addcmul(x, torch.where(done, zero, alpha), p)
        r = torch.where(done, r, r_new)
        p = torch.where(done, p, torch.addcmul(r, rn / rr, p))
        rr = torch.where(done, rr, rn)
        if (it + 1) % sync_every == 0 and bool(done):
            break
    return views(x)
