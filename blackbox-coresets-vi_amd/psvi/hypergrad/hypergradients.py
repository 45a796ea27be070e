"""psvi.hypergrad's hypergradient approximations (reference:
psvi/hypergrad/hypergradients.py:14-349) on the HIP inner objective.

Every method keeps the reference's signature, draw order and result: the
outer objective's direct gradients, then a linear solve against the
fixed-point map ``fp_map`` (a psvi.hypergrad optimiser over PSVI.inner_elbo),
then the mixed product ``torch.autograd.grad(w_mapped, hparams, v)``.  With
the map a ``GradientDescent`` over a HIP objective, the products the
reference takes by double backward are psvi_hvp calls: ``J^T v`` through the
map's autograd node (diff_optimizers._HipGradStep), ``J v`` (``jvp``) by the
same product, J = I - lr H being symmetric -- evaluated, like the
reference's jvp, on the SECOND of two fresh evaluations of the map (each one
a new draw of the inner objective's noise).

The linear solves (fixed_point, CG, CG_normaleq, neumann) run their vectors
in float64 (the Hessian-vector products themselves are fp32 on the GPU), as
PSVI.hyper_step does: the reference's fp32 CG after K = 30 iterations sits
1e-5 .. 1e-4 from its own float64 run."""
import torch
from torch.autograd import grad as torch_grad

from . import CG_torch
from .diff_optimizers import hip_jvp, params_only

__all__ = ["reverse_unroll", "reverse", "fixed_point", "CG", "CG_normaleq", "neumann", "exact",
           "grd", "list_dot", "jvp", "get_outer_gradients", "cat_list_to_tensor",
           "update_tensor_grads", "grad_unused_zero"]


def _f64(ts):
    return [t.detach().to(torch.float64) for t in ts]


def _like(ts, ref):
    return [t.to(r.dtype) for t, r in zip(ts, ref)]


def _norm(ts):
    return float(torch.linalg.vector_norm(cat_list_to_tensor(ts)))


def reverse_unroll(params, hparams, outer_loss, set_grad=True):
    """hypergradients.py:14-35: backpropagation through the stored unroll."""
    o_loss = outer_loss(params, hparams)
    grads = torch.autograd.grad(o_loss, hparams, retain_graph=True)
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


def reverse(params_history, hparams, update_map_history, outer_loss, set_grad=True):
    """hypergradients.py:38-80: reverse mode recomputing each update map from
    the stored iterates (truncated when given part of the trajectory)."""
    hist = [[w.detach().requires_grad_(True) for w in ps] for ps in params_history]
    o_loss = outer_loss(hist[-1], hparams)
    g_w, g_h = get_outer_gradients(o_loss, hist[-1], hparams)
    alphas = g_w
    grads = [torch.zeros_like(h) for h in hparams]
    K = len(hist) - 1
    for k in range(-2, -(K + 2), -1):
        w_mapped = update_map_history[k + 1](hist[k], hparams)
        bs = grad_unused_zero(w_mapped, hparams, grad_outputs=alphas, retain_graph=True)
        grads = [g + b for g, b in zip(grads, bs)]
        with params_only(w_mapped):
            alphas = torch_grad(w_mapped, hist[k], grad_outputs=alphas)
    grads = [g + v for g, v in zip(grads, g_h)]
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


def fixed_point(params, hparams, K, fp_map, outer_loss, tol=1e-10, set_grad=True,
                stochastic=False):
    """hypergradients.py:83-140: v <- J^T v + d outer / d w, K times (or until
    two iterates are within tol); stochastic=True draws a new map per
    iteration and one more for the mixed product."""
    params = [w.detach().requires_grad_(True) for w in params]
    o_loss = outer_loss(params, hparams)
    g_w, g_h = get_outer_gradients(o_loss, params, hparams)
    g64 = _f64(g_w)
    w_mapped = None if stochastic else fp_map(params, hparams)
    vs = [torch.zeros_like(g) for g in g64]
    for _ in range(K):
        prev = vs
        if stochastic:
            w_mapped = fp_map(params, hparams)
        with params_only(w_mapped):
            jt = torch_grad(w_mapped, params, grad_outputs=_like(vs, w_mapped),
                            retain_graph=not stochastic)
        vs = [j.to(torch.float64) + g for j, g in zip(jt, g64)]
        if _norm([a - b for a, b in zip(vs, prev)]) < tol:
            break
    if stochastic:
        w_mapped = fp_map(params, hparams)
    grads = torch_grad(w_mapped, hparams, grad_outputs=_like(vs, w_mapped), allow_unused=True)
    grads = [g + v if g is not None else v for g, v in zip(grads, g_h)]
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


def CG(params, hparams, K, fp_map, outer_loss, tol=1e-10, set_grad=True, stochastic=False):
    """hypergradients.py:143-196: K conjugate-gradient steps on
    (I - J^T) v = d outer / d w."""
    params = [w.detach().requires_grad_(True) for w in params]
    o_loss = outer_loss(params, hparams)
    g_w, g_h = get_outer_gradients(o_loss, params, hparams)
    w_mapped = None if stochastic else fp_map(params, hparams)

    def A(xs):
        wm = fp_map(params, hparams) if stochastic else w_mapped
        with params_only(wm):
            jt = torch_grad(wm, params, grad_outputs=_like(xs, wm), retain_graph=not stochastic)
        return [torch.sub(x, j) for x, j in zip(xs, jt)]  # fp64 - fp32: promoted in the one kernel

    vs = CG_torch.cg(A, _f64(g_w), max_iter=K, epsilon=tol)
    if stochastic:
        w_mapped = fp_map(params, hparams)
    grads = torch_grad(w_mapped, hparams, grad_outputs=_like(vs, w_mapped))
    grads = [g + v for g, v in zip(grads, g_h)]
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


def CG_normaleq(params, hparams, K, fp_map, outer_loss, tol=1e-10, set_grad=True):
    """hypergradients.py:199-244: conjugate gradient on the normal equations
    (I - J)(I - J^T) v = (I - J) d outer / d w.  Draws: the outer objective,
    one map (w_mapped: every J^T product), then two maps per J product (the
    second one differentiated), as the reference's jvp."""
    params = [w.detach().requires_grad_(True) for w in params]
    o_loss = outer_loss(params, hparams)
    g_w, g_h = get_outer_gradients(o_loss, params, hparams)
    w_mapped = fp_map(params, hparams)

    def fmap(ps):
        return fp_map(ps, hparams)

    def A(xs):
        with params_only(w_mapped):
            jt = torch_grad(w_mapped, params, grad_outputs=_like(xs, w_mapped), retain_graph=True)
        r = [torch.sub(x, j) for x, j in zip(xs, jt)]  # fp64 - fp32: promoted in the one kernel
        jr = jvp(fmap, params, r)
        return [torch.sub(a, b.detach()) for a, b in zip(r, jr)]

    g64 = _f64(g_w)
    b = [g - j.detach().to(torch.float64) for g, j in zip(g64, jvp(fmap, params, g64))]
    vs = CG_torch.cg(A, b, max_iter=K, epsilon=tol)
    grads = torch_grad(w_mapped, hparams, grad_outputs=_like(vs, w_mapped), allow_unused=True)
    grads = [g + v if g is not None else v for g, v in zip(grads, g_h)]
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


def neumann(params, hparams, K, fp_map, outer_loss, tol=1e-10, set_grad=True):
    """hypergradients.py:247-281: the Neumann series sum_k (J^T)^k g."""
    params = [w.detach().requires_grad_(True) for w in params]
    o_loss = outer_loss(params, hparams)
    g_w, g_h = get_outer_gradients(o_loss, params, hparams)
    w_mapped = fp_map(params, hparams)
    vs = gs = _f64(g_w)
    for _ in range(K):
        prev = gs
        with params_only(w_mapped):
            jt = torch_grad(w_mapped, params, grad_outputs=_like(vs, w_mapped), retain_graph=True)
        vs = [j.to(torch.float64) for j in jt]
        gs = [g + v for g, v in zip(gs, vs)]
        if _norm([a - b for a, b in zip(gs, prev)]) < tol:
            break
    grads = torch_grad(w_mapped, hparams, grad_outputs=_like(gs, w_mapped))
    grads = [g + v for g, v in zip(grads, g_h)]
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


def exact(opt_params_f, hparams, outer_loss, set_grad=True):
    """hypergradients.py:284-297: differentiate a closed-form solution."""
    grads = torch_grad(outer_loss(opt_params_f(hparams), hparams), hparams)
    if set_grad:
        update_tensor_grads(hparams, grads)
    return grads


# ------------------------------------------------------------------ utils
def grd(a, b):
    return torch.autograd.grad(a, b, create_graph=True, retain_graph=True)


def list_dot(l1, l2):
    return torch.stack([(a * b).sum() for a, b in zip(l1, l2)]).sum()


def jvp(fp_map, params, vs):
    """hypergradients.py:308-311: J vs of fp_map at params.  Like the reference
    the map is evaluated twice (its first output only shapes the dummy of the
    double-backward trick) and the second evaluation is differentiated; for a
    HIP gradient-descent map J vs is one psvi_hvp at that evaluation's draw."""
    first = fp_map(params)
    second = fp_map(params)
    fast = hip_jvp(second, vs)
    if fast is not None:
        return fast
    dummy = [torch.ones_like(t).requires_grad_(True) for t in first]
    g1 = grd(list_dot(second, dummy), params)
    return grd(list_dot(_like(vs, g1), g1), dummy)


def get_outer_gradients(outer_loss, params, hparams, retain_graph=True):
    g_w = grad_unused_zero(outer_loss, params, retain_graph=retain_graph)
    g_h = grad_unused_zero(outer_loss, hparams, retain_graph=retain_graph)
    return g_w, g_h


def cat_list_to_tensor(list_tx):
    return torch.cat([t.reshape(-1) for t in list_tx])


def update_tensor_grads(hparams, grads):
    """hparam.grad += the hypergradient (created as zeros when absent)."""
    for h, g in zip(hparams, grads):
        if h.grad is None:
            h.grad = torch.zeros_like(h)
        if g is not None:
            h.grad += g.to(h.dtype)


def grad_unused_zero(output, inputs, grad_outputs=None, retain_graph=False, create_graph=False):
    grads = torch.autograd.grad(output, inputs, grad_outputs=grad_outputs, allow_unused=True,
                                retain_graph=retain_graph, create_graph=create_graph)
    return tuple(torch.zeros_like(v) if g is None else g for g, v in zip(grads, inputs))
