"""psvi.hypergrad's differentiable optimisers (reference:
psvi/hypergrad/diff_optimizers.py:10-213) over the HIP inner objective.

An optimiser is a map ``params, hparams -> new params`` whose loss
``loss_f(params, hparams)`` is typically ``PSVI.inner_elbo(model=fmodel,
params=p, hyperopt=True)``.  The step functions keep the reference's names and
arithmetic; two of them take a fast path when the loss is a HIP inner
objective (it carries ``_psvi_inner``: plan, rows, draw and its gradient):

  * ``adam_step`` with ``create_graph=False`` (the inner solver of
    PSVI.hyper_step, psvi_classes.py:624-646) applies the gradient the
    objective already computed with the fused hypergrad-Adam kernel
    (psvi_adam_update, PSVI_ADAM_HYPERGRAD: ``v + 1e-12`` stored,
    diff_optimizers.py:184-213) instead of a dozen elementwise ops;
  * ``gd_step`` with ``create_graph=True`` (GradientDescent as the fixed-point
    map of CG_normaleq / fixed_point, psvi_classes.py:652-667) returns
    ``w - lr grad`` as ONE autograd node whose backward is the Hessian-vector
    product of the inner objective at the objective's own draw (psvi_hvp):
    v -> v - lr H v for the parameters and -lr d/du (v . grad), -lr d/dw
    (v . grad) for the rows -- what autograd's double backward through
    ``torch.autograd.grad(loss, params, create_graph=True)`` gives in the
    reference, so ``torch.autograd.grad(w_mapped, params / hparams,
    grad_outputs=v)`` works on it unchanged.

Any other loss goes through torch autograd exactly as in the reference."""
import contextlib
from itertools import repeat

import torch

from ..runtime import adam_update_

__all__ = ["DifferentiableOptimizer", "GradientDescent", "HeavyBall", "Momentum",
           "DifferentiableAdam", "gd_step", "heavy_ball_step", "torch_momentum_step",
           "adam_step"]


def _flat32(ts):
    return torch.cat([t.detach().reshape(-1).to(torch.float32) for t in ts]).contiguous()


def _split(vec, like):
    out, o = [], 0
    for t in like:
        n = t.numel()
        out.append(vec[o:o + n].reshape(t.shape).to(t.dtype))
        o += n
    return out


class _HipGradStep(torch.autograd.Function):
    """w' = w - lr grad_w L(w) for a HIP inner objective L (meta: its
    ``_psvi_inner``), one node over the parameter list and the objective's
    rows u_g, w_g (whose graphs lead to u, v, alpha)."""

    @staticmethod
    def forward(ctx, lr, meta, u_g, w_g, *params):
        ctx.meta, ctx.lr, ctx.like = meta, float(lr), [p.detach() for p in params]
        ctx.rows = (u_g.shape, u_g.dtype, w_g.shape, w_g.dtype)
        new = _flat32(params) - ctx.lr * meta["grad"]
        return tuple(_split(new, params))

    @staticmethod
    def backward(ctx, *gouts):
        meta, lr = ctx.meta, ctx.lr
        v = torch.cat([(g if g is not None else torch.zeros_like(p)).reshape(-1).to(torch.float32)
                       for g, p in zip(gouts, ctx.like)]).contiguous()
        # needs_input_grad is fixed when the node is built; a solver's J^T
        # products (torch_grad(w_mapped, params)) discard the rows' gradients,
        # and say so through params_only(): only the mixed-product pass pays
        # for d/du, d/dw (at C5 the separate d/du pass of every CG iteration)
        mixed = (ctx.needs_input_grad[2] or ctx.needs_input_grad[3]) and \
            not meta.get("params_only", False)
        hv, du, dw = meta["plan"].hvp(meta["u"], meta["z"], meta["w"], meta["eps"],
                                      meta["params"], v, mixed=mixed)
        us, ut, ws, wt = ctx.rows
        gu = (-lr * du).reshape(us).to(ut) if mixed and ctx.needs_input_grad[2] else None
        gw = (-lr * dw).reshape(ws).to(wt) if mixed and ctx.needs_input_grad[3] else None
        return (None, None, gu, gw, *_split(v - lr * hv, ctx.like))


@contextlib.contextmanager
def params_only(w_mapped):
    """Scope of J^T products that only the parameters receive
    (torch_grad(w_mapped, params, ...)): the map's HIP node skips the mixed
    products d/du, d/dw its backward would otherwise form.  The flag lives on
    the map's own objective (one dict per map evaluation), so ranks running
    in threads do not see each other's setting.  No effect on other maps."""
    tag = getattr(w_mapped[0], "_psvi_gd", None) if w_mapped is not None and len(w_mapped) \
        else None
    if tag is None:
        yield
        return
    meta = tag[0]
    prev = meta.get("params_only", False)
    meta["params_only"] = True
    try:
        yield
    finally:
        meta["params_only"] = prev


def hip_jvp(w_mapped, vs):
    """J vs for a fixed-point map output of gd_step on a HIP objective (None
    otherwise): J = I - lr H with H the objective's Hessian at its draw --
    symmetric, so J vs is the same product the node's backward forms."""
    tag = getattr(w_mapped[0], "_psvi_gd", None) if len(w_mapped) else None
    if tag is None:
        return None
    meta, lr = tag
    v = _flat32(vs)
    hv, _, _ = meta["plan"].hvp(meta["u"], meta["z"], meta["w"], meta["eps"], meta["params"], v,
                                mixed=False)
    return _split(v - lr * hv, vs)


def gd_step(params, loss, step_size, create_graph=True):
    """diff_optimizers.py:157-159: w - step_size * grad."""
    meta = getattr(loss, "_psvi_inner", None)
    if meta is not None and create_graph and not torch.is_tensor(step_size):
        out = list(_HipGradStep.apply(float(step_size), meta, meta["u_g"], meta["w_g"], *params))
        for t in out:
            t._psvi_gd = (meta, float(step_size))
        return out
    grads = torch.autograd.grad(loss, params, create_graph=create_graph)
    return [w - step_size * g for w, g in zip(params, grads)]


def heavy_ball_step(params, aux_params, loss, step_size, momentum, create_graph=True):
    """diff_optimizers.py:162-167."""
    grads = torch.autograd.grad(loss, params, create_graph=create_graph)
    return [w - step_size * g + momentum * (w - v)
            for g, w, v in zip(grads, params, aux_params)], params


def torch_momentum_step(params, aux_params, loss, step_size, momentum=0.9, create_graph=True):
    """diff_optimizers.py:170-181 (torch.optim.SGD momentum)."""
    grads = torch.autograd.grad(loss, params, create_graph=create_graph)
    vel = [momentum * v + g for v, g in zip(aux_params, grads)]
    return [w - step_size * v for w, v in zip(params, vel)], vel


def adam_step(params, ms, us, loss, step_size, step_cnt, beta1, beta2, eps, momentum=0.9,
              create_graph=True):
    """diff_optimizers.py:184-213: m' = b1 m + (1-b1) g, u' = b2 u + (1-b2) g^2
    + 1e-12, w' = w - lr (m'/(1-b1^t)) / (sqrt(u'/(1-b2^t)) + eps)."""
    meta = getattr(loss, "_psvi_inner", None)
    if meta is not None and not create_graph and not torch.is_tensor(step_size) and \
            all(t.is_cuda for t in params):
        p, m, u = _flat32(params), _flat32(ms), _flat32(us)
        adam_update_(p, meta["grad"], m, u, int(step_cnt), float(step_size), kind="hypergrad",
                     betas=(float(beta1), float(beta2)), eps=float(eps))
        return _split(p, params), _split(m, ms), _split(u, us)
    grads = torch.autograd.grad(loss, params, create_graph=create_graph)
    m1 = [beta1 * m + (1.0 - beta1) * g for m, g in zip(ms, grads)]
    u1 = [beta2 * u + (1.0 - beta2) * g ** 2 + 1e-12 for u, g in zip(us, grads)]
    bc1, bc2 = 1.0 - beta1 ** step_cnt, 1.0 - beta2 ** step_cnt
    return ([w - step_size * (m / bc1 / (torch.sqrt(u / bc2) + eps))
             for w, m, u in zip(params, m1, u1)], m1, u1)


class DifferentiableOptimizer:
    """diff_optimizers.py:10-47: loss_f(params, hparams[, data]) -> loss."""

    def __init__(self, loss_f, dim_mult, data_or_iter=None):
        self.data_iterator = None
        if data_or_iter:
            self.data_iterator = (data_or_iter if hasattr(data_or_iter, "__next__")
                                  else repeat(data_or_iter))
        self.loss_f = loss_f
        self.dim_mult = dim_mult
        self.curr_loss = None

    def get_opt_params(self, params):
        """params followed by (dim_mult - 1) zero-initialised state lists."""
        out = list(params)
        for _ in range(self.dim_mult - 1):
            out += [torch.zeros_like(p) for p in params]
        return out

    def step(self, params, hparams, create_graph):
        raise NotImplementedError

    def __call__(self, params, hparams, create_graph=True):
        with torch.enable_grad():
            return self.step(params, hparams, create_graph)

    def get_loss(self, params, hparams):
        if self.data_iterator:
            self.curr_loss = self.loss_f(params, hparams, next(self.data_iterator))
        else:
            self.curr_loss = self.loss_f(params, hparams)
        return self.curr_loss


def _as_fn(x):
    return x if callable(x) else (lambda _h: x)


class GradientDescent(DifferentiableOptimizer):
    """diff_optimizers.py:50-59."""

    def __init__(self, loss_f, step_size, data_or_iter=None):
        super().__init__(loss_f, dim_mult=1, data_or_iter=data_or_iter)
        self.step_size_f = _as_fn(step_size)

    def step(self, params, hparams, create_graph):
        loss = self.get_loss(params, hparams)
        return gd_step(params, loss, self.step_size_f(hparams), create_graph=create_graph)


class HeavyBall(DifferentiableOptimizer):
    """diff_optimizers.py:62-77."""

    def __init__(self, loss_f, step_size, momentum, data_or_iter=None):
        super().__init__(loss_f, dim_mult=2, data_or_iter=data_or_iter)
        self.step_size_f, self.momentum_f = _as_fn(step_size), _as_fn(momentum)

    def step(self, params, hparams, create_graph):
        n = len(params) // 2
        loss = self.get_loss(params[:n], hparams)
        p, aux = heavy_ball_step(params[:n], params[n:], loss, self.step_size_f(hparams),
                                 self.momentum_f(hparams), create_graph=create_graph)
        return [*p, *aux]


class Momentum(DifferentiableOptimizer):
    """diff_optimizers.py:80-101 (torch.optim.SGD with momentum)."""

    def __init__(self, loss_f, step_size, momentum=0.9, data_or_iter=None):
        super().__init__(loss_f, dim_mult=2, data_or_iter=data_or_iter)
        self.step_size_f, self.momentum_f = _as_fn(step_size), _as_fn(momentum)

    def step(self, params, hparams, create_graph):
        n = len(params) // 2
        loss = self.get_loss(params[:n], hparams)
        p, aux = torch_momentum_step(params[:n], params[n:], loss, self.step_size_f(hparams),
                                     self.momentum_f(hparams), create_graph=create_graph)
        return [*p, *aux]


class DifferentiableAdam(DifferentiableOptimizer):
    """diff_optimizers.py:104-154: params = [p..., m..., u...], step count
    from step_cnt (1), advanced by every step."""

    def __init__(self, loss_f, step_size, data_or_iter=None, betas=(0.9, 0.999), eps=1e-8,
                 step_cnt=1):
        super().__init__(loss_f, dim_mult=3, data_or_iter=data_or_iter)
        self.step_size_f = _as_fn(step_size)
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.step_cnt = step_cnt

    def step(self, params, hparams, create_graph):
        n = len(params) // 3
        loss = self.get_loss(params[:n], hparams)
        p, m, u = adam_step(params[:n], params[n:2 * n], params[2 * n:], loss,
                            self.step_size_f(hparams), self.step_cnt, self.beta1, self.beta2,
                            self.eps, create_graph=create_graph)
        self.step_cnt += 1
        return [*p, *m, *u]
