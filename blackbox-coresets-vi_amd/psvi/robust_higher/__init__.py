"""psvi.robust_higher: the differentiable inner-loop API of the reference's
psvi/robust_higher (``innerloop_ctx``, ``monkeypatch``,
``DifferentiableAdam.step``; psvi/robust_higher/__init__.py:27-95,
optim.py:152-257, 299-367) on the HIP library.

The reference unrolls the inner loop on autograd's tape: every
``diffopt.step(inner_elbo(fmodel))`` takes ``autograd.grad(create_graph=True)``
of the inner objective and applies a differentiable Adam step, and the outer
``psvi_elbo(model=fmodel).backward()`` differentiates through all of them.
Here each step is ONE autograd node over the flat parameter vector:

  forward   the gradient comes from the inner objective's psvi_elbo_grad call
            (PSVI.inner_elbo already made it), the Adam step is the fused
            higher-Adam kernel (psvi_adam_update);
  backward  given the adjoints of (p', m', v'): psvi_adam_adjoint gives the
            adjoint of the step's gradient lg, and psvi_hvp at the step's
            parameters and noise gives H lg and the mixed products d/du, d/dw
            (v . grad) -- so the adjoint of p is lt + H lg, and u / w (hence v,
            alpha, and soft labels through their expanded rows) receive the
            mixed products through their autograd graphs.

This is the reverse pass PSVI.nested_step runs by hand, expressed so that the
reference's nested_step body runs unchanged: ``with innerloop_ctx(model,
optim_net) as (fmodel, diffopt): ... diffopt.step(self.inner_elbo(model=fmodel))
... self.psvi_elbo(x, y, model=fmodel).backward()``.

``fmodel`` is a view of the module's parameters (``parameters()``,
``fast_params``, ``update_params``) that PSVI's objectives accept as ``model``;
it has no forward of its own (the objectives run the HIP kernels), and calling
it raises.
"""
from contextlib import contextmanager

import torch
import torch.nn as nn

from ..runtime import adam_adjoint_, adam_update_

__all__ = ["innerloop_ctx", "monkeypatch", "FunctionalModel", "DifferentiableAdam"]


class FunctionalModel:
    """Fast weights of ``module`` as one flat vector (the library's parameter
    order = parameters_to_vector's), exposed as per-parameter views."""

    def __init__(self, module, copy_initial_weights=True, track_higher_grads=True):
        self._psvi_module = module
        plist = list(module.parameters())
        self._shapes = [p.shape for p in plist]
        vec = nn.utils.parameters_to_vector(plist)
        if copy_initial_weights:
            vec = vec.detach().clone().requires_grad_(track_higher_grads)
        self.track_higher_grads = track_higher_grads
        self._set(vec)

    def _set(self, vec):
        self.flat = vec
        self.fast_params, o = [], 0
        for shp in self._shapes:
            n = int(torch.Size(shp).numel())
            self.fast_params.append(vec[o:o + n].view(shp))
            o += n

    def parameters(self):
        return iter(self.fast_params)

    def modules(self):
        return self._psvi_module.modules()

    def children(self):
        return self._psvi_module.children()

    def update_params(self, params):
        params = list(params)
        if len(params) == 1 and params[0].dim() == 1 and params[0].numel() == self.flat.numel():
            self._set(params[0])
        else:
            self._set(torch.cat([p.reshape(-1) for p in params]))

    def __call__(self, *args, **kwargs):
        raise NotImplementedError("the functional model has no forward on the HIP path: pass it "
                                  "as model= to PSVI.inner_elbo / PSVI.psvi_elbo")


def monkeypatch(module, device=None, copy_initial_weights=True, track_higher_grads=True):
    """psvi/robust_higher/patch.py monkeypatch: a FunctionalModel view."""
    return FunctionalModel(module, copy_initial_weights, track_higher_grads)


class _UnrolledAdamStep(torch.autograd.Function):
    """One differentiable inner Adam step: (p, m, v) -> (p', m', v') at the
    gradient g of the inner objective drawn with ``meta``'s noise; u_g / w_g
    are the objective's rows (their graphs lead to u, v, alpha, z)."""

    @staticmethod
    def forward(ctx, p, m, v, u_g, w_g, g, meta, step, hp):
        p1 = p.detach().to(torch.float32).clone()
        m1 = m.detach().to(torch.float32).clone()
        v1 = v.detach().to(torch.float32).clone()
        adam_update_(p1, g, m1, v1, step, hp["lr"], kind=hp["kind"], betas=hp["betas"],
                     eps=hp["eps"])
        ctx.save_for_backward(p.detach().to(torch.float32), m1, v1, g)
        ctx.meta, ctx.step, ctx.hp = meta, step, hp
        ctx.rows = (u_g.shape, u_g.dtype, w_g.shape, w_g.dtype)
        return p1, m1, v1

    @staticmethod
    def backward(ctx, lp, lm, lv):
        p, m1, v1, g = ctx.saved_tensors
        hp, meta = ctx.hp, ctx.meta
        z = torch.zeros_like(p)
        lt = lp.to(torch.float32).contiguous() if lp is not None else z
        lm = lm.to(torch.float32).clone() if lm is not None else z.clone()
        lv = lv.to(torch.float32).clone() if lv is not None else z.clone()
        lg = torch.empty_like(p)
        adam_adjoint_(lt, lm, lv, m1, v1, g, ctx.step, hp["lr"], lg, kind=hp["kind"],
                      betas=hp["betas"], eps=hp["eps"])
        want = ctx.needs_input_grad[3] or ctx.needs_input_grad[4]
        hv, du, dw = meta["plan"].hvp(meta["u"], meta["z"], meta["w"], meta["eps"], p, lg,
                                      mixed=want)
        us, ut, ws, wt = ctx.rows
        gu = du.reshape(us).to(ut) if ctx.needs_input_grad[3] else None
        gw = dw.reshape(ws).to(wt) if ctx.needs_input_grad[4] else None
        return lt + hv, lm, lv, gu, gw, None, None, None, None


class DifferentiableAdam:
    """robust_higher's DifferentiableAdam (optim.py:299-367) over a
    FunctionalModel: ``step(loss)`` with ``loss`` a PSVI.inner_elbo result of
    that model.  State (step count, m, v) starts from the wrapped optimiser's
    state when it has one (higher copies it), else fresh."""

    def __init__(self, opt, fmodel, override=None, track_higher_grads=True, kind="higher"):
        groups = opt.param_groups
        if len(groups) != 1:
            raise NotImplementedError("one parameter group (the PSVI trainers' optim_net)")
        g = dict(groups[0])
        for k, val in (override or {}).items():
            g[k] = val[0] if isinstance(val, (list, tuple)) else val
        if g.get("weight_decay", 0) or g.get("amsgrad", False):
            raise NotImplementedError("weight decay / amsgrad are not in the reference's "
                                      "DifferentiableAdam path")
        self.hp = dict(lr=float(g["lr"]), betas=tuple(float(b) for b in g["betas"]),
                       eps=float(g["eps"]), kind=kind)
        self._fmodel = fmodel
        self.track_higher_grads = track_higher_grads
        n = fmodel.flat.numel()
        dev = fmodel.flat.device
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.t = 0
        st = [opt.state.get(p, {}) for p in groups[0]["params"]]
        if st and all("exp_avg" in s for s in st):
            self.m = torch.cat([s["exp_avg"].reshape(-1) for s in st]).float().to(dev)
            self.v = torch.cat([s["exp_avg_sq"].reshape(-1) for s in st]).float().to(dev)
            self.t = int(float(st[0]["step"]))

    def step(self, loss, params=None, override=None, grad_callback=None, **kwargs):
        if override:
            for k, val in override.items():
                self.hp[k] = float(val[0] if isinstance(val, (list, tuple)) else val)
        if grad_callback is not None:
            raise NotImplementedError("grad_callback: the step's gradient is the HIP objective's")
        meta = getattr(loss, "_psvi_inner", None)
        if meta is None:
            raise TypeError("diffopt.step takes the 0-dim result of PSVI.inner_elbo(model=fmodel) "
                            "as it is (its HIP gradient and noise drive the step)")
        if params is not None:
            self._fmodel.update_params(params)
        p = self._fmodel.flat
        self.t += 1
        g = meta["grad"]
        if self.track_higher_grads:
            p1, self.m, self.v = _UnrolledAdamStep.apply(p, self.m, self.v, meta["u_g"],
                                                         meta["w_g"], g, meta, self.t, self.hp)
        else:
            p1 = p.detach().to(torch.float32).clone()
            adam_update_(p1, g, self.m, self.v, self.t, self.hp["lr"], kind=self.hp["kind"],
                         betas=self.hp["betas"], eps=self.hp["eps"])
            p1.requires_grad_()
        self._fmodel._set(p1)
        return self._fmodel.fast_params


@contextmanager
def innerloop_ctx(model, opt, device=None, copy_initial_weights=True, override=None,
                  track_higher_grads=True):
    """psvi/robust_higher/__init__.py:27-95: yields (fmodel, diffopt)."""
    fmodel = monkeypatch(model, device, copy_initial_weights=copy_initial_weights,
                         track_higher_grads=track_higher_grads)
    diffopt = DifferentiableAdam(opt, fmodel, override=override,
                                 track_higher_grads=track_higher_grads)
    yield fmodel, diffopt
