"""PSVI classes: the inner-loop surface of the reference's
psvi/inference/psvi_classes.py on the HIP library.

What runs where
  * ``PSVI.inner_elbo(model, params, hyperopt)`` (psvi_classes.py:488-511): the
    negative inner ELBO  sum_s sum_m N f(v)_m NLL_sm + sum_layers KL  and its
    gradient w.r.t. the variational parameters come from one
    ``psvi_elbo_grad`` call (libpsvi_hip); the result is a 0-dim tensor whose
    ``backward()`` delivers that gradient to the model's parameters.
  * ``PSVI.inner_loop(T)``: the T inner steps that ``nested_step`` /
    ``hyper_step`` run as ``diffopt.step(inner_elbo(fmodel))`` /
    ``inner_opt(params)`` (psvi_classes.py:549-555, 624-650), each one fused
    ``psvi_inner_step`` (reparameterisation, forward, weighted NLL + KL,
    backward, Adam) -- with the Adam variant of the trainer: ``higher``
    (robust_higher/optim.py:299-367, state restarted every outer step) or
    ``hypergrad`` (hypergrad/diff_optimizers.py:184-213).  Parameters are
    written back into the model, as nested_step / hyper_step do at their end.
  * the coreset weights  N f(v):  PSVI f = identity on v = 1/M,
    PSVILearnV softmax(v) (v = 0), PSVIAV exp(alpha) softmax(v)
    (psvi_classes.py:111,177-183, 1350-1360, 1482-1488).

Not on the HIP path: the outer objective ``psvi_elbo``
and everything that differentiates *through* the inner loop (the nested
unroll, CG hypergradients), evaluation and data plumbing.  Those entry points
raise NotImplementedError instead of silently running elsewhere, and
``inner_elbo`` treats u and v as constants (no gradient flows to them).

There is no CPU fallback: a missing libpsvi_hip.so or GPU raises.
"""
import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from ..models.neural_net import categorical_fn, model_spec
from ..runtime import InnerLoopPlan, randn_

__all__ = ["PSVI", "PSVILearnV", "PSVIAV", "PSVIFreeV", "PSVI_No_Rescaling", "PSVI_Ablated",
           "PSVI_No_IW", "PSVIFixedU", "PSVIAFixedU", "HipInnerELBO"]

_OUTER = ("is differentiated through the inner loop (second order); that is the next "
          "row of the hot-path scope (SURVEY.md 8(f)), not part of the HIP inner loop")


class HipInnerELBO(torch.autograd.Function):
    """Negative inner ELBO and its parameter gradient in one HIP call.
    Inputs other than the flat parameter vector are constants."""

    @staticmethod
    def forward(ctx, pvec, plan, u, z, w, eps):
        elbo, grad = plan.elbo_grad(u, z, w, eps, pvec.detach().contiguous())
        ctx.save_for_backward(grad)
        return elbo.to(pvec.dtype).reshape(())

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        return gout * grad, None, None, None, None, None


class PSVI:
    """Pseudodata (coreset) VI with fixed rescaled coefficients v = 1/M
    (psvi_classes.py:83).  Keyword names follow the reference; arguments that
    only concern the outer loop / data plumbing are accepted and ignored."""

    def __init__(self, u=None, z=None, N=None, D=None, model=None, num_pseudo=None, seed=0,
                 mc_samples=None, learn_v=False, f=lambda *x: x[0], distr_fn=categorical_fn,
                 nc=None, register_elbos=True, inner_it=10, log_every=10, lr0net=1e-3,
                 device_id=None, learn_z=False, **kwargs):
        if learn_z:
            raise NotImplementedError("soft labels (learn_z) are not on the HIP inner loop")
        if distr_fn is not categorical_fn:
            raise NotImplementedError("the HIP inner loop implements the categorical likelihood")
        torch.manual_seed(seed)
        # as the reference: cuda when present (the HIP path then refuses anything else)
        self.device = torch.device(f"cuda:{device_id}" if device_id is not None else
                                   ("cuda" if torch.cuda.is_available() else "cpu"))
        self.u, self.z, self.N, self.D, self.nc = u, z, N, D, nc
        self.model = model
        self.num_pseudo = num_pseudo if num_pseudo is not None else (
            u.shape[0] if u is not None else None)
        self.mc_samples = mc_samples
        self.learn_v, self.learn_z = learn_v, False
        self.f = f
        self.distr_fn = distr_fn
        self.register_elbos, self.elbos = register_elbos, []
        self.inner_it, self.log_every, self.lr0net = inner_it, log_every, lr0net
        self.seed = seed
        with torch.no_grad():
            self.v = torch.full((self.num_pseudo,), 1.0 / self.num_pseudo, device=self.device)
        self.v.requires_grad_(self.learn_v)
        self._plans = {}
        self._eps_offset = 0

    # ------------------------------------------------------------ helpers
    def coreset_weights(self):
        """N f(v): the per-pseudopoint NLL weights (detached, fp32)."""
        with torch.no_grad():
            return (self.N * self.f(self.v, 0)).to(torch.float32).contiguous()

    def _plan(self, model):
        fam, layers, prior_sd, S = model_spec(model)
        if self.mc_samples is not None and S != self.mc_samples:
            raise ValueError(f"model mc_samples {S} != PSVI mc_samples {self.mc_samples}")
        M = int(self.u.shape[0])
        key = (fam, tuple(layers), S, M, prior_sd)
        if key not in self._plans:
            self._plans[key] = InnerLoopPlan(fam, layers, S, M, prior_sd=prior_sd)
        return self._plans[key]

    def _data(self, plan):
        M, D = plan.M, plan.layers[0][0]
        u = self.u.detach().to(self.device, torch.float32).reshape(M, D).contiguous()
        z = self.z.detach().to(self.device)
        if z.is_floating_point() and not torch.equal(z, z.round()):
            raise ValueError("z must hold class ids (learn_z is not supported)")
        z = z.to(torch.int32).contiguous()
        C = plan.layers[-1][1]
        if int(z.min()) < 0 or int(z.max()) >= C:
            raise ValueError(f"class ids must lie in [0, {C})")
        return u, z, self.coreset_weights()

    def _draw_eps(self, plan):
        eps = torch.empty(plan.eps_count, device=self.device)
        randn_(eps, self.seed, self._eps_offset)
        self._eps_offset += plan.eps_count
        return eps

    # ---------------------------------------------------------- objectives
    def inner_elbo(self, model=None, params=None, hyperopt=False, eps=None):
        """Negative inner ELBO (psvi_classes.py:488-511), a 0-dim tensor.

        ``params`` (hyperopt=True) is the list of fast weights in module order;
        otherwise the model's own parameters are used.  Fresh eps per call
        (Philox stream of this instance) unless ``eps`` (the library's eps
        layout, ``InnerLoopPlan.eps_count`` floats) is given.  Differentiable
        w.r.t. those parameters (first order); u and v are constants here."""
        model = self.model if model is None else model
        plan = self._plan(model)
        plist = list(params) if (hyperopt and params is not None) else list(model.parameters())
        pvec = nn.utils.parameters_to_vector(plist)
        if pvec.numel() != plan.param_count:
            raise ValueError(f"{pvec.numel()} parameters, plan expects {plan.param_count}")
        u, z, w = self._data(plan)
        eps = self._draw_eps(plan) if eps is None else eps
        return HipInnerELBO.apply(pvec, plan, u, z, w, eps)

    def inner_loop(self, T=None, model=None, lr=None, kind="higher", eps=None):
        """T fused HIP inner steps from the model's current parameters with a
        fresh Adam state (steps 1..T), written back into the model.  Returns the
        negative ELBO before each step (float64, device).  ``eps``: optional
        (T, eps_count) tensor to replay; default draws from this instance's
        Philox stream."""
        model = self.model if model is None else model
        T = self.inner_it if T is None else int(T)
        lr = self.lr0net if lr is None else float(lr)
        plan = self._plan(model)
        u, z, w = self._data(plan)
        plist = list(model.parameters())
        with torch.no_grad():
            params = nn.utils.parameters_to_vector(plist).detach().to(torch.float32).clone()
        if params.numel() != plan.param_count:
            raise ValueError(f"{params.numel()} parameters, plan expects {plan.param_count}")
        m = torch.zeros_like(params)
        v = torch.zeros_like(params)
        ws = plan.workspace(params.device)
        elbos = torch.empty(T, dtype=torch.float64, device=params.device)
        if eps is None:
            step_eps = torch.empty(plan.eps_count, device=params.device)
        for t in range(T):
            if eps is None:
                randn_(step_eps, self.seed, self._eps_offset)
                self._eps_offset += plan.eps_count
                e = step_eps
            else:
                e = eps[t]
            plan.inner_step(u, z, w, e, params, m, v, step=t + 1, lr=lr, kind=kind,
                            elbo_out=elbos[t:t + 1], ws=ws)
        with torch.no_grad():
            nn.utils.vector_to_parameters(params.to(plist[0].dtype), plist)
        if self.register_elbos:
            host = elbos.cpu()
            for t in range(0, T, self.log_every):
                self.elbos.append((1, -float(host[t])))
        return elbos

    # ------------------------------------------------- outer loop (not here)
    def psvi_elbo(self, xbatch, ybatch, model=None, params=None, hyperopt=False):
        raise NotImplementedError("psvi_elbo (outer objective) " + _OUTER)

    def nested_step(self, xbatch, ybatch, truncated=False, K=5):
        raise NotImplementedError("nested_step " + _OUTER)

    def hyper_step(self, xbatch, ybatch, **kwargs):
        raise NotImplementedError("hyper_step " + _OUTER)

    def joint_step(self, xbatch, ybatch):
        raise NotImplementedError("joint_step " + _OUTER)

    def alternating_step(self, xbatch, ybatch):
        raise NotImplementedError("alternating_step " + _OUTER)

    def run_psvi(self, *args, **kwargs):
        raise NotImplementedError("run_psvi drives the outer loop, which " + _OUTER)


class PSVILearnV(PSVI):
    """Learnable v on the simplex: f = softmax, v initialised to 0
    (psvi_classes.py:1344-1360)."""

    def __init__(self, learn_v=True, parameterised=True, **kwargs):
        super().__init__(**kwargs)
        self.learn_v, self.parameterised = learn_v, parameterised
        with torch.no_grad():
            self.v = torch.zeros(self.num_pseudo, device=self.device)
        self.v.requires_grad_(True)
        self.f = torch.softmax


class PSVI_No_Rescaling(PSVI):
    """v = 1/(M N): no dependence on the dataset size (psvi_classes.py:1363-1373)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        with torch.no_grad():
            self.v *= 1.0 / self.N


class PSVIFreeV(PSVI):
    """Learnable non-negative v (psvi_classes.py:1376-1385)."""

    def __init__(self, learn_v=True, **kwargs):
        super().__init__(**kwargs)
        self.learn_v = True
        self.v.requires_grad_(True)


class PSVI_Ablated(PSVILearnV):
    """Differs from PSVILearnV only in the outer objective (psvi_classes.py:1388-1408)."""


class PSVI_No_IW(PSVI_Ablated):
    """Single-sample training (psvi_classes.py:1411-1420)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.mc_samples = 1


class PSVIAV(PSVILearnV):
    """Learnable simplex weights times a learnable total evidence exp(alpha)
    (psvi_classes.py:1475-1490)."""

    def __init__(self, learn_v=True, **kwargs):
        super().__init__(**kwargs)
        self.alpha = torch.tensor([0.0], device=self.device)
        self.alpha.requires_grad_(True)
        self.f = lambda *x: torch.exp(self.alpha) * torch.softmax(x[0], x[1])


class PSVIFixedU(PSVILearnV):
    """u held fixed; same inner loop (psvi_classes.py:1622)."""


class PSVIAFixedU(PSVIAV):
    """u held fixed, learnable evidence scale; same inner loop (psvi_classes.py:1743)."""
