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

  * ``PSVI.psvi_elbo(xbatch, ybatch, model, params, hyperopt)``
    (psvi_classes.py:445-486): the outer objective with the sampled KL of every
    layer, one ``psvi_outer_elbo_grad`` call; its ``backward()`` delivers the
    first-order gradients to the parameters, to u and -- through the host's
    N f(v) -- to v and alpha.  ``joint_step`` / ``alternating_step``
    (517-539) run on it unchanged.

Not on the HIP path: everything that differentiates
*through* the inner loop (the nested unroll, CG hypergradients), evaluation
and data plumbing.  Those entry points raise NotImplementedError instead of
silently running elsewhere, and ``inner_elbo`` treats u and v as constants (no
gradient flows to them).

There is no CPU fallback: a missing libpsvi_hip.so or GPU raises.
"""
import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from ..models.neural_net import categorical_fn, model_spec
from ..runtime import InnerLoopPlan, randn_

__all__ = ["PSVI", "PSVILearnV", "PSVIAV", "PSVIFreeV", "PSVI_No_Rescaling", "PSVI_Ablated",
           "PSVI_No_IW", "PSVIFixedU", "PSVIAFixedU", "HipInnerELBO", "HipOuterELBO"]

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


class HipOuterELBO(torch.autograd.Function):
    """Negative PSVI-ELBO (outer objective) and its first-order gradients
    w.r.t. the flat parameters, the pseudo-inputs u and the pseudopoint
    weights N f(v) in one HIP call (psvi_outer_elbo_grad)."""

    @staticmethod
    def forward(ctx, pvec, u, wp, plan, xb, z_all, w_data, eps):
        Mu = u.shape[0]
        x_all = torch.cat([u.detach().reshape(Mu, -1), xb]).to(torch.float32).contiguous()
        w_all = torch.cat([wp.detach().to(torch.float32), w_data]).contiguous()
        out = plan.outer_elbo_grad(Mu, x_all, z_all, w_all, eps, pvec.detach().contiguous(),
                                   grad=True, grad_u=Mu > 0, grad_w=True)
        gu = out["grad_u"] if Mu > 0 else torch.zeros_like(x_all[:0])
        ctx.save_for_backward(out["grad"], gu.reshape(u.shape), out["grad_w"])
        ctx.dtypes = (pvec.dtype, u.dtype, wp.dtype)
        return out["loss"].to(pvec.dtype).reshape(())

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        gp, gu, gw = ctx.saved_tensors
        tp, tu, tw = ctx.dtypes
        return ((gout * gp).to(tp), (gout * gu).to(tu), (gout * gw).to(tw),
                None, None, None, None, None)


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

    # ------------------------------------------------------ outer objective
    def psvi_elbo(self, xbatch, ybatch, model=None, params=None, hyperopt=False, eps=None):
        """Negative PSVI-ELBO (psvi_classes.py:445-486), a 0-dim tensor:
        sum_s W_s (data_s - pseudo_s) - mean_s lw_s over a fresh sample of the
        weights, W = softmax_s(lw), lw_s = -pseudo_s + sampled_nkl_s.
        Differentiable (first order) w.r.t. the parameters (or ``params`` with
        hyperopt=True), u, and v / alpha through N f(v).  ``eps``: the
        library's eps layout (``eps_count`` floats) to replay a draw."""
        assert self.mc_samples is None or self.mc_samples > 1  # psvi_classes.py:449
        model = self.model if model is None else model
        fam, layers, prior_sd, S = model_spec(model)
        if S < 2:
            raise ValueError("psvi_elbo needs mc_samples > 1 (psvi_classes.py:449)")
        Mu = int(self.u.shape[0])
        xb = xbatch.detach().to(self.device, torch.float32).reshape(xbatch.shape[0], -1)
        Nx = int(xb.shape[0])
        key = ("outer", fam, tuple(layers), S, Mu + Nx, prior_sd)
        if key not in self._plans:
            self._plans[key] = InnerLoopPlan(fam, layers, S, Mu + Nx, prior_sd=prior_sd)
        plan = self._plans[key]
        plist = list(params) if (hyperopt and params is not None) else list(model.parameters())
        pvec = nn.utils.parameters_to_vector(plist)
        if pvec.numel() != plan.param_count:
            raise ValueError(f"{pvec.numel()} parameters, plan expects {plan.param_count}")
        z = torch.cat([self.z.detach().to(self.device).reshape(-1),
                       ybatch.detach().to(self.device).reshape(-1)])
        if z.is_floating_point() and not torch.equal(z, z.round()):
            raise ValueError("labels must hold class ids (learn_z is not supported)")
        z_all = z.to(torch.int32).contiguous()
        C = layers[-1][1]
        if int(z_all.min()) < 0 or int(z_all.max()) >= C:
            raise ValueError(f"class ids must lie in [0, {C})")
        wp = (self.N * self.f(self.v, 0)).to(torch.float32).reshape(-1)
        w_data = torch.full((Nx,), float(self.N) / max(Nx, 1), device=self.device)
        if eps is None:
            eps = self._draw_eps(plan)
        loss = HipOuterELBO.apply(pvec, self.u, wp, plan, xb, z_all, w_data, eps)
        return loss

    def setup_optimizers(self, lr0net=1e-3, lr0u=1e-3, lr0v=1e-2, lr0joint=1e-3,
                         trainer="nested"):
        """The optimisers run_psvi creates (psvi_classes.py:867-885): Adam on
        the network, on u, on v (learn_v), and for trainer 'joint' one Adam
        over all of them."""
        self.u.requires_grad_(True)
        self.optim_net = torch.optim.Adam(list(self.model.parameters()), lr0net)
        self.optim_u = torch.optim.Adam([self.u], lr0u)
        if self.learn_v:
            self.optim_v = torch.optim.Adam([self.v], lr0v)
        if trainer == "joint":
            vp = list(self.model.parameters()) + [self.u] + ([self.v] if self.learn_v else [])
            self.optim = torch.optim.Adam(vp, lr0joint)

    def joint_step(self, xbatch, ybatch):
        """psvi_classes.py:517-525: one Adam step on the outer objective over
        the network, u (and v)."""
        self.optim.zero_grad()
        loss = self.psvi_elbo(xbatch, ybatch, model=self.model)
        with torch.no_grad():
            if self.register_elbos:
                self.elbos.append((2, -loss.item()))
        loss.backward()
        self.optim.step()
        return loss

    def alternating_step(self, xbatch, ybatch):
        """psvi_classes.py:527-539: a step of optim_net, then of optim_u, each
        on a fresh evaluation of the outer objective."""
        for i in range(2):
            self.optim = self.optim_net if i == 0 else self.optim_u
            self.optim.zero_grad()
            loss = self.psvi_elbo(xbatch, ybatch, model=self.model)
            with torch.no_grad():
                if self.register_elbos:
                    self.elbos.append((1, -loss.item())) if i == 1 else self.elbos.append(
                        (0, -loss.item()))
            loss.backward()
            self.optim.step()
        return loss

    # -------------------------------------------- second order (not here)
    def nested_step(self, xbatch, ybatch, truncated=False, K=5):
        raise NotImplementedError("nested_step " + _OUTER)

    def hyper_step(self, xbatch, ybatch, **kwargs):
        raise NotImplementedError("hyper_step " + _OUTER)

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
