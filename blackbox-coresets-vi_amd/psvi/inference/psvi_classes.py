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

  * ``PSVI.hyper_step`` (psvi_classes.py:602-687): the T-step first-order inner
    loop (hypergrad Adam, ``psvi_inner_loop``), then hypergrad's
    ``CG_normaleq`` (hypergradients.py:199-244) on Hessian-vector products of
    the inner objective (``psvi_hvp``: J^T x and the jvp J x of
    GradientDescent's fp_map are x - lr H x), the mixed products for the
    hypergradient of u and v, and the outer objective's direct gradients;
    then the u / v Adam steps.  The CG vectors are float64 device tensors.

  * ``PSVI.nested_step`` (psvi_classes.py:541-600, the reference's default
    trainer): T higher-Adam steps (``psvi_elbo_grad`` + ``psvi_adam_update``,
    the trajectory kept on the device), the outer objective at the result,
    and ``psvi_elbo.backward()`` through the unroll as reverse mode: per step
    back, ``psvi_adam_adjoint`` and one ``psvi_hvp`` with its mixed products;
    then the u / v Adam steps.

  * ``PSVI.evaluate`` / ``pred_on_grid`` (psvi_classes.py:1031-1175): the
    importance-weighted predictive, one ``psvi_evaluate`` per test batch.

  * The plugin variants (psvi_classes.py:1344-1884) differ only in what the
    outer step learns and which outer objective it differentiates:
    ``PSVIAV`` / ``PSVIAFixedU`` add alpha (w = N exp(alpha) softmax(v)) with
    its own Adam ``optim_alpha``; ``PSVIFixedU`` / ``PSVIAFixedU`` freeze u;
    ``PSVI_Ablated`` / ``PSVI_No_IW`` use the ablated outer objective
    (``psvi_outer_ablated_elbo_grad``: mean data NLL minus mean sampled KL, no
    importance weights); ``PSVI_No_IW`` trains single-sample, where the
    reference's inner objective scores every pseudo row against every pseudo
    label (its 2-d logits broadcast in Categorical.log_prob) -- reproduced as
    the standard objective over M*C expanded rows.

``inner_elbo`` is differentiable (first order) w.r.t. the parameters and,
as the reference's autograd, w.r.t. u and v / alpha where they require grad
(the row node ``HipInnerRows``); the trainers carry the hypergradients of u, v
and alpha through ``psvi_hvp``'s mixed products.  Soft labels (``learn_z``:
expanded (row, class) rows, z through the softmax over rows) and
``nested_step(truncated=True)`` are built (fixtures w01-w05); ``hyper_step``
with ``learn_z`` raises NotImplementedError as the reference does
(psvi_classes.py:619-620).  With samples sharded over ranks (world > 1) the
soft-label outer objective runs on ``ShardedOuter`` (``HipOuterRowsELBO``).

There is no CPU fallback: a missing libpsvi_hip.so or GPU raises.
"""
import contextlib
import functools
import time

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from ..models.neural_net import (VILinear, VILinearMultivariateNormal, categorical_fn,
                                 make_fc2net, make_fcnet, make_lenet, model_spec)
from ..runtime import InnerLoopPlan, adam_adjoint_, adam_update_, nonfinite_, randn_

__all__ = ["PSVI", "PSVILearnV", "PSVIAV", "PSVIFreeV", "PSVI_No_Rescaling", "PSVI_Ablated",
           "PSVI_No_IW", "PSVIFixedU", "PSVIAFixedU", "HipInnerELBO", "HipInnerRows",
           "HipOuterELBO"]

class HipInnerELBO(torch.autograd.Function):
    """Negative inner ELBO as an autograd node over one psvi_elbo_grad call
    (value and parameter gradient computed by the caller, PSVI.inner_elbo)."""

    @staticmethod
    def forward(ctx, pvec, elbo, grad):
        ctx.save_for_backward(grad)
        return elbo.to(pvec.dtype).reshape(()).clone()

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        return gout * grad, None, None


class HipInnerRows(torch.autograd.Function):
    """The inner objective's dependence on its rows: a zero-valued term whose
    backward gives d/du and d/dw of the weighted NLL with ``rows_fn`` (the
    outer-objective kernel in coefficient mode, every sample's pseudo term with
    coefficient 1) -- what the reference's autograd delivers to u, v and alpha
    through inner_elbo (psvi_classes.py:488-511).  A separate node, so a
    gradient asked for the parameters only (the inner optimisers' steps) never
    runs the row pass."""

    @staticmethod
    def forward(ctx, u_g, w_g, rows_fn, dtype):
        ctx.rows_fn = rows_fn
        ctx.shapes = (u_g.shape, u_g.dtype, w_g.shape, w_g.dtype)
        return torch.zeros((), dtype=dtype, device=u_g.device)

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        us, ut, ws, wt = ctx.shapes
        du, dw = ctx.rows_fn()
        gu = (gout * du).reshape(us).to(ut) if ctx.needs_input_grad[0] else None
        gw = (gout * dw).reshape(ws).to(wt) if ctx.needs_input_grad[1] else None
        return gu, gw, None, None


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


class HipAblatedELBO(torch.autograd.Function):
    """PSVI_Ablated's outer objective (mean data NLL minus mean sampled KL over
    the data batch) and its parameter gradient in one HIP call
    (psvi_outer_ablated_elbo_grad).  No pseudopoint enters it."""

    @staticmethod
    def forward(ctx, pvec, plan, xb, yb, w_data, eps):
        out = plan.outer_ablated_elbo_grad(xb, yb, w_data, eps, pvec.detach().contiguous())
        ctx.save_for_backward(out["grad"])
        ctx.ptype = pvec.dtype
        return out["loss"].to(pvec.dtype).reshape(())

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        (gp,) = ctx.saved_tensors
        return (gout * gp).to(ctx.ptype), None, None, None, None, None


class HipOuterRowsELBO(torch.autograd.Function):
    """PSVI.psvi_elbo over caller-formed rows whose weights -- pseudo AND data
    rows -- carry autograd graphs: learn_z's soft labels as expanded rows
    (psvi_classes.py:450-486), where every row's target depends on z through
    the softmax over all rows.  One psvi_outer_elbo_grad (loss, parameter,
    pseudo-row input and weight gradients, the sample weights W_s), then one
    psvi_outer_elbo_grad_coef with every row as a pseudo row and coefficient
    W_s for the data rows' weight gradients sum_s W_s NLL_s,row."""

    @staticmethod
    def forward(ctx, pvec, u_rows, w_rows, plan, x_all, z_all, eps, n_pseudo):
        from ..runtime.sharded import ShardedOuter, pack_coef

        p = pvec.detach().to(torch.float32).contiguous()
        w = w_rows.detach().to(torch.float32).contiguous()
        R = x_all.shape[0]
        if isinstance(plan, ShardedOuter):
            # samples split over ranks: pass 1 + the all-reduced coefficients
            # give the loss, the gradients and every sample's W_s; the data
            # rows' weight gradients sum_s W_s NLL_s,row are one more coefficient
            # pass over this rank's samples, all-reduced
            out = plan.elbo_grad(n_pseudo, x_all, z_all, w, eps, p, grad_u=n_pseudo > 0,
                                 grad_w=True, sample_weights=True)
            W = out["W"]
            zero = torch.zeros_like(W)
            gd = plan.coef_grads(R, x_all, z_all, w, eps, p, W, zero, zero, grad_u=False,
                                 grad_w=True)["grad_w"][n_pseudo:]
        else:
            out = plan.outer_elbo_grad(n_pseudo, x_all, z_all, w, eps, p, grad=True,
                                       grad_u=n_pseudo > 0, grad_w=True, sample_stats=True)
            S = out["samples"].shape[0]
            W = out["samples"][:, 3].cpu()
            zero = torch.zeros(S, dtype=torch.float64)
            gd = plan.outer_grad_coef(R, x_all, z_all, w, eps, p,
                                      pack_coef(W, zero, zero, 0, S).to(p.device),
                                      grad_u=False, grad_w=True)["grad_w"][n_pseudo:]
        gu = out["grad_u"] if n_pseudo > 0 else torch.zeros_like(x_all[:0])
        ctx.save_for_backward(out["grad"], gu, torch.cat([out["grad_w"], gd]))
        ctx.meta = (pvec.dtype, u_rows.shape, u_rows.dtype, w_rows.dtype)
        return out["loss"].to(pvec.dtype).reshape(())

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        gp, gu, gw = ctx.saved_tensors
        tp, us, ut, wt = ctx.meta
        return ((gout * gp).to(tp), (gout * gu).reshape(us).to(ut), (gout * gw).to(wt),
                None, None, None, None, None)


def _trainer_step(fn):
    """One outer step of a trainer (PSVI._outer_step's scope)."""
    @functools.wraps(fn)
    def run(self, *args, **kwargs):
        with self._outer_step():
            return fn(self, *args, **kwargs)
    return run


class PSVI:
    """Pseudodata (coreset) VI with fixed rescaled coefficients v = 1/M
    (psvi_classes.py:83).  Keyword names follow the reference; arguments that
    only concern the outer loop / data plumbing are accepted and ignored.

    Variant switches (set by the subclasses): ``_learn_u`` (False: u frozen,
    PSVIFixedU / PSVIAFixedU), ``_outer_mode`` ("iw" PSVI.psvi_elbo, "ablated"
    PSVI_Ablated.psvi_elbo), ``_noiw`` (PSVI_No_IW's single-sample inner
    objective)."""

    _learn_u = True
    _outer_mode = "iw"
    _noiw = False

    def __init__(self, u=None, z=None, N=None, D=None, model=None, num_pseudo=None, seed=0,
                 mc_samples=None, learn_v=False, f=lambda *x: x[0], distr_fn=categorical_fn,
                 nc=None, register_elbos=True, inner_it=10, log_every=10, lr0net=1e-3,
                 device_id=None, learn_z=False, compute_weights_entropy=True, world=1, rank=0,
                 comm=None, **kwargs):
        if distr_fn is not categorical_fn:
            raise NotImplementedError("the HIP inner loop implements the categorical likelihood")
        torch.manual_seed(seed)
        # as the reference: cuda when present (the HIP path then refuses anything else)
        self.device = torch.device(f"cuda:{device_id}" if device_id is not None else
                                   ("cuda" if torch.cuda.is_available() else "cpu"))
        self.u, self.z, self.N, self.D, self.nc = u, z, N, D, nc
        self.train_dataset = kwargs.get("train_dataset")
        self.test_dataset = kwargs.get("test_dataset")
        self.init_dataset = kwargs.get("init_dataset")
        for k in ("prune", "increment", "retrain_on_coreset", "reset"):
            if kwargs.get(k):
                raise NotImplementedError(f"{k}=True (coreset pruning / incremental learning / "
                                          "retraining / resets) is not on the HIP path")
        self.chosen_indices = []
        self.model = model
        self.num_pseudo = num_pseudo if num_pseudo is not None else (
            u.shape[0] if u is not None else None)
        self.mc_samples = mc_samples
        self.learn_v, self.learn_z = learn_v, bool(learn_z)
        self.f = f
        self.distr_fn = distr_fn
        self.register_elbos, self.elbos = register_elbos, []
        self.inner_it, self.log_every, self.lr0net = inner_it, log_every, lr0net
        self.seed = seed
        self.lr0alpha = kwargs.get("lr0alpha", 1e-3)
        self.compute_weights_entropy = compute_weights_entropy
        self.results = {}
        with torch.no_grad():
            self.v = torch.full((self.num_pseudo,), 1.0 / self.num_pseudo, device=self.device)
        self.v.requires_grad_(self.learn_v)
        self._plans = {}
        self._eps_offset = 0
        self._eps_feed, self._eps_short = None, False
        self._labels_ok = None
        self._label_flag, self._label_C, self._defer_labels = None, None, False
        # samples split over `world` ranks (one process per GPU):
        # every objective / HVP sums the ranks' shares with one all-reduce
        self.world, self.rank = int(world), int(rank)
        if self.world > 1 and comm is None:
            from ..runtime.sharded import TorchDistComm
            comm = TorchDistComm()
        self.comm = comm
        self._make_plan = InnerLoopPlan

    # ------------------------------------------------------------ helpers
    def coreset_weights(self):
        """N f(v): the per-pseudopoint NLL weights (detached, fp32)."""
        with torch.no_grad():
            return (self.N * self.f(self.v, 0)).to(torch.float32).contiguous()

    def _noiw_rows(self, model):
        """PSVI_No_IW trains with one sample; a single-sample mean-field model
        gives 2-d logits, which inner_elbo unsqueezes to (M, 1, C)
        (psvi_classes.py:492-493), so Categorical.log_prob(z) broadcasts to
        (M, M): every pseudo row is scored against every pseudo label."""
        if not self._noiw:
            return False
        fam, _, _, S = model_spec(model)
        if S != 1:
            return False
        if fam != "meanfield":
            raise NotImplementedError("PSVI_No_IW runs mean-field models on the HIP path "
                                      "(the reference's ablated outer objective fails on "
                                      "full-covariance ones)")
        return True

    def _plan(self, model):
        fam, layers, prior_sd, S = model_spec(model)
        if self.mc_samples is not None and S != self.mc_samples:
            raise ValueError(f"model mc_samples {S} != PSVI mc_samples {self.mc_samples}")
        M = int(self.u.shape[0])
        if self._noiw_rows(model) or self.learn_z:
            if self._noiw and self.learn_z:
                raise NotImplementedError("PSVI_No_IW with soft labels (learn_z)")
            M *= layers[-1][1]
        key = (fam, tuple(layers), S, M, prior_sd)
        if key not in self._plans:
            self._plans[key] = self._new_plan(fam, layers, S, M, prior_sd, outer=False)
        return self._plans[key]

    def _new_plan(self, fam, layers, S, M, prior_sd, outer):
        """A world-1 plan, or with world > 1 the sample-sharded form of one
        (this rank's samples; results all-reduced): SampleShardedPlan for the
        inner objective and its HVP, ShardedOuter for the outer objective."""
        if self.world == 1:
            return self._make_plan(fam, layers, S, M, prior_sd=prior_sd)
        from ..runtime.sharded import SampleShardedPlan, ShardedOuter, sample_split

        s_cnt = sample_split(S, self.world)[self.rank][1]
        local = self._make_plan(fam, layers, s_cnt, M, prior_sd=prior_sd)
        cls = ShardedOuter if outer else SampleShardedPlan
        return cls(fam, layers, S, M, self.world, self.rank, prior_sd=prior_sd, comm=self.comm,
                   plan=local)

    def _check_labels(self, z, C):
        """Class ids in [0, C) -- validated once per label tensor version (a
        device-to-host read; not on every objective call)."""
        if self.learn_z:
            if tuple(z.shape[-1:]) != (C,):
                raise ValueError(f"learn_z: z must be (M, {C}) label logits")
            return
        key = (id(z), getattr(z, "_version", 0), C)
        if self._labels_ok == key:
            return
        if z.is_floating_point() and not torch.equal(z, z.round()):
            raise ValueError("z must hold class ids (learn_z is not supported)")
        if z.numel() and (int(z.min()) < 0 or int(z.max()) >= C):
            raise ValueError(f"class ids must lie in [0, {C})")
        self._labels_ok = key

    def _batch_labels(self, y, C):
        """Minibatch labels as int32 on the device.  Ids outside [0, C) (or
        non-integral float ids) raise ValueError as the reference's
        Categorical.log_prob does: a device-side flag is formed here (the ids
        are clamped only so the kernels never read out of bounds) and read on
        the host once -- at once per outer step inside the trainers (before any
        hyperparameter moves), at once per call otherwise."""
        yi = y.reshape(-1)
        bad = (yi < 0) | (yi >= C)
        if yi.is_floating_point():
            bad = bad | (yi != yi.round())
        flag = bad.any()
        self._label_flag = flag if self._label_flag is None else (self._label_flag | flag)
        self._label_C = C
        if not self._defer_labels:
            self._raise_bad_labels()
        return yi.to(torch.int32).clamp_(0, C - 1).contiguous()

    def _raise_bad_labels(self):
        """The one host read of the accumulated minibatch-label flag."""
        f, self._label_flag = self._label_flag, None
        if f is not None and bool(f):
            raise ValueError(f"minibatch class ids must lie in [0, {self._label_C})")

    @contextlib.contextmanager
    def _outer_step(self):
        """Scope of one trainer step: minibatch-label checks are deferred to
        _raise_bad_labels (called before the hyperparameter steps) and a replay
        feed that the step did not use up is dropped, not served later."""
        prev = self._defer_labels
        self._defer_labels = True
        try:
            yield
        except BaseException:
            # a step that fails for another reason must not leave a flag from
            # its (possibly bad) batch behind for the next call to raise on
            if not prev:
                self._label_flag = None
            raise
        finally:
            self._defer_labels = prev
            self._eps_feed = None
        if not prev:
            self._raise_bad_labels()

    def _data(self, plan):
        """(u, z, w) of the inner objective's rows: the pseudopoints, or for
        PSVI_No_IW's single-sample objective the M*C expanded rows (u_i, class
        c, W_c = sum of w_j over the pseudopoints labelled c)."""
        C = plan.layers[-1][1]
        M0 = int(self.u.shape[0])
        D = plan.in_features
        self._check_labels(self.z, C)
        u = self.u.detach().to(self.device, torch.float32).reshape(M0, D).contiguous()
        w = self.coreset_weights()
        if self.learn_z:
            # soft labels as M*C rows (u_i, class c, w_i q_ic), q = softmax(z, 0):
            # sum_c q (log q - log p) = sum_c q NLL(c) + sum_c q log q
            # (psvi_classes.py:496-505; the constant is added by inner_elbo)
            q = torch.softmax(self.z.detach().to(self.device, torch.float32), 0)
            return (u.repeat_interleave(C, 0).contiguous(),
                    torch.arange(C, dtype=torch.int32, device=self.device).repeat(M0).contiguous(),
                    (w[:, None] * q).reshape(-1).contiguous())
        z = self.z.detach().to(self.device).to(torch.int32).contiguous()
        if plan.M == M0:
            return u, z, w
        Wc = torch.zeros(C, dtype=torch.float32, device=self.device).index_add_(0, z.long(), w)
        return (u.repeat_interleave(C, 0).contiguous(),
                torch.arange(C, dtype=torch.int32, device=self.device).repeat(M0).contiguous(),
                Wc.repeat(M0).contiguous())

    def _rows_graph(self, plan):
        """_data's rows as functions of the hyperparameters: the row inputs
        (from u) and weights (N f(v), through v / alpha) with their autograd
        graphs, for the functional inner loop (psvi.robust_higher) and for
        inner_elbo's gradients w.r.t. u and v."""
        M0 = int(self.u.shape[0])
        u_g = self.u.reshape(M0, plan.in_features)
        w_g = (self.N * self.f(self.v, 0)).reshape(-1)
        if self.learn_z:
            q = torch.softmax(self.z, 0)
            return u_g.repeat_interleave(q.shape[1], 0), (w_g[:, None] * q).reshape(-1)
        if plan.M == M0:
            return u_g, w_g
        C = plan.layers[-1][1]
        z = self.z.detach().to(w_g.device).long()
        Wc = torch.zeros(C, dtype=w_g.dtype, device=w_g.device).index_add(0, z, w_g)
        return u_g.repeat_interleave(C, 0), Wc.repeat(M0)

    def _row_grad_fn(self, model, plan, u, z, w, eps, pvec):
        """() -> (d/du, d/dw) of sum_s sum_m w_m NLL_sm over the plan's rows:
        psvi_outer_elbo_grad_coef with pseudo coefficient 1 for every sample
        (the KL term does not depend on the rows)."""
        from ..runtime.sharded import ShardedOuter, pack_coef

        fam, layers, prior_sd, S = model_spec(model)
        key = ("rows", fam, tuple(layers), S, plan.M, prior_sd)

        def fn():
            # built on the first backward that asks for d/du or d/dw, not per objective
            if key not in self._plans:
                self._plans[key] = self._new_plan(fam, layers, S, plan.M, prior_sd, outer=True)
            op = self._plans[key]
            one = torch.ones(S, dtype=torch.float64)
            zero = torch.zeros(S, dtype=torch.float64)
            if isinstance(op, ShardedOuter):
                g = op.coef_grads(plan.M, u, z, w, eps, pvec, one, zero, zero)
            else:
                g = op.outer_grad_coef(plan.M, u, z, w, eps, pvec,
                                       pack_coef(one, zero, zero, 0, S).to(pvec.device))
            return g["grad_u"], g["grad_w"]
        return fn

    def _fold(self, plan, du, dw):
        """Row gradients of _data's rows back onto the pseudopoints."""
        M0 = int(self.u.shape[0])
        if plan.M == M0:
            return du, dw
        C = plan.layers[-1][1]
        z = self.z.detach().to(self.device).long()
        return (du.reshape(M0, C, -1).sum(1),
                dw.reshape(M0, C).sum(0)[z])

    def _anomaly_check(self, what, *tensors):
        """With torch.autograd.set_detect_anomaly on (the reference driver's
        setting, flow_psvi.py:50), a device-side non-finite scan of the step's
        objective values and gradients (psvi_nonfinite) and ONE flag read per
        outer step; raises RuntimeError as anomaly mode does.  Off: nothing."""
        if not torch.is_anomaly_enabled():
            return
        ts = [t.detach().contiguous() for t in tensors if t is not None and t.is_cuda]
        if not ts:
            return
        flag = torch.zeros(1, dtype=torch.int32, device=ts[0].device)
        nonfinite_(flag, *[t if t.dtype in (torch.float32, torch.float64) else t.float()
                           for t in ts])
        if int(flag.item()):
            raise RuntimeError(f"{type(self).__name__}.{what}: non-finite value in the objective "
                               "or its gradients (anomaly detection)")

    def replay_eps(self, draws):
        """Serve the next objective evaluations' noise from ``draws`` (the
        library's eps layout, in call order) instead of the Philox stream --
        to replay the reference's own draws through code that calls
        inner_elbo / psvi_elbo itself (the functional inner loop)."""
        self._eps_feed = iter(list(draws))
        self._eps_short = False

    def _draw_eps(self, plan):
        feed = self._eps_feed
        if feed is not None:
            e = next(feed, None)
            if e is not None:
                return e.to(self.device, torch.float32).reshape(-1).contiguous()
            self._eps_feed = None
            self._eps_short = True   # asked for more draws than were replayed
        eps = torch.empty(plan.eps_count, device=self.device)
        randn_(eps, self.seed, self._eps_offset)
        self._eps_offset += plan.eps_stride  # Philox offsets move in quads
        return eps

    # ---------------------------------------------------------- objectives
    def inner_elbo(self, model=None, params=None, hyperopt=False, eps=None):
        """Negative inner ELBO (psvi_classes.py:488-511), a 0-dim tensor.

        ``params`` (hyperopt=True) is the list of fast weights in module order;
        otherwise the model's own parameters are used.  Fresh eps per call
        (Philox stream of this instance) unless ``eps`` (the library's eps
        layout, ``InnerLoopPlan.eps_count`` floats) is given.  Differentiable
        (first order) w.r.t. those parameters and -- as the reference's
        autograd -- w.r.t. u and v / alpha where they require grad.  The result
        carries ``_psvi_inner`` (plan, rows, draw, gradient) for
        psvi.robust_higher's differentiable optimiser."""
        model = self.model if model is None else model
        plan = self._plan(model)
        plist = list(params) if (hyperopt and params is not None) else list(model.parameters())
        pvec = nn.utils.parameters_to_vector(plist)
        if pvec.numel() != plan.param_count:
            raise ValueError(f"{pvec.numel()} parameters, plan expects {plan.param_count}")
        u, z, w = self._data(plan)
        eps = self._draw_eps(plan) if eps is None else eps
        p = pvec.detach().to(torch.float32).contiguous()
        elbo, grad = plan.elbo_grad(u, z, w, eps, p)
        u_g, w_g = self._rows_graph(plan)
        out = HipInnerELBO.apply(pvec, elbo, grad)
        if u_g.requires_grad or w_g.requires_grad:
            out = out + HipInnerRows.apply(u_g, w_g,
                                           self._row_grad_fn(model, plan, u, z, w, eps, p),
                                           out.dtype)
        if self.learn_z:   # + S sum_m w_m sum_c q log q (KLDivLoss's target entropy term)
            q = torch.softmax(self.z, 0)
            wq = (self.N * self.f(self.v, 0)).reshape(-1, 1) * torch.special.xlogy(q, q)
            out = out + (model_spec(model)[3] * wq.sum()).to(out.dtype)
        out._psvi_inner = dict(plan=plan, u=u, z=z, w=w, eps=eps, u_g=u_g, w_g=w_g, grad=grad,
                               params=p)
        return out

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
                self._eps_offset += plan.eps_stride
                e = step_eps
            else:
                e = eps[t]
            plan.inner_step(u, z, w, e, params, m, v, step=t + 1, lr=lr, kind=kind,
                            elbo_out=elbos[t:t + 1], ws=ws)
        self._anomaly_check("inner_loop", elbos, params)
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
        model = self.model if model is None else model
        fam, layers, prior_sd, S = model_spec(model)
        C = layers[-1][1]
        plist = list(params) if (hyperopt and params is not None) else list(model.parameters())
        pvec = nn.utils.parameters_to_vector(plist)
        xb, yb, w_data = self._outer_rows(xbatch, ybatch, C)
        Nx = int(xb.shape[0])
        if self._outer_mode == "ablated":
            # PSVI_Ablated.psvi_elbo (psvi_classes.py:1397-1408): model(xbatch) only
            if fam == "fullcov":
                raise AttributeError("'int' object has no attribute 'mean': PSVI_Ablated's "
                                     "sampled KL sums VILinear modules only, a full-covariance "
                                     "model has none (psvi_classes.py:1403-1408)")
            plan = self._outer_plan(model, Nx, n_pseudo=0)
            if pvec.numel() != plan.param_count:
                raise ValueError(f"{pvec.numel()} parameters, plan expects {plan.param_count}")
            if eps is None:
                eps = self._draw_eps(plan)
            return HipAblatedELBO.apply(pvec, plan, xb, yb, w_data, eps)
        assert self.mc_samples is None or self.mc_samples > 1  # psvi_classes.py:449
        if S < 2:
            raise ValueError("psvi_elbo needs mc_samples > 1 (psvi_classes.py:449)")
        if self.learn_z:
            return self._soft_psvi_elbo(model, fam, layers, S, pvec, xb, yb, Nx, eps)
        plan = self._outer_plan(model, Nx)
        if pvec.numel() != plan.param_count:
            raise ValueError(f"{pvec.numel()} parameters, plan expects {plan.param_count}")
        self._check_labels(self.z, C)
        z_all = torch.cat([self.z.detach().to(self.device).reshape(-1).to(torch.int32),
                           yb]).contiguous()
        wp = (self.N * self.f(self.v, 0)).to(torch.float32).reshape(-1)
        if eps is None:
            eps = self._draw_eps(plan)
        return HipOuterELBO.apply(pvec, self.u, wp, plan, xb, z_all, w_data, eps)

    def _soft_psvi_elbo(self, model, fam, layers, S, pvec, xb, yb, Nx, eps):
        """psvi_elbo with soft labels (psvi_classes.py:450-486, learn_z): the
        targets of all rows are softmax over rows of cat(z, nc onehot(y)),
        each row r scored sum_c Q_rc (log Q_rc - log p_src).  Rows expand to
        (r, c) with weight w_r Q_rc; the entropy terms shift every sample's
        pseudo term by one constant (no effect on the loss) and its data term
        by cd = N / Nx sum_x sum_c Q_xc log Q_xc, added here."""
        C = layers[-1][1]
        Mu = int(self.u.shape[0])
        R0 = Mu + Nx
        key = ("soft-outer", fam, tuple(layers), S, R0 * C, model_spec(model)[2])
        if key not in self._plans:
            self._plans[key] = self._new_plan(fam, layers, S, R0 * C, model_spec(model)[2],
                                              outer=True)
        plan = self._plans[key]
        if pvec.numel() != plan.param_count:
            raise ValueError(f"{pvec.numel()} parameters, plan expects {plan.param_count}")
        onehot = torch.nn.functional.one_hot(yb.long(), C).to(self.z.dtype) * self.nc_or(C)
        Q = torch.softmax(torch.cat([self.z, onehot]), 0)
        wp = (self.N * self.f(self.v, 0)).reshape(-1)
        w_rows = torch.cat([(wp[:, None] * Q[:Mu]).reshape(-1),
                            (float(self.N) / max(Nx, 1) * Q[Mu:]).reshape(-1)])
        u_rows = self.u.reshape(Mu, -1).repeat_interleave(C, 0)
        x_all = torch.cat([u_rows.detach(), xb.repeat_interleave(C, 0)]).to(torch.float32)
        z_all = torch.arange(C, dtype=torch.int32, device=self.device).repeat(R0).contiguous()
        if eps is None:
            eps = self._draw_eps(plan)
        loss = HipOuterRowsELBO.apply(pvec, u_rows, w_rows, plan, x_all.contiguous(), z_all,
                                      eps, Mu * C)
        cd = float(self.N) / max(Nx, 1) * torch.special.xlogy(Q[Mu:], Q[Mu:]).sum()
        return loss + cd.to(loss.dtype)

    def nc_or(self, C):
        return self.nc if self.nc is not None else C

    def setup_optimizers(self, lr0net=1e-3, lr0u=1e-3, lr0v=1e-2, lr0joint=1e-3,
                         trainer="hyper", lr0z=1e-2):
        """The optimisers run_psvi creates (psvi_classes.py:867-885): Adam on
        the network, on u, on v (learn_v), and for trainer 'joint' one Adam
        over all of them."""
        self.u.requires_grad_(True)
        self.optim_net = torch.optim.Adam(list(self.model.parameters()), lr0net)
        self.optim_u = torch.optim.Adam([self.u], lr0u)
        if self.learn_v:
            self.optim_v = torch.optim.Adam([self.v], lr0v)
        if self._alpha() is not None:   # PSVIAV / PSVIAFixedU (psvi_classes.py:1489, 1761)
            self.optim_alpha = torch.optim.Adam([self.alpha], self.lr0alpha)
        if self.learn_z:                 # psvi_classes.py:869-870
            self.z.requires_grad_(True)
            self.optim_z = torch.optim.Adam([self.z], lr0z)
        if trainer == "joint":
            vp = list(self.model.parameters()) + [self.u] + ([self.v] if self.learn_v else [])
            self.optim = torch.optim.Adam(vp, lr0joint)

    @_trainer_step
    def joint_step(self, xbatch, ybatch):
        """psvi_classes.py:517-525: one Adam step on the outer objective over
        the network, u (and v)."""
        self.optim.zero_grad()
        loss = self.psvi_elbo(xbatch, ybatch, model=self.model)
        with torch.no_grad():
            if self.register_elbos:
                self.elbos.append((2, -loss.item()))
        loss.backward()
        self._raise_bad_labels()
        self.optim.step()
        return loss

    @_trainer_step
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
            self._raise_bad_labels()
            self.optim.step()
        return loss

    # ------------------------------------------------------------ evaluation
    def _predict(self, x_rows, y_rows, correction, probs, eps):
        model = self.model
        plan = self._outer_plan(model, int(x_rows.shape[0]))
        Mu = int(self.u.shape[0])
        x_all = torch.cat([self.u.detach().reshape(Mu, -1).to(torch.float32),
                           x_rows]).contiguous()
        if self.learn_z:
            # psvi_classes.py:1049-1056: with soft labels the pseudo term is one
            # scalar summed over the samples, so W = softmax_s(sampled_nkl_s)
            zp = torch.zeros(Mu, dtype=torch.int32, device=self.device)
            wp = torch.zeros(Mu, device=self.device)
        else:
            zp = self.z.detach().to(self.device).reshape(-1)
            wp = self.coreset_weights()
        z_all = torch.cat([zp, y_rows.to(self.device).reshape(-1)]).to(torch.int32).contiguous()
        w_all = torch.cat([wp, torch.zeros(x_rows.shape[0], device=self.device)]).contiguous()
        with torch.no_grad():
            pvec = nn.utils.parameters_to_vector(model.parameters()).detach().to(torch.float32)
        e = eps if eps is not None else self._draw_eps(plan)
        return plan.evaluate(Mu, x_all, z_all, w_all, e, pvec.contiguous(), correction, probs)

    def evaluate(self, correction=True, eps=None, **kwargs):
        """Importance-weighted predictive metrics over self.test_loader
        (psvi_classes.py:1031-1108): (accuracy, mean test NLL, entropy of the
        importance weights, normalised ESS, v-entropy), one psvi_evaluate per
        test batch (fresh weights per batch; entropy / ESS from the last one,
        as the reference).  ``eps``: optional list of draws, one per batch."""
        assert self.mc_samples is None or self.mc_samples > 1
        it = iter(eps) if eps is not None else None
        correct = nll = last = None
        total = 0
        for xt, yt in self.test_loader:
            xt = xt.to(self.device, torch.float32).reshape(xt.shape[0], -1)
            st, _ = self._predict(xt, yt, correction, False, next(it) if it else None)
            correct = st[2] if correct is None else correct + st[2]
            nll = st[3] if nll is None else nll + st[3]
            total += int(xt.shape[0])
            last = st
        iw_entropy = last[0] if self.compute_weights_entropy else None
        ness = last[1]
        vs = self.f(self.v, 0)
        v_entropy = (vs.sum().square() / vs.square().sum() / self.num_pseudo
                     if self.compute_weights_entropy else None)
        return correct / float(total), nll / float(total), iw_entropy, ness, v_entropy

    def pred_on_grid(self, n_test_per_dim=250, correction=True, eps=None, **kwargs):
        """Predictive probabilities over a 2-d grid (psvi_classes.py:1130-1175):
        (n_test_per_dim^2, C) with the same importance weights as evaluate."""
        x0 = torch.linspace(-3, 4, n_test_per_dim)
        x1 = torch.linspace(-2, 3, n_test_per_dim)
        x_test = torch.stack(torch.meshgrid(x0, x1, indexing="ij"), dim=-1).to(self.device)
        x_rows = x_test.reshape(-1, 2).to(torch.float32).contiguous()
        y = torch.zeros(x_rows.shape[0], device=self.device)
        _, probs = self._predict(x_rows, y, correction, True, eps)
        return probs

    # ------------------------------------------------------- second order
    def _outer_plan(self, model, Nx, n_pseudo=None):
        fam, layers, prior_sd, S = model_spec(model)
        Mu = int(self.u.shape[0]) if n_pseudo is None else int(n_pseudo)
        key = ("outer", fam, tuple(layers), S, Mu + Nx, prior_sd)
        if key not in self._plans:
            self._plans[key] = self._new_plan(fam, layers, S, Mu + Nx, prior_sd, outer=True)
        return self._plans[key]

    def _alpha(self):
        return getattr(self, "alpha", None)

    def _chain_w(self, dw):
        """(d/dv, d/dalpha) of a linear function of w = N f(v) with coefficients
        dw; d/dalpha is None without alpha (PSVIAV / PSVIAFixedU have it)."""
        alpha = self._alpha()
        with torch.enable_grad():
            v = self.v.detach().requires_grad_(True)
            hp = [v]
            if alpha is not None:
                a = alpha.detach().requires_grad_(True)
                hp.append(a)
                wp = self.N * torch.exp(a) * torch.softmax(v, 0)
            else:
                wp = self.N * self.f(v, 0)
            gs = torch.autograd.grad(wp, hp, grad_outputs=dw.to(wp.dtype).reshape(wp.shape))
        return gs[0], (gs[1] if alpha is not None else None)

    @staticmethod
    def _add_grad(t, g):
        g = g.reshape(t.shape).to(t.dtype)
        if t.grad is None:
            t.grad = g.clone()
        else:
            t.grad += g

    def _hparam_steps(self, u_grad, w_grad):
        """Accumulate the hypergradients and step the outer optimisers: optim_u
        (unless u is frozen), optim_v (learn_v; clamped at 0 unless
        parameterised) and optim_alpha (psvi_classes.py:585-591, 676-681,
        1576-1579, 1610-1612, 1650-1651, 1843-1845, 1873-1875)."""
        self._raise_bad_labels()
        if self._learn_u:
            self._add_grad(self.u, u_grad)
            self.optim_u.step()
        if self.learn_v:
            gv, ga = self._chain_w(w_grad)
            self._add_grad(self.v, gv)
            if ga is not None:
                self._add_grad(self.alpha, ga)
            self.optim_v.step()
            if ga is not None:
                self.optim_alpha.step()
            if not getattr(self, "parameterised", False):
                with torch.no_grad():
                    torch.clamp_(self.v, min=0.0)

    def _zero_hparam_grads(self):
        if self._learn_u:
            self.optim_u.zero_grad()
        else:
            self.u.requires_grad_(False)        # psvi_classes.py:1632, 1664, 1821, 1863
        if self.learn_v:
            self.optim_v.zero_grad()
        if self._alpha() is not None and hasattr(self, "optim_alpha"):
            self.optim_alpha.zero_grad()

    def _outer_rows(self, xbatch, ybatch, C):
        xb = xbatch.detach().to(self.device, torch.float32).reshape(xbatch.shape[0], -1)
        yb = self._batch_labels(ybatch.detach().to(self.device), C)
        Nx = int(xb.shape[0])
        return xb.contiguous(), yb, torch.full((Nx,), float(self.N) / max(Nx, 1),
                                               device=self.device)

    def _outer_fn(self, model, xbatch, ybatch, u, z, params):
        """(plan, f(u, w, eps, grads) -> dict(loss, grad, grad_u, grad_w)) of this
        class's outer objective at fixed parameters (float32 device tensors)."""
        fam, layers, _, _ = model_spec(model)
        xb, yb, w_data = self._outer_rows(xbatch, ybatch, layers[-1][1])
        Nx = int(xb.shape[0])
        if self._outer_mode == "ablated":
            if fam == "fullcov":
                raise AttributeError("'int' object has no attribute 'mean': PSVI_Ablated's "
                                     "sampled KL sums VILinear modules only, a full-covariance "
                                     "model has none (psvi_classes.py:1403-1408)")
            oplan = self._outer_plan(model, Nx, n_pseudo=0)

            def f(uu, ww, eps, grads=True):
                o = oplan.outer_ablated_elbo_grad(xb, yb, w_data, eps, params, grad=grads)
                if grads:
                    o["grad_u"] = torch.zeros_like(uu)
                    o["grad_w"] = torch.zeros(uu.shape[0], device=uu.device)
                return o
            return oplan, f
        oplan = self._outer_plan(model, Nx)
        z_all = torch.cat([z, yb]).contiguous()

        def f(uu, ww, eps, grads=True):
            x_all = torch.cat([uu.detach().reshape(uu.shape[0], -1), xb]).contiguous()
            w_all = torch.cat([ww.detach().to(torch.float32), w_data]).contiguous()
            return oplan.outer_elbo_grad(int(uu.shape[0]), x_all, z_all, w_all, eps, params,
                                         grad=grads, grad_u=grads, grad_w=grads)
        return oplan, f

    @_trainer_step
    def hyper_step(self, xbatch, ybatch, T=50, inner_opt_class=None, K=30, linsys_lr=1e-4,
                   hypergrad_approx="CG_normaleq", eps_inner=None, eps_outer=None, **kwargs):
        """psvi_classes.py:602-687 with hypergrad's CG_normaleq
        (hypergradients.py:199-244, CG_torch.py:9-45): T = self.inner_it
        first-order inner steps (hypergrad adam_step, step count 1..T) from the
        model's parameters, then the implicit hypergradient of the hparams --
        u (unless frozen), v (learn_v) and alpha (PSVIAV / PSVIAFixedU,
        1504-1581, 1774-1850) -- from K conjugate-gradient iterations on the
        normal equations of fp_map(p) = p - linsys_lr * grad_p inner, their
        Adam steps, and the outer loss at the new hparams -- returned as a
        float; the final parameters are written into the model.
        ``eps_inner`` / ``eps_outer``: optional sequences of draws (library eps
        layout) in the reference's call order, to replay; default: this
        instance's Philox stream."""
        if hypergrad_approx not in ("CG_normaleq", "fixed_point"):
            raise NotImplementedError(f"hypergrad_approx={hypergrad_approx!r}: the reference's "
                                      "hyper_step offers CG_normaleq and fixed_point")
        if self.learn_z:
            raise NotImplementedError  # as the reference (psvi_classes.py:619-620)
        T = self.inner_it
        lr_net = self.optim_net.param_groups[0]["lr"]
        model = self.model
        self._zero_hparam_grads()
        plan = self._plan(model)
        u, z, w = self._data(plan)
        it_in = iter(eps_inner) if eps_inner is not None else None
        it_out = iter(eps_outer) if eps_outer is not None else None

        def draw_inner():
            return next(it_in) if it_in is not None else self._draw_eps(plan)

        # 1. the inner problem: T first-order steps (trainer hyper: hypergrad adam_step)
        plist = list(model.parameters())
        with torch.no_grad():
            params = nn.utils.parameters_to_vector(plist).detach().to(torch.float32).clone()
        m = torch.zeros_like(params)
        v2 = torch.zeros_like(params)
        if it_in is None:  # fused loop on this instance's Philox stream
            plan.inner_loop(u, z, w, params, m, v2, T, lr_net, kind="hypergrad", seed=self.seed,
                            offset=self._eps_offset)
            self._eps_offset += T * plan.eps_stride
        else:
            ws = plan.workspace(params.device)
            for t in range(T):
                plan.inner_step(u, z, w, draw_inner(), params, m, v2, step=t + 1, lr=lr_net,
                                kind="hypergrad", ws=ws)
        # 2. the outer objective's direct gradients, then CG_normaleq / fixed_point
        u0 = self.u.detach().to(self.device, torch.float32).reshape(self.u.shape[0], -1)
        z0 = self.z.detach().to(self.device).reshape(-1).to(torch.int32)
        oplan, outer = self._outer_fn(model, xbatch, ybatch, u0, z0, params)

        def draw_outer():
            return next(it_out) if it_out is not None else self._draw_eps(oplan)

        o = outer(u0, self.coreset_weights(), draw_outer())
        g_w = o["grad"].to(torch.float64)
        lr = float(linsys_lr)
        hws = torch.empty(plan.hvp_ws_bytes, dtype=torch.uint8, device=params.device)

        def hvp(e, x, mixed=False, f64=True):
            hv, du, dw = plan.hvp(u, z, w, e, params, x.to(torch.float32).contiguous(),
                                  mixed=mixed, ws=hws)
            if mixed:
                du, dw = self._fold(plan, du, dw)
            return (hv.to(torch.float64) if f64 else hv), du, dw

        if hypergrad_approx == "fixed_point":
            # hypergradients.py:83-140 with stochastic=True: a fresh fp_map per iteration
            vs = torch.zeros_like(g_w)
            for _ in range(int(K)):
                prev = vs
                vs = vs - lr * hvp(draw_inner(), vs)[0] + g_w
                if float(torch.linalg.vector_norm(vs - prev)) < 1e-10:
                    break
            xk, eA = vs, draw_inner()
        else:
            # replayed draws: the reference's exact number of fp_map draws (the
            # host reads the stopping flag every iteration); the Philox stream:
            # every 5th iteration (up to 4 discarded iterations after convergence)
            eA = self._cg_normaleq(hvp, draw_inner, g_w, lr, K,
                                   sync_every=1 if it_in is not None else 5)
            xk = self._cg_x
        _, du, dw = hvp(eA, xk, mixed=True)     # torch_grad(w_mapped, hparams, vs)
        # 3. hypergradient = -lr * mixed products + the outer objective's direct gradients
        u_grad = (-lr * du.to(torch.float64) + o["grad_u"].to(torch.float64)).to(self.u.dtype)
        w_grad = -lr * dw.to(torch.float64) + o["grad_w"].to(torch.float64)
        self._anomaly_check("hyper_step", o["loss"], params, u_grad, w_grad)
        self._hparam_steps(u_grad, w_grad)
        # 4. the outer loss at the new hparams, and the inner solution into the model
        u1 = self.u.detach().to(self.device, torch.float32).reshape(self.u.shape[0], -1)
        ll = outer(u1, self.coreset_weights(), draw_outer(), grads=False)["loss"]
        with torch.no_grad():
            nn.utils.vector_to_parameters(params.to(plist[0].dtype), plist)
        return float(ll.item())

    def _cg_normaleq(self, hvp, draw_inner, g_w, lr, K, sync_every=1):
        """CG_normaleq's linear solve (hypergradients.py:199-244, CG_torch.py:9-45);
        returns the draw of w_mapped, leaves the solution in self._cg_x.
        The iteration's vector work runs fused on the device
        (psvi.runtime.cg.DeviceCG: psvi_cg_*), its stopping test too: x and p
        freeze where the reference breaks, and the host leaves the loop when
        it reads the flag, every ``sync_every`` iterations (1: the reference's
        number of A calls, hence of draws)."""
        from psvi.runtime.cg import DeviceCG

        eA = draw_inner()                       # w_mapped = fp_map(params, hparams)

        def hv_a(x32):                          # H_A x (fp32, as psvi_hvp returns it)
            return hvp(eA, x32, f64=False)[0]

        def hv_b(x32):                          # J's product: fp_map drawn twice
            draw_inner()
            return hvp(draw_inner(), x32, f64=False)[0]

        # b = g_w - J g_w, J g_w = g_w - lr H g_w (fp32 H g_w promoted in the one pass)
        b = g_w - torch.sub(g_w, hv_b(g_w.to(torch.float32)), alpha=lr)
        if not b.is_cuda:
            # host tensors (the CPU rehearsals of the sharded trainers, whose
            # plans are stand-ins): the same iteration in torch
            from psvi.hypergrad.CG_torch import cg as torch_cg

            def A(xs):
                vmj = hv_a(xs[0].to(torch.float32)).to(torch.float64) * lr
                return [vmj - torch.sub(vmj, hv_b(vmj.to(torch.float32)), alpha=lr)]

            self._cg_x = torch_cg(A, [b], max_iter=int(K), epsilon=1e-10,
                                  sync_every=sync_every)[0]
            return eA
        cg = getattr(self, "_cg_dev", None)
        if cg is None or cg.n != b.numel() or cg.state.device != b.device:
            cg = self._cg_dev = DeviceCG(b.numel(), b.device)
        xk = cg.solve(hv_a, hv_b, b.contiguous(), lr, K, tol=1e-10, sync_every=sync_every)
        self._cg_x = xk
        return eA

    @_trainer_step
    def nested_step(self, xbatch, ybatch, truncated=False, K=5, eps_inner=None, eps_outer=None):
        """psvi_classes.py:541-600 (and the variants' overrides, 1583-1620,
        1631-1657, 1852-1884): T = self.inner_it higher-Adam steps on the inner
        objective from the model's parameters with a fresh Adam state, the
        outer objective at the result, its gradient w.r.t. the hparams (u
        unless frozen, v, alpha) through the unrolled steps, their Adam steps;
        the final parameters are written into the model.  Returns the outer
        loss (0-dim tensor).  ``eps_inner`` (T draws) / ``eps_outer`` (1):
        optional replay of the reference's draws; default this instance's
        Philox stream."""
        if truncated or self.learn_z:
            replay = eps_inner is not None or eps_outer is not None
            if replay:
                self.replay_eps(list(eps_inner or []) + list(eps_outer or []))
            out = self._nested_step_unrolled(xbatch, ybatch, truncated, K)
            if replay and (self._eps_short or next(self._eps_feed or iter(()), None) is not None):
                raise ValueError("eps_inner / eps_outer do not hold exactly the draws the step "
                                 "consumed")
            return out
        self._zero_hparam_grads()
        self.optim_net.zero_grad()
        model = self.model
        T = int(self.inner_it)
        lr_net = self.optim_net.param_groups[0]["lr"]
        plan = self._plan(model)
        u, z, w = self._data(plan)
        it_in = iter(eps_inner) if eps_inner is not None else None
        plist = list(model.parameters())
        with torch.no_grad():
            p = nn.utils.parameters_to_vector(plist).detach().to(torch.float32).clone()
        m = torch.zeros_like(p)
        v2 = torch.zeros_like(p)
        ws = plan.workspace(p.device)
        hist, elbos = [], []
        # forward: the unrolled inner loop, trajectory kept for the reverse pass
        for t in range(T):
            e = next(it_in) if it_in is not None else self._draw_eps(plan)
            elbo, g = plan.elbo_grad(u, z, w, e, p, ws=ws)
            p_prev = p.clone()
            adam_update_(p, g, m, v2, t + 1, lr_net, kind="higher")
            hist.append((p_prev, m.clone(), v2.clone(), g, e))
            elbos.append(elbo)
        # the outer objective at the inner solution, and its direct gradients
        u0 = self.u.detach().to(self.device, torch.float32).reshape(self.u.shape[0], -1)
        z0 = self.z.detach().to(self.device).reshape(-1).to(torch.int32)
        oplan, outer = self._outer_fn(model, xbatch, ybatch, u0, z0, p)
        eo = next(iter(eps_outer)) if eps_outer is not None else self._draw_eps(oplan)
        o = outer(u0, self.coreset_weights(), eo)
        if self.register_elbos:
            host = torch.cat(elbos).cpu()
            for t in range(0, T, self.log_every):
                self.elbos.append((1, -float(host[t])))
            self.elbos.append((0, -float(o["loss"].item())))
        # reverse mode through the T Adam steps
        lt = o["grad"].clone()
        lm = torch.zeros_like(p)
        lv = torch.zeros_like(p)
        lg = torch.empty_like(p)
        gu = o["grad_u"].clone()
        gw = o["grad_w"].clone()
        hws = torch.empty(plan.hvp_ws_bytes, dtype=torch.uint8, device=p.device)
        for t in range(T - 1, -1, -1):
            p_prev, mt, vt, gt, e = hist[t]
            adam_adjoint_(lt, lm, lv, mt, vt, gt, t + 1, lr_net, lg, kind="higher")
            hv, du, dw = plan.hvp(u, z, w, e, p_prev, lg, ws=hws)
            du, dw = self._fold(plan, du, dw)
            lt += hv
            gu += du.reshape(gu.shape)
            gw += dw
        self._anomaly_check("nested_step", torch.cat(elbos), o["loss"], p, gu, gw)
        self._hparam_steps(gu, gw)
        if getattr(self, "scheduler_optim_net", None):
            self.scheduler_optim_net.step()
        with torch.no_grad():
            nn.utils.vector_to_parameters(p.to(plist[0].dtype), plist)
        return o["loss"].reshape(()).to(torch.float32)

    def _nested_step_unrolled(self, xbatch, ybatch, truncated=False, K=5):
        """nested_step on psvi.robust_higher's differentiable inner loop, in the
        reference's own order (psvi_classes.py:541-600, PSVIAV 1587-1620,
        PSVIAFixedU 1852-1884): the hypergradients of u, v, alpha and the soft
        labels z reach them through autograd.  truncated (561-583): first
        inner_it - K non-differentiable steps of torch.optim.Adam (lr 1e-4) on
        the inner objective, whose backward accumulates into the network's,
        u's, v's and z's gradients without zeroing between steps (as the
        reference's loop: the psvi_elbo hypergradient is added on top); then K
        differentiable steps."""
        from ..robust_higher import innerloop_ctx

        self._zero_hparam_grads()
        self.optim_net.zero_grad()
        if self.learn_z:
            self.optim_z.zero_grad()
        n_diff = self.inner_it
        if truncated:
            plist = list(self.model.parameters())
            p = nn.utils.parameters_to_vector(plist).detach().to(torch.float32).clone()
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            for in_it in range(self.inner_it - K):
                mfvi_loss = self.inner_elbo(model=self.model)
                with torch.no_grad():
                    if self.register_elbos and in_it % self.log_every == 0:
                        self.elbos.append((1, -mfvi_loss.item()))
                mfvi_loss.backward()
                # inner_opt.step(): torch.optim.Adam on the accumulated gradients
                g = torch.cat([(q.grad if q.grad is not None else torch.zeros_like(q)).reshape(-1)
                               for q in plist]).to(torch.float32).contiguous()
                adam_update_(p, g, m, v, in_it + 1, 1e-4, kind="torch")
                with torch.no_grad():
                    nn.utils.vector_to_parameters(p.to(plist[0].dtype), plist)
            for q in plist:           # inner_opt.zero_grad()
                q.grad = None
            n_diff = K
        with innerloop_ctx(self.model, self.optim_net) as (fmodel, diffopt):
            for in_it in range(n_diff):
                mfvi_loss = self.inner_elbo(model=fmodel)
                with torch.no_grad():
                    if self.register_elbos and in_it % self.log_every == 0:
                        self.elbos.append((1, -mfvi_loss.item()))
                diffopt.step(mfvi_loss)
            psvi_loss = self.psvi_elbo(xbatch, ybatch, model=fmodel)
            with torch.no_grad():
                if self.register_elbos:
                    self.elbos.append((0, -psvi_loss.item()))
            psvi_loss.backward()
        self._anomaly_check("nested_step", psvi_loss.reshape(1), fmodel.flat,
                            *[t.grad for t in (self.u, self.v, self.z) if t is not None
                              and getattr(t, "grad", None) is not None])
        if self._learn_u:
            self.optim_u.step()
        if self.learn_v:
            self.optim_v.step()
            if self._alpha() is not None:
                self.optim_alpha.step()
            if not getattr(self, "parameterised", False):
                with torch.no_grad():
                    torch.clamp_(self.v, min=0.0)
        if self.learn_z:
            self.optim_z.step()
        if getattr(self, "scheduler_optim_net", None):
            self.scheduler_optim_net.step()
        with torch.no_grad():
            nn.utils.vector_to_parameters(
                nn.utils.parameters_to_vector(list(fmodel.parameters())).to(
                    next(self.model.parameters()).dtype), self.model.parameters())
        return psvi_loss

    # ------------------------------------------------------------ the driver
    def set_up_model(self):
        """psvi_classes.py:689-758 for the architectures the HIP path runs:
        logistic_regression (VILinear), logistic_regression_fullcov, fn
        (make_fcnet, n_layers), fn2 (make_fc2net: always 2 hidden layers, the
        reference does not forward n_layers)."""
        kw = dict(init_sd=self.init_sd, mc_samples=self.mc_samples)
        if self.logistic_regression:
            self.model = nn.Sequential(VILinear(self.D, self.nc, **kw))
        elif self.architecture == "logistic_regression_fullcov":
            self.model = nn.Sequential(VILinearMultivariateNormal(self.D, self.nc, **kw))
        elif self.architecture == "fn":
            self.model = make_fcnet(self.D, self.n_hidden, self.nc, n_layers=self.n_layers,
                                    linear_class=VILinear, nonl_class=nn.ReLU, **kw)
        elif self.architecture == "fn2":
            self.model = make_fc2net(self.D, self.n_hidden, self.nc,
                                     linear_class=VILinearMultivariateNormal, nonl_class=nn.ReLU,
                                     **kw)
        elif self.architecture == "lenet":
            # inner loop only on the HIP path (psvi_elbo / HVP for LeNet: not built)
            self.model = make_lenet(linear_class=VILinear, nonl_class=nn.ReLU, **kw)
        else:
            raise NotImplementedError(f"architecture {self.architecture!r} is not on the HIP path "
                                      "(alexnet / resnet / residual_fn / regressor_net)")
        self.model = self.model.to(self.device)

    @staticmethod
    def _xy(dataset):
        x = getattr(dataset, "data", None)
        y = getattr(dataset, "targets", None)
        if x is None or y is None:
            if hasattr(dataset, "tensors"):
                x, y = dataset.tensors[0], dataset.tensors[1]
            else:
                x = torch.stack([dataset[i][0] for i in range(len(dataset))])
                y = torch.as_tensor([dataset[i][1] for i in range(len(dataset))])
        return torch.as_tensor(x).float(), torch.as_tensor(y)

    def pseudo_subsample_init(self):
        """psvi_classes.py:229-285: the pseudodata start on a random subset with
        an equal number of points per class (the remainder on the last class)."""
        x, y = self._xy(self.train_dataset if self.init_dataset is None else self.init_dataset)
        ppc = [self.num_pseudo // self.nc] * self.nc
        ppc[-1] = self.num_pseudo - sum(ppc[:-1])
        self.z = torch.tensor([c for c, k in enumerate(ppc) for _ in range(k)]).float().to(
            self.device)
        us = []
        for c in range(self.nc):
            idx = (y == c).nonzero().reshape(-1)
            us.append(x[idx[torch.randperm(idx.numel())[:ppc[c]]]])
        self.u = torch.cat(us).reshape(self.num_pseudo, -1).to(self.device).requires_grad_(True)
        self._soft_label_init()

    def pseudo_rand_init(self, variance=1.0):
        """psvi_classes.py:287-308: noisy empirical mean, labels split over classes."""
        x, _ = self._xy(self.train_dataset)
        mean = x.reshape(x.shape[0], -1).mean(0)
        self.u = (mean + variance * torch.randn(self.num_pseudo, self.D)).to(
            self.device).requires_grad_(True)
        per = self.num_pseudo // self.nc
        self.z = torch.cat([c * torch.ones(per if c < self.nc - 1
                                           else self.num_pseudo - (self.nc - 1) * per)
                            for c in range(self.nc)]).to(self.device)
        self._soft_label_init()

    def _soft_label_init(self):
        """learn_z: labels as logits close to one-hot (psvi_classes.py:259-264)."""
        if self.learn_z:
            self.z = torch.nn.functional.one_hot(self.z.long(), num_classes=self.nc).float()
            self.z.requires_grad_(True)

    def run_psvi(self, init_args="subsample", trainer="nested", n_layers=1,
                 logistic_regression=True, n_hidden=None, architecture=None, log_every=10,
                 inner_it=10, data_minibatch=None, lr0net=1e-3, lr0u=1e-3, lr0joint=1e-3,
                 lr0v=1e-2, lr0z=1e-2, init_sd=1e-3, num_epochs=1000, log_pseudodata=False,
                 prune_idx=0, increment_idx=0, gamma=1.0, **kwargs):
        """psvi_classes.py:761-1028 on the HIP trainers: data loaders, model set-up,
        pseudodata initialisation, the optimisers and StepLR of the reference,
        then num_epochs outer steps of `trainer` (nested / hyper / joint /
        alternating), evaluating every log_every; returns the results dict
        (accs, nlls, csizes, times, elbos, went, ness, vent, vs, avg_epoch_time,
        gpu_memory, chosen_indices; us, zs, grid_preds with log_pseudodata)."""
        from torch.utils.data import DataLoader

        if init_args not in ("subsample", "random"):
            raise NotImplementedError(f"init_args={init_args!r}: custom / saved initialisations "
                                      "read the reference's selection and results files")
        self.init_args, self.trainer = init_args, trainer
        self.logistic_regression, self.architecture = logistic_regression, architecture
        self.n_hidden, self.n_layers, self.init_sd = n_hidden, n_layers, init_sd
        self.log_every, self.log_pseudodata = log_every, log_pseudodata
        self.data_minibatch, self.inner_it, self.num_epochs = data_minibatch, inner_it, num_epochs
        self.gamma = gamma
        epoch_quarter = (self.N // self.data_minibatch) // 4
        self.train_loader = DataLoader(self.train_dataset, batch_size=self.data_minibatch,
                                       shuffle=True)
        self.test_loader = DataLoader(self.test_dataset, batch_size=self.data_minibatch,
                                      shuffle=False)
        self.set_up_model()
        (self.pseudo_subsample_init if init_args == "subsample" else self.pseudo_rand_init)()
        self.setup_optimizers(lr0net=lr0net, lr0u=lr0u, lr0v=lr0v, lr0joint=lr0joint,
                              trainer=trainer, lr0z=lr0z)
        self.scheduler_optim_net = torch.optim.lr_scheduler.StepLR(
            self.optim_net, step_size=epoch_quarter if epoch_quarter > 0 else 10000,
            gamma=self.gamma)
        steps = {"nested": self.nested_step, "hyper": self.hyper_step,
                 "alternating": self.alternating_step, "joint": self.joint_step}
        if trainer not in steps:
            raise ValueError(f"unknown trainer {trainer!r}")
        psvi_step = steps[trainer]
        accs, nlls, csizes, went, ness_l, vent, us, zs, vs, grid, times = \
            [], [], [], [], [], [], [], [], [], [], [0]
        t_start = time.time()
        lpit = list(range(num_epochs))[::log_every]
        for it in range(num_epochs):
            xbatch, ybatch = next(iter(self.train_loader))
            xbatch, ybatch = xbatch.to(self.device), ybatch.to(self.device)
            if it % log_every == 0:
                acc, nll, iw_ent, ness, v_ent = self.evaluate()
                if log_pseudodata and it in lpit and self.D == 2:
                    grid.append(self.pred_on_grid().detach().cpu().numpy().T)
                with torch.no_grad():
                    nlls.append(nll.item())
                    accs.append(acc.item())
                    csizes.append(self.num_pseudo)
                    times.append(times[-1] + time.time() - t_start)
                    vs.append(self.v.clone().cpu().detach().numpy())
                    if iw_ent is not None:
                        went.append(iw_ent.item())
                    if ness is not None:
                        ness_l.append(ness.item())
                    if v_ent is not None:
                        vent.append(v_ent.item())
                    if log_pseudodata:
                        us.append(self.u.clone().cpu().detach().numpy())
                        zs.append(self.z.clone().cpu().detach().numpy())
            psvi_step(xbatch, ybatch)
        torch.cuda.synchronize()
        self.results.update(
            accs=accs, nlls=nlls, csizes=csizes, times=times[1:], elbos=self.elbos, went=went,
            ness=ness_l, vent=vent, vs=vs,
            avg_epoch_time=(time.time() - t_start) / max(num_epochs, 1),
            gpu_memory=torch.cuda.max_memory_allocated(self.device) / 2 ** 30,
            chosen_indices=self.chosen_indices)
        if log_pseudodata:
            self.results.update(us=us, zs=zs, grid_preds=grid)
        return self.results


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
    """PSVILearnV with the ablated outer objective (psvi_classes.py:1388-1408):
    psvi_elbo = mean_s (N/Nx) sum_x NLL_s(x) - mean_s sampled_nkl_s over the data
    batch only, no importance weights over samples; u and v reach it only
    through the inner loop.  On a full-covariance model the reference's sum over
    VILinear modules is the int 0 and raises AttributeError; so does this."""

    _outer_mode = "ablated"


class PSVI_No_IW(PSVI_Ablated):
    """Single-sample training, multi-sample testing (psvi_classes.py:1411-1472):
    mc_samples = 1 for the inner loop and the ablated outer objective;
    evaluate / pred_on_grid switch the mean-field layers to mc_samples_eval
    samples and back.  With one sample the reference's inner objective scores
    every pseudo row against every pseudo label (2-d logits unsqueezed to
    (M, 1, C), psvi_classes.py:492-493); the HIP path runs it as M*C expanded
    rows.  Mean-field models only (full-covariance ones fail in the reference's
    ablated objective)."""

    _noiw = True

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.mc_samples = 1

    def _multi(self, mc_samples_eval, mc_samples_train, fn):
        from ..models.neural_net import set_mc_samples

        self.mc_samples = mc_samples_eval
        set_mc_samples(self.model, mc_samples_eval)
        try:
            return fn()
        finally:
            self.mc_samples = 1
            set_mc_samples(self.model, mc_samples_train)

    def evaluate(self, correction=True, mc_samples_eval=5, mc_samples_train=1, **kwargs):
        """psvi_classes.py:1423-1447: PSVI.evaluate with mc_samples_eval samples."""
        return self._multi(mc_samples_eval, mc_samples_train,
                           lambda: PSVI.evaluate(self, correction=True, **kwargs))

    def pred_on_grid(self, correction=True, n_test_per_dim=250, mc_samples_eval=5,
                     mc_samples_train=1, **kwargs):
        """psvi_classes.py:1449-1472."""
        return self._multi(mc_samples_eval, mc_samples_train,
                           lambda: PSVI.pred_on_grid(self, n_test_per_dim=n_test_per_dim,
                                                     correction=correction, **kwargs))


class PSVIAV(PSVILearnV):
    """Learnable simplex weights times a learnable total evidence exp(alpha)
    (psvi_classes.py:1475-1620): hparams [u, v, alpha]; optim_alpha (Adam,
    lr0alpha) steps with optim_v in nested_step / hyper_step.  Like the
    reference, trainer 'joint' leaves alpha out of its optimiser (867-881)."""

    def __init__(self, learn_v=True, **kwargs):
        super().__init__(**kwargs)
        _init_alpha(self)

    def evaluate(self, **kwargs):
        """psvi_classes.py:1492-1499: records alpha, then PSVI.evaluate."""
        self.results.setdefault("alpha", []).append(self.alpha.clone().cpu().detach().numpy())
        return super().evaluate(**kwargs)


class PSVIFixedU(PSVILearnV):
    """Fixed pseudopoint locations (psvi_classes.py:1622-1740): u is frozen
    (requires_grad False, optim_u never stepped), only v is learned."""

    _learn_u = False

    def hyper_step(self, xbatch, ybatch, *args, **kwargs):
        """The reference hands hypergrad a DifferentiableAdam as fp_map
        (psvi_classes.py:1710-1712): its 3-way split of the plain parameter list
        makes the functional model call fail with IndexError before anything
        moves.  Reproduced: the same error."""
        self.u.requires_grad_(False)
        if self.learn_v:
            self.optim_v.zero_grad()
        raise IndexError("list index out of range: PSVIFixedU.hyper_step's fp_map is a "
                         "DifferentiableAdam over the plain parameter list "
                         "(psvi_classes.py:1710-1712), as in the reference")


class PSVIAFixedU(PSVILearnV):
    """Fixed pseudopoint locations, learnable simplex weights and evidence scale
    exp(alpha) (psvi_classes.py:1743-1884): hparams [v, alpha]."""

    _learn_u = False

    def __init__(self, learn_v=True, **kwargs):
        super().__init__(**kwargs)
        _init_alpha(self)

    def evaluate(self, **kwargs):
        """psvi_classes.py:1761-1768: records alpha, then PSVI.evaluate."""
        self.results.setdefault("alpha", []).append(self.alpha.clone().cpu().detach().numpy())
        return super().evaluate(**kwargs)


def _init_alpha(obj):
    """alpha = 0, f = exp(alpha) softmax(v) and its Adam (psvi_classes.py:1482-1490)."""
    obj.alpha = torch.tensor([0.0], device=obj.device)
    obj.alpha.requires_grad_(True)
    obj.f = lambda *x: torch.exp(obj.alpha) * torch.softmax(x[0], x[1])
    obj.optim_alpha = torch.optim.Adam([obj.alpha], obj.lr0alpha)
    obj.results["alpha"] = []
