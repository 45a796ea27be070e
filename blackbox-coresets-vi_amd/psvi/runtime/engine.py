"""Host wrapper around one libpsvi_hip plan.

``InnerLoopPlan`` owns a ``psvi_plan`` (geometry + device work lists) and
launches the fused HIP inner step, the autograd-boundary ELBO/gradient, or the
sharded phases on torch's current HIP stream.  All tensors are caller-owned
torch tensors on the GPU; this module only checks shapes and passes pointers.
"""
import ctypes

import torch
from torch.autograd.graph import increment_version

from . import _lib
from ._lib import AdamHP, NetDesc, check


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need(t, name, numel, dtype=torch.float32):
    if t is None:
        raise ValueError(f"{name} is required")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device})")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} has {t.numel()} elements, expected {numel}")


def _wrote(*tensors):
    """Bump the version counters of tensors the library wrote in place (no
    torch op saw the write), so that a resident inner-loop state keyed to
    them is not taken up after it (InnerLoopPlan.inner_loop(keep=True)).
    Every method that hands a workspace to the library marks it written (the
    library also drops its resident state in every entry point but the loop's
    own)."""
    for t in tensors:
        if t is not None:
            increment_version(t)


def make_adam(lr, step, kind="higher", betas=(0.9, 0.999), eps=1e-8):
    k = {"higher": _lib.ADAM_HIGHER, "hypergrad": _lib.ADAM_HYPERGRAD,
         "torch": _lib.ADAM_TORCH}[kind]
    return AdamHP(float(lr), float(betas[0]), float(betas[1]), float(eps), int(step), k)


class _Token:
    """What a KEEP inner loop left resident: compared by tensor identity,
    version counters, seed and the continuing Philox offset."""

    __slots__ = ("tensors", "versions", "seed", "offset")

    def __init__(self, tensors, versions, seed, offset):
        self.tensors, self.versions, self.seed, self.offset = tensors, versions, seed, offset

    def __eq__(self, o):
        return (all(a is b for a, b in zip(self.tensors, o.tensors)) and self.versions == o.versions
                and self.seed == o.seed and self.offset == o.offset)


class InnerLoopPlan:
    """family: 'meanfield' (VILinear stack) or 'fullcov' (VILinearMultivariateNormal
    stack); layers: [(in, out), ...]; S: global MC samples; M: pseudopoints."""

    def __init__(self, family, layers, S, M, prior_sd=1.0, world=1, rank=0):
        self.lib = _lib.load()
        self._resident = None  # inner_loop(keep=True)'s token
        self.family = family
        fam = {"meanfield": _lib.FAMILY_MEANFIELD, "fullcov": _lib.FAMILY_FULLCOV,
               "lenet": _lib.FAMILY_LENET}[family]
        layers = [tuple(int(x) for x in l) for l in layers]
        if family == "lenet":
            # fixed make_lenet stack (conv "in" = in_channels * 25); input 1x28x28
            if layers != [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]:
                raise ValueError(f"not make_lenet's layer table: {layers}")
            self.in_features = 784
        else:
            for a, b in zip(layers[:-1], layers[1:]):
                if a[1] != b[0]:
                    raise ValueError(f"layer sizes do not chain: {layers}")
            self.in_features = layers[0][0]
        if not 1 <= len(layers) <= _lib.MAX_LAYERS:
            raise ValueError("1..8 layers supported")
        self.layers = layers
        self.S, self.M, self.world, self.rank = int(S), int(M), int(world), int(rank)
        d = NetDesc()
        d.n_layers = len(layers)
        dims = [layers[0][0]] + [o for _, o in layers]
        for i, v in enumerate(dims):
            d.dims[i] = v
        d.S, d.M, d.prior_sd = self.S, self.M, float(prior_sd)
        self.desc = d
        h = ctypes.c_void_p()
        check(self.lib.psvi_plan_create(fam, ctypes.byref(d), self.world, self.rank,
                                        ctypes.byref(h)), "psvi_plan_create")
        self.handle = h
        q = self._query
        self.param_count = q(_lib.Q_PARAM_COUNT)
        self.eps_count = q(_lib.Q_EPS_COUNT)
        self.ws_bytes = q(_lib.Q_WS_BYTES)
        self.s_local = q(_lib.Q_S_LOCAL)
        self.s_offset = q(_lib.Q_S_OFFSET)
        self.acc_count = q(_lib.Q_ACC_COUNT)
        self.rows_local = q(_lib.Q_ROWS_LOCAL)
        self.xshard_count = q(_lib.Q_XSHARD_COUNT)
        self.xrecv_count = q(_lib.Q_XRECV_COUNT)
        self.loop_ws_bytes = q(_lib.Q_LOOP_WS_BYTES)
        self.tiled_floats = q(_lib.Q_TILED_FLOATS)  # 0: no tiled state for this plan
        self.outer_ws_bytes = q(_lib.Q_OUTER_WS_BYTES)
        self.hvp_ws_bytes = q(_lib.Q_HVP_WS_BYTES)
        self.eval_ws_bytes = q(_lib.Q_EVAL_WS_BYTES)
        self.net_part_ok = bool(q(_lib.Q_NET_PART_OK))
        self.eps_stride = (self.eps_count + 3) // 4 * 4   # Philox offset per loop step
        self.n_tot = sum(i * o + o for i, o in layers)

    def _query(self, key):
        v = ctypes.c_int64()
        check(self.lib.psvi_plan_query(self.handle, key, ctypes.byref(v)), "psvi_plan_query")
        return v.value

    def shard_info(self, r):
        """Rank r's samples and rows: s_offset, s_count, rows (x-shard columns),
        row_lo / row_cnt per layer (row_lo -1 when the layer's rows are several
        runs) and runs = [(layer, first row, count, x-shard column)] in column
        order (psvi_plan_shard_runs)."""
        out = (ctypes.c_int64 * (3 + 2 * _lib.MAX_LAYERS))()
        check(self.lib.psvi_plan_shard_info(self.handle, r, out), "psvi_plan_shard_info")
        L = len(self.layers)
        n = ctypes.c_int32()
        check(self.lib.psvi_plan_shard_runs(self.handle, r, None, 0, ctypes.byref(n)),
              "psvi_plan_shard_runs")
        buf = (ctypes.c_int64 * max(4 * n.value, 1))()
        check(self.lib.psvi_plan_shard_runs(self.handle, r, buf, n.value, ctypes.byref(n)),
              "psvi_plan_shard_runs")
        runs = [tuple(int(buf[4 * i + k]) for k in range(4)) for i in range(n.value)]
        return dict(s_offset=out[0], s_count=out[1], rows=out[2],
                    row_lo=[out[3 + l] for l in range(L)],
                    row_cnt=[out[3 + _lib.MAX_LAYERS + l] for l in range(L)], runs=runs)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.psvi_plan_destroy(h)
            except Exception:
                pass
            self.handle = None

    # ----------------------------------------------------------- buffers
    def workspace(self, device="cuda"):
        return torch.empty(self.ws_bytes, dtype=torch.uint8, device=device)

    def _inputs(self, u, z, w, eps):
        _need(u, "u", self.M * self.in_features)
        _need(z, "z", self.M, torch.int32)
        _need(w, "w", self.M)
        _need(eps, "eps", self.eps_count)

    # --------------------------------------------------------- world == 1
    def inner_step(self, u, z, w, eps, params, adam_m, adam_v, step, lr, kind="higher",
                   elbo_out=None, ws=None):
        """One fused inner step (psvi_inner_step); params/m/v updated in place.
        Returns the (device, float64) negative ELBO at the incoming params."""
        self._inputs(u, z, w, eps)
        for t, n in ((params, "params"), (adam_m, "adam_m"), (adam_v, "adam_v")):
            _need(t, n, self.param_count)
        if elbo_out is None:
            elbo_out = torch.empty(1, dtype=torch.float64, device=params.device)
        _need(elbo_out, "elbo_out", 1, torch.float64)
        if ws is None:
            ws = self.workspace(params.device)
        hp = make_adam(lr, step, kind)
        check(self.lib.psvi_inner_step(self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(eps),
                                       _ptr(params), _ptr(adam_m), _ptr(adam_v),
                                       ctypes.byref(hp), _ptr(elbo_out), _ptr(ws),
                                       ws.numel(), _stream()), "psvi_inner_step")
        _wrote(params, adam_m, adam_v, ws)
        return elbo_out

    def inner_loop(self, u, z, w, params, adam_m, adam_v, T, lr, kind="higher", step0=1,
                   eps=None, seed=0, offset=0, elbo_out=None, ws=None, keep=False):
        """T chained inner steps (psvi_inner_loop).  eps: (T, eps_count) device
        tensor, or None for in-library Philox draws (seed, offset + t * eps_stride).
        Returns the (T,) float64 device tensor of negative ELBOs before each step.

        keep=True (Philox mode, full-cov plans with a tiled state): the loop's
        state stays in ws -- the tiled corr / m / v, the next step's draw and
        sample -- and the next call that continues this one takes it up
        instead of redoing the first steps' fixed work (psvi_inner_loop_ex
        KEEP / RESUME).  It continues when it passes the same ws, params,
        adam_m, adam_v tensors, unmodified since (version counters; this
        plan's own in-place writers bump them), the same seed and offset +
        T * eps_stride.  The resumed numbers are those of one call over all
        the steps, bit for bit, when the last call of the run has keep=False
        (a keep=True call's last step takes the fused update with the next
        sample, where a plain call's last step takes the packed-out one:
        the same values up to fp32 rounding)."""
        _need(u, "u", self.M * self.in_features)
        _need(z, "z", self.M, torch.int32)
        _need(w, "w", self.M)
        for t, n in ((params, "params"), (adam_m, "adam_m"), (adam_v, "adam_v")):
            _need(t, n, self.param_count)
        T = int(T)
        if eps is not None:
            _need(eps, "eps", T * self.eps_count)
        if elbo_out is None:
            elbo_out = torch.empty(max(T, 1), dtype=torch.float64, device=params.device)
        _need(elbo_out, "elbo_out", None, torch.float64)
        if elbo_out.numel() < T:
            raise ValueError("elbo_out holds fewer than T doubles")
        if ws is None or ws.numel() < self.loop_ws_bytes:
            ws = torch.empty(self.loop_ws_bytes, dtype=torch.uint8, device=params.device)
        hp = make_adam(lr, step0, kind)
        flags = 0
        tok, self._resident = self._resident, None
        if eps is None:
            if keep:
                flags |= _lib.LOOP_KEEP
            if tok is not None and tok == self._loop_token(ws, params, adam_m, adam_v, seed, offset):
                flags |= _lib.LOOP_RESUME
        else:
            keep = False
        check(self.lib.psvi_inner_loop_ex(self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(eps),
                                          int(seed) & (2**64 - 1), int(offset), T, _ptr(params),
                                          _ptr(adam_m), _ptr(adam_v), ctypes.byref(hp),
                                          _ptr(elbo_out), _ptr(ws), ws.numel(), flags, _stream()),
              "psvi_inner_loop_ex")
        _wrote(params, adam_m, adam_v, ws)
        if keep and T > 0:
            self._resident = self._loop_token(ws, params, adam_m, adam_v, seed,
                                              int(offset) + T * self.eps_stride)
        return elbo_out[:T]

    @staticmethod
    def _loop_token(ws, params, adam_m, adam_v, seed, offset):
        # the tensors themselves (held, so that no new tensor reuses the
        # addresses) and their version counters: any torch write in between
        # makes the next call start cold
        ts = (ws, params, adam_m, adam_v)
        return _Token(ts, tuple(t._version for t in ts), int(seed) & (2**64 - 1), int(offset))

    def elbo_grad(self, u, z, w, eps, params, include_kl=True, ws=None):
        self._inputs(u, z, w, eps)
        _need(params, "params", self.param_count)
        elbo = torch.empty(1, dtype=torch.float64, device=params.device)
        grad = torch.empty(self.param_count, dtype=torch.float32, device=params.device)
        if ws is None:
            ws = self.workspace(params.device)
        check(self.lib.psvi_elbo_grad(self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(eps),
                                      _ptr(params), int(bool(include_kl)), _ptr(elbo),
                                      _ptr(grad), _ptr(ws), ws.numel(), _stream()),
              "psvi_elbo_grad")
        _wrote(ws)
        return elbo, grad

    def outer_elbo_grad(self, n_pseudo, x_all, z_all, w_all, eps, params, grad=True,
                        grad_u=True, grad_w=True, sample_stats=False, ws=None):
        """Outer objective (PSVI.psvi_elbo) over this plan's M rows (pseudopoints
        first, n_pseudo of them) -- psvi_outer_elbo_grad.  Returns a dict of
        device tensors: loss (float64, 1), and as requested grad (P), grad_u
        (n_pseudo, D), grad_w (n_pseudo), samples (S, 4: pseudo, data, nkl,
        weight; float64)."""
        D = self.in_features
        n_pseudo = int(n_pseudo)
        _need(x_all, "x_all", self.M * D)
        _need(z_all, "z_all", self.M, torch.int32)
        _need(w_all, "w_all", self.M)
        _need(eps, "eps", self.eps_count)
        _need(params, "params", self.param_count)
        dev = params.device
        out = {"loss": torch.empty(1, dtype=torch.float64, device=dev)}
        if grad:
            out["grad"] = torch.empty(self.param_count, dtype=torch.float32, device=dev)
        if grad and grad_u:
            out["grad_u"] = torch.empty(n_pseudo, D, dtype=torch.float32, device=dev)
        if grad_w:
            out["grad_w"] = torch.empty(n_pseudo, dtype=torch.float32, device=dev)
        if sample_stats:
            out["samples"] = torch.empty(self.S, 4, dtype=torch.float64, device=dev)
        if ws is None or ws.numel() < self.outer_ws_bytes:
            ws = torch.empty(self.outer_ws_bytes, dtype=torch.uint8, device=dev)
        check(self.lib.psvi_outer_elbo_grad(
            self.handle, n_pseudo, _ptr(x_all), _ptr(z_all), _ptr(w_all), _ptr(eps),
            _ptr(params), _ptr(out["loss"]), _ptr(out.get("grad")), _ptr(out.get("grad_u")),
            _ptr(out.get("grad_w")), _ptr(out.get("samples")), _ptr(ws), ws.numel(),
            _stream()), "psvi_outer_elbo_grad")
        _wrote(ws)
        return out

    def outer_ablated_elbo_grad(self, x_all, z_all, w_all, eps, params, grad=True,
                                sample_stats=False, ws=None):
        """PSVI_Ablated.psvi_elbo over this plan's M data rows (no pseudopoints):
        mean_s data_s - mean_s nkl_s -- psvi_outer_ablated_elbo_grad.  Returns
        a dict: loss (float64, 1), grad (P) when requested, samples (S, 4)."""
        D = self.in_features
        _need(x_all, "x_all", self.M * D)
        _need(z_all, "z_all", self.M, torch.int32)
        _need(w_all, "w_all", self.M)
        _need(eps, "eps", self.eps_count)
        _need(params, "params", self.param_count)
        dev = params.device
        out = {"loss": torch.empty(1, dtype=torch.float64, device=dev)}
        if grad:
            out["grad"] = torch.empty(self.param_count, dtype=torch.float32, device=dev)
        if sample_stats:
            out["samples"] = torch.empty(self.S, 4, dtype=torch.float64, device=dev)
        if ws is None or ws.numel() < self.outer_ws_bytes:
            ws = torch.empty(self.outer_ws_bytes, dtype=torch.uint8, device=dev)
        check(self.lib.psvi_outer_ablated_elbo_grad(
            self.handle, _ptr(x_all), _ptr(z_all), _ptr(w_all), _ptr(eps), _ptr(params),
            _ptr(out["loss"]), _ptr(out.get("grad")), _ptr(out.get("samples")), _ptr(ws),
            ws.numel(), _stream()), "psvi_outer_ablated_elbo_grad")
        _wrote(ws)
        return out

    def outer_grad_coef(self, n_pseudo, x_all, z_all, w_all, eps, params, coef, grad_u=True,
                        grad_w=True, ws=None):
        """Backward of the outer objective with caller-given per-sample
        coefficients coef = [rowcoef (S, 2) | ck (S) | sck] (float32, 3S + 1)
        -- psvi_outer_elbo_grad_coef, the second pass of the sample-sharded
        outer objective (sharded.ShardedOuter).  Returns grad (P), grad_u
        (n_pseudo, D) and grad_w (n_pseudo) as requested."""
        D = self.in_features
        n_pseudo = int(n_pseudo)
        _need(x_all, "x_all", self.M * D)
        _need(z_all, "z_all", self.M, torch.int32)
        _need(w_all, "w_all", self.M)
        _need(eps, "eps", self.eps_count)
        _need(params, "params", self.param_count)
        _need(coef, "coef", 3 * self.S + 1)
        dev = params.device
        out = {"grad": torch.empty(self.param_count, dtype=torch.float32, device=dev)}
        if grad_u:
            out["grad_u"] = torch.empty(n_pseudo, D, dtype=torch.float32, device=dev)
        if grad_w:
            out["grad_w"] = torch.empty(n_pseudo, dtype=torch.float32, device=dev)
        if ws is None or ws.numel() < self.outer_ws_bytes:
            ws = torch.empty(self.outer_ws_bytes, dtype=torch.uint8, device=dev)
        check(self.lib.psvi_outer_elbo_grad_coef(
            self.handle, n_pseudo, _ptr(x_all), _ptr(z_all), _ptr(w_all), _ptr(eps),
            _ptr(params), _ptr(coef), _ptr(out["grad"]), _ptr(out.get("grad_u")),
            _ptr(out.get("grad_w")), _ptr(ws), ws.numel(), _stream()),
            "psvi_outer_elbo_grad_coef")
        _wrote(ws)
        return out

    def evaluate(self, n_pseudo, x_all, z_all, w_all, eps, params, correction=True, probs=False,
                 ws=None):
        """Importance-weighted predictive evaluation of the data rows of this
        plan's M rows (psvi_evaluate).  Returns (stats, probs): stats a float64
        device tensor [entropy of W, normalised ESS, correct, summed NLL];
        probs ([M - n_pseudo, C]) when requested."""
        D, C = self.in_features, self.layers[-1][1]
        _need(x_all, "x_all", self.M * D)
        _need(z_all, "z_all", self.M, torch.int32)
        _need(w_all, "w_all", self.M)
        _need(eps, "eps", self.eps_count)
        _need(params, "params", self.param_count)
        dev = params.device
        stats = torch.empty(4, dtype=torch.float64, device=dev)
        pr = torch.empty(self.M - int(n_pseudo), C, dtype=torch.float32, device=dev) if probs else None
        if ws is None or ws.numel() < self.eval_ws_bytes:
            ws = torch.empty(self.eval_ws_bytes, dtype=torch.uint8, device=dev)
        check(self.lib.psvi_evaluate(self.handle, int(n_pseudo), _ptr(x_all), _ptr(z_all),
                                     _ptr(w_all), _ptr(eps), _ptr(params), int(bool(correction)),
                                     _ptr(pr), _ptr(stats), _ptr(ws), ws.numel(), _stream()),
              "psvi_evaluate")
        _wrote(ws)
        return stats, pr

    def hvp(self, u, z, w, eps, params, vec, mixed=True, out=None, ws=None, include_kl=True):
        """Hessian-vector product of the negative inner ELBO at fixed eps
        (psvi_hvp).  Returns (hv, d_u, d_w): H vec and, with mixed=True, the
        mixed products d/du and d/dw of vec . grad (else None, None).
        include_kl=False: this plan's samples' share without the KL Hessian
        (psvi_hvp_partial, one rank of a sample-sharded product)."""
        self._inputs(u, z, w, eps)
        _need(params, "params", self.param_count)
        _need(vec, "vec", self.param_count)
        dev = params.device
        hv = torch.empty(self.param_count, dtype=torch.float32, device=dev) if out is None else out
        _need(hv, "hv_out", self.param_count)
        du = torch.empty(self.M, self.in_features, dtype=torch.float32, device=dev) if mixed else None
        dw = torch.empty(self.M, dtype=torch.float32, device=dev) if mixed else None
        if ws is None or ws.numel() < self.hvp_ws_bytes:
            ws = torch.empty(self.hvp_ws_bytes, dtype=torch.uint8, device=dev)
        check(self.lib.psvi_hvp_partial(self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(eps),
                                        _ptr(params), _ptr(vec), int(bool(include_kl)), _ptr(hv),
                                        _ptr(du), _ptr(dw), _ptr(ws), ws.numel(), _stream()),
              "psvi_hvp_partial")
        _wrote(ws)
        return hv, du, dw

    # ------------------------------------------------------------ phases
    def mf_accumulate(self, u, z, w, eps, params, acc, nll_out):
        """acc <- [sum_s dW | sum_s dW*eps] (this rank's samples); nll_out += NLL."""
        self._inputs(u, z, w, eps)
        _need(params, "params", self.param_count)
        _need(acc, "acc", self.acc_count)
        _need(nll_out, "nll_out", 1, torch.float64)
        check(self.lib.psvi_mf_phase_accumulate(self.handle, _ptr(u), _ptr(z), _ptr(w),
                                                _ptr(eps), _ptr(params), _ptr(acc),
                                                _ptr(nll_out), _stream()),
              "psvi_mf_phase_accumulate")

    def mf_update(self, acc, params, adam_m=None, adam_v=None, step=1, lr=1e-3,
                  kind="higher", kl_out=None, grad_out=None, include_kl=True):
        _need(acc, "acc", self.acc_count)
        _need(params, "params", self.param_count)
        if kl_out is not None:
            _need(kl_out, "kl_out", 1, torch.float64)
        hp = make_adam(lr, step, kind)
        check(self.lib.psvi_mf_phase_update(self.handle, _ptr(acc), _ptr(params), _ptr(adam_m),
                                            _ptr(adam_v), ctypes.byref(hp), _ptr(kl_out),
                                            _ptr(grad_out), int(bool(include_kl)), _stream()),
              "psvi_mf_phase_update")
        _wrote(params, adam_m, adam_v)

    def mvn_sample(self, eps, params, x_shard):
        _need(eps, "eps", self.eps_count)
        _need(params, "params", self.param_count)
        _need(x_shard, "x_shard", self.xshard_count)
        check(self.lib.psvi_mvn_phase_sample(self.handle, _ptr(eps), _ptr(params),
                                             _ptr(x_shard), _stream()), "psvi_mvn_phase_sample")

    def tiled_state(self, device="cuda"):
        if not self.tiled_floats:
            raise ValueError("this plan has no tiled state (full-cov, world 1, S <= 128)")
        return torch.empty(self.tiled_floats, dtype=torch.float32, device=device)

    def tiled_convert(self, params, adam_m, adam_v, tstate, to_tiled):
        for t, n in ((params, "params"), (adam_m, "adam_m"), (adam_v, "adam_v")):
            _need(t, n, self.param_count)
        _need(tstate, "tstate", self.tiled_floats)
        check(self.lib.psvi_mvn_tiled_convert(self.handle, _ptr(params), _ptr(adam_m),
                                              _ptr(adam_v), _ptr(tstate), int(bool(to_tiled)),
                                              _stream()), "psvi_mvn_tiled_convert")
        _wrote(params, adam_m, adam_v, tstate)

    def mvn_update_tiled(self, eps, g_shard, params, adam_m, adam_v, tstate, step, lr,
                         kind="higher", kl_out=None, include_kl=True, eps_next=None,
                         x_next=None):
        _need(eps, "eps", self.eps_count)
        _need(g_shard, "g_shard", self.xshard_count)
        for t, n in ((params, "params"), (adam_m, "adam_m"), (adam_v, "adam_v")):
            _need(t, n, self.param_count)
        _need(tstate, "tstate", self.tiled_floats)
        if kl_out is not None:
            _need(kl_out, "kl_out", 1, torch.float64)
        if (eps_next is None) != (x_next is None):
            raise ValueError("eps_next and x_next go together")
        if eps_next is not None:
            _need(eps_next, "eps_next", self.eps_count)
            _need(x_next, "x_next", self.xshard_count)
        hp = make_adam(lr, step, kind)
        check(self.lib.psvi_mvn_phase_update_tiled(
            self.handle, _ptr(eps), _ptr(g_shard), _ptr(params), _ptr(adam_m), _ptr(adam_v),
            _ptr(tstate), ctypes.byref(hp), _ptr(kl_out), int(bool(include_kl)), _ptr(eps_next),
            _ptr(x_next), _stream()), "psvi_mvn_phase_update_tiled")
        _wrote(params, adam_m, adam_v, tstate)

    def mvn_net(self, u, z, w, x_recv, g_send, nll_out, draw=None, samples=None, draw_part=(0, 1)):
        """draw = (eps_out, seed, offset): the next step's global eps drawn in the
        same launch (psvi_mvn_phase_net_draw; psvi_randn's values).  samples =
        (s_begin, s_count): only those local samples (psvi_mvn_phase_net_part),
        with part draw_part[0] of draw_part[1] of the draw."""
        _need(u, "u", self.M * self.in_features)
        _need(z, "z", self.M, torch.int32)
        _need(w, "w", self.M)
        _need(x_recv, "x_recv", self.xrecv_count)
        _need(g_send, "g_send", self.xrecv_count)
        _need(nll_out, "nll_out", 1, torch.float64)
        if samples is not None:
            out, seed, offset = draw if draw is not None else (None, 0, 0)
            n = 0 if out is None else out.numel()
            check(self.lib.psvi_mvn_phase_net_part(
                self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(x_recv), _ptr(g_send), _ptr(nll_out),
                int(samples[0]), int(samples[1]), _ptr(out), n, int(seed), int(offset),
                int(draw_part[0]), int(draw_part[1]), _stream()), "psvi_mvn_phase_net_part")
            return
        if draw is None:
            check(self.lib.psvi_mvn_phase_net(self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(x_recv),
                                              _ptr(g_send), _ptr(nll_out), _stream()),
                  "psvi_mvn_phase_net")
            return
        out, seed, offset = draw
        _need(out, "eps_out", out.numel())
        check(self.lib.psvi_mvn_phase_net_draw(self.handle, _ptr(u), _ptr(z), _ptr(w), _ptr(x_recv),
                                               _ptr(g_send), _ptr(nll_out), _ptr(out), out.numel(),
                                               int(seed), int(offset), _stream()),
              "psvi_mvn_phase_net_draw")

    def mvn_update(self, eps, g_shard, params, adam_m=None, adam_v=None, step=1, lr=1e-3,
                   kind="higher", kl_out=None, grad_out=None, include_kl=True, eps_next=None,
                   x_next=None):
        """Full-cov update phase; with eps_next / x_next also the next step's
        sample from the updated parameters (psvi_mvn_phase_update_sample)."""
        _need(eps, "eps", self.eps_count)
        _need(g_shard, "g_shard", self.xshard_count)
        _need(params, "params", self.param_count)
        if kl_out is not None:
            _need(kl_out, "kl_out", 1, torch.float64)
        hp = make_adam(lr, step, kind)
        if eps_next is not None or x_next is not None:
            if grad_out is not None:
                raise ValueError("the fused next-step sample runs with the Adam update only")
            _need(eps_next, "eps_next", self.eps_count)
            _need(x_next, "x_next", self.xshard_count)
            check(self.lib.psvi_mvn_phase_update_sample(
                self.handle, _ptr(eps), _ptr(g_shard), _ptr(params), _ptr(adam_m), _ptr(adam_v),
                ctypes.byref(hp), _ptr(kl_out), int(bool(include_kl)), _ptr(eps_next),
                _ptr(x_next), _stream()), "psvi_mvn_phase_update_sample")
            _wrote(params, adam_m, adam_v)
            return
        check(self.lib.psvi_mvn_phase_update(self.handle, _ptr(eps), _ptr(g_shard),
                                             _ptr(params), _ptr(adam_m), _ptr(adam_v),
                                             ctypes.byref(hp), _ptr(kl_out), _ptr(grad_out),
                                             int(bool(include_kl)), _stream()),
              "psvi_mvn_phase_update")
        _wrote(params, adam_m, adam_v)


def randn_(out, seed, offset=0):
    """Fill a float32 device tensor with N(0,1) (Philox4x32-10 + Box-Muller)."""
    _need(out, "out", None)
    lib = _lib.load()
    check(lib.psvi_randn(_ptr(out), out.numel(), int(seed) & (2**64 - 1),
                         int(offset), _stream()), "psvi_randn")
    return out


def nonfinite_(flag, *tensors):
    """flag (device int32, 1 element) |= 1 if any value of the float32 /
    float64 device tensors is NaN or +-inf (psvi_nonfinite; no host sync)."""
    _need(flag, "flag", 1, torch.int32)
    lib = _lib.load()
    for t in tensors:
        if t is None:
            continue
        if t.dtype not in (torch.float32, torch.float64) or not t.is_cuda or not t.is_contiguous():
            raise ValueError("nonfinite_: contiguous float32 / float64 device tensors")
        check(lib.psvi_nonfinite(_ptr(t), t.numel(), int(t.dtype == torch.float64), _ptr(flag),
                                 _stream()), "psvi_nonfinite")
    return flag


def adam_adjoint_(lt, lm, lv, adam_m, adam_v, grad, step, lr, lg_out, kind="higher",
                  betas=(0.9, 0.999), eps=1e-8):
    """Reverse of one Adam step (psvi_adam_adjoint): lm, lv updated in place,
    lg_out <- adjoint of the step's gradient."""
    n = lt.numel()
    for t, nm in ((lt, "lt"), (lm, "lm"), (lv, "lv"), (adam_m, "adam_m"), (adam_v, "adam_v"),
                  (grad, "grad"), (lg_out, "lg_out")):
        _need(t, nm, n)
    hp = make_adam(lr, step, kind, betas, eps)
    lib = _lib.load()
    check(lib.psvi_adam_adjoint(n, _ptr(lt), _ptr(lm), _ptr(lv), _ptr(adam_m), _ptr(adam_v),
                                _ptr(grad), _ptr(lg_out), ctypes.byref(hp), _stream()),
          "psvi_adam_adjoint")
    return lg_out


def adam_update_(params, grad, adam_m, adam_v, step, lr, kind="higher", betas=(0.9, 0.999),
                 eps=1e-8):
    n = params.numel()
    for t, nm in ((params, "params"), (grad, "grad"), (adam_m, "adam_m"), (adam_v, "adam_v")):
        _need(t, nm, n)
    hp = make_adam(lr, step, kind, betas, eps)
    lib = _lib.load()
    check(lib.psvi_adam_update(n, _ptr(params), _ptr(grad), _ptr(adam_m), _ptr(adam_v),
                               ctypes.byref(hp), _stream()), "psvi_adam_update")
