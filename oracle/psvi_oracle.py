"""CPU oracle for the coreset-ELBO inner step -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  The product path (the HIP library behind
blackbox-coresets-vi_amd/psvi) never calls into oracle/.

Float64 numpy restatement of the reference hot path, hand-derived backward
included.  Parity pinned by tests/golden/*.npz, generated from the reference
itself by tools/gen_golden.py (see tests/test_oracle_golden.py).

Reference anchors (paths relative to /root/reference):
  inner objective      psvi/inference/psvi_classes.py:488-511 (sum over S, w = N f(v))
  f(v)                 psvi_classes.py:1358-1360 (softmax), 1486-1488 (exp(a) softmax)
  mean-field layer     psvi/models/neural_net.py:60-179 (rsample 155-170, kl 101-108)
  full-cov layer       neural_net.py:408-491 (scale_tril 452-461, rsample 467-476, kl 435-436)
  higher Adam          psvi/robust_higher/optim.py:299-367
  hypergrad adam_step  psvi/hypergrad/diff_optimizers.py:184-213

Flat layouts (identical to torch.nn.utils.parameters_to_vector on the reference
modules, i.e. module registration order):
  mean-field layer (in, out): [mu_W (out*in), mu_b (out), rho_W (out*in), rho_b (out)]
  full-cov layer   (in, out): n = out*in + out; [mean (n), sd (n), corr ((n-1)(n-2)/2)]
Noise, per layer in forward order: mean-field eps_W (S,out,in) then eps_b (S,out);
full-cov eps (S, n).
"""
import numpy as np


# ---------------------------------------------------------------- helpers
def softplus(x):
    """torch.nn.functional.softplus(beta=1, threshold=20)."""
    x = np.asarray(x, dtype=np.float64)
    return np.where(x > 20.0, x, np.log1p(np.exp(np.minimum(x, 20.0))))


def sigmoid(x):
    x = np.asarray(x, dtype=np.float64)
    return 0.5 * (1.0 + np.tanh(0.5 * x))


def coreset_weights(v, N, f="softmax", alpha=None):
    """w = N * f(v): PSVI identity (psvi_classes.py:111), PSVILearnV softmax
    (1358-1360), PSVIAV exp(alpha)*softmax (1486-1488)."""
    v = np.asarray(v, dtype=np.float64)
    if f == "identity":
        return N * v
    e = np.exp(v - v.max())
    sm = e / e.sum()
    if f == "softmax":
        return N * sm
    if f == "exp_alpha_softmax":
        return N * np.exp(alpha) * sm
    raise ValueError(f)


def mf_sizes(layers):
    out = []
    for din, dout in layers:
        out.append(dict(nw=din * dout, nb=dout))
    return out


def mf_param_count(layers):
    return sum(2 * (i * o + o) for i, o in layers)


def mf_eps_count(layers, S):
    return sum(S * (i * o + o) for i, o in layers)


def mvn_n(din, dout):
    return din * dout + dout


def mvn_ncorr(n):
    return (n - 1) * (n - 2) // 2


def mvn_param_count(layers):
    return sum(2 * mvn_n(i, o) + mvn_ncorr(mvn_n(i, o)) for i, o in layers)


def mvn_eps_count(layers, S):
    return sum(S * mvn_n(i, o) for i, o in layers)


def tril_rows_cols(n):
    """Row-major strict-lower indices of the (n-1)x(n-1) block
    (torch.tril_indices(n-1, n-1, -1), neural_net.py:458-460)."""
    r, c = np.tril_indices(n - 1, -1)
    return r, c


# ------------------------------------------------------------ per-sample net
def net_forward_backward(u, z, w, Ws, bs):
    """Batched-over-S MLP forward + weighted NLL + hand-derived backward.

    u (M, D); z (M,) int; w (M,); Ws[l] (S, out, in); bs[l] (S, out).
    Returns (data_term, dWs, dbs) with data_term = sum_s sum_m w_m NLL_sm
    (psvi_classes.py:495-505,511) and dWs[l] = d data / d W_s (S, out, in).
    """
    S = Ws[0].shape[0]
    M = u.shape[0]
    L = len(Ws)
    hs = [np.broadcast_to(u[None], (S,) + u.shape)]
    acts = []
    for l in range(L):
        a = np.einsum("smi,soi->smo", hs[-1], Ws[l]) + bs[l][:, None, :]
        acts.append(a)
        hs.append(np.maximum(a, 0.0) if l < L - 1 else a)
    logits = hs[-1]
    mx = logits.max(-1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(-1, keepdims=True)))[..., 0]
    zi = z.astype(np.int64)
    picked = logits[:, np.arange(M), zi]
    nll = lse - picked
    data = float((nll * w[None]).sum())
    p = np.exp(logits - lse[..., None])
    p[:, np.arange(M), zi] -= 1.0
    g = p * w[None, :, None]
    dWs = [None] * L
    dbs = [None] * L
    for l in range(L - 1, -1, -1):
        dWs[l] = np.einsum("smo,smi->soi", g, hs[l])
        dbs[l] = g.sum(1)
        if l > 0:
            g = np.einsum("smo,soi->smi", g, Ws[l]) * (acts[l - 1] > 0)
    return data, dWs, dbs


def relu_margin(u, Ws, bs):
    """Per-sample min over hidden pre-activations of |a| / (sum_i |h_i W_ji| + |b_j|):
    how far each sample sits from a ReLU kink in units of its own fp32 rounding
    scale.  Samples with a margin below ~1e-5 can legitimately flip a mask
    between an fp32 and an fp64 evaluation."""
    S = Ws[0].shape[0]
    h = np.broadcast_to(u[None], (S,) + u.shape)
    marg = np.full(S, np.inf)
    for l in range(len(Ws) - 1):
        a = np.einsum("smi,soi->smo", h, Ws[l]) + bs[l][:, None, :]
        scale = np.einsum("smi,soi->smo", np.abs(h), np.abs(Ws[l])) + np.abs(bs[l])[:, None, :]
        marg = np.minimum(marg, (np.abs(a) / np.maximum(scale, 1e-300)).reshape(S, -1).min(1))
        h = np.maximum(a, 0.0)
    return marg


def mvn_split_x(layers, X):
    """(S, n_tot) per-sample weight vectors -> per-layer W_s, b_s."""
    Ws, bs, col = [], [], 0
    S = X.shape[0]
    for din, dout in layers:
        n = din * dout + dout
        Ws.append(X[:, col:col + din * dout].reshape(S, dout, din))
        bs.append(X[:, col + din * dout:col + n])
        col += n
    return Ws, bs


def mvn_grad_from_G(layers, params, G, eps, S, prior_sd=1.0):
    """Update-phase restatement: gradient of the full-cov parameters from the
    per-sample weight gradients G (S, n_tot)."""
    params = np.asarray(params, np.float64)
    eps = np.asarray(eps, np.float64)
    G = np.asarray(G, np.float64)
    s0 = float(prior_sd)
    grad = np.zeros_like(params)
    po = eo = col = 0
    for din, dout in layers:
        n = mvn_n(din, dout)
        nc = mvn_ncorr(n)
        mean, sd, corr = params[po:po + n], params[po + n:po + 2 * n], params[po + 2 * n:po + 2 * n + nc]
        E = eps[eo:eo + S * n].reshape(S, n)
        Gl = G[:, col:col + n]
        spd = softplus(sd)
        grad[po:po + n] = Gl.sum(0) + mean / s0 ** 2
        grad[po + n:po + 2 * n] = ((Gl * E).sum(0) + spd / s0 ** 2 - 1.0 / spd) * sigmoid(sd)
        r, c = tril_rows_cols(n)
        grad[po + 2 * n:po + 2 * n + nc] = (Gl.T @ E)[r, c] + corr / s0 ** 2
        po += 2 * n + nc
        eo += S * n
        col += n
    return grad


# --------------------------------------------------------------- Adam steps
def adam_higher(p, g, m, v, t, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """robust_higher DifferentiableAdam._update (optim.py:318-367), t 1-based."""
    m = beta1 * m + (1.0 - beta1) * g
    v = beta2 * v + (1.0 - beta2) * g * g
    bc1 = 1.0 - beta1 ** t
    bc2 = 1.0 - beta2 ** t
    denom = np.sqrt(v + 1e-8) / np.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def adam_hypergrad(p, g, m, v, t, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """hypergrad adam_step (diff_optimizers.py:184-213): v stores +1e-12."""
    m = beta1 * m + (1.0 - beta1) * g
    v = beta2 * v + (1.0 - beta2) * g * g + 1e-12
    p = p - lr * (m / (1.0 - beta1 ** t)) / (np.sqrt(v / (1.0 - beta2 ** t)) + eps)
    return p, m, v


def adam(kind, *a, **k):
    return (adam_higher if kind == "higher" else adam_hypergrad)(*a, **k)


# ------------------------------------------------------------ mean-field MLP
def mf_elbo_grad(layers, params, u, z, w, eps, S, prior_sd=1.0):
    """Negative inner ELBO and its gradient for a VILinear stack
    (make_fcnet / logistic_regression)."""
    params = np.asarray(params, dtype=np.float64)
    eps = np.asarray(eps, dtype=np.float64)
    Ws, bs, sW, sb, eW, eb, views = [], [], [], [], [], [], []
    po = 0
    eo = 0
    kl = 0.0
    s0 = float(prior_sd)
    for din, dout in layers:
        nw, nb = din * dout, dout
        muW = params[po:po + nw].reshape(dout, din)
        mub = params[po + nw:po + nw + nb]
        rW = params[po + nw + nb:po + 2 * nw + nb].reshape(dout, din)
        rb = params[po + 2 * nw + nb:po + 2 * nw + 2 * nb]
        views.append((po, nw, nb, muW, mub, rW, rb))
        po += 2 * (nw + nb)
        e_w = eps[eo:eo + S * nw].reshape(S, dout, din)
        eo += S * nw
        e_b = eps[eo:eo + S * nb].reshape(S, dout)
        eo += S * nb
        sdW, sdb = softplus(rW), softplus(rb)
        Ws.append(muW[None] + sdW[None] * e_w)
        bs.append(mub[None] + sdb[None] * e_b)
        eW.append(e_w)
        eb.append(e_b)
        sW.append(sdW)
        sb.append(sdb)
        for mu, sd in ((muW, sdW), (mub, sdb)):
            vr = (sd / s0) ** 2
            kl += float((0.5 * (vr + (mu / s0) ** 2 - 1.0 - np.log(vr))).sum())
    data, dWs, dbs = net_forward_backward(np.asarray(u, np.float64), np.asarray(z),
                                          np.asarray(w, np.float64), Ws, bs)
    grad = np.zeros_like(params)
    for l, (po, nw, nb, muW, mub, rW, rb) in enumerate(views):
        gW = dWs[l].sum(0) + muW / s0 ** 2
        gb = dbs[l].sum(0) + mub / s0 ** 2
        grW = ((dWs[l] * eW[l]).sum(0) + sW[l] / s0 ** 2 - 1.0 / sW[l]) * sigmoid(rW)
        grb = ((dbs[l] * eb[l]).sum(0) + sb[l] / s0 ** 2 - 1.0 / sb[l]) * sigmoid(rb)
        grad[po:po + nw] = gW.reshape(-1)
        grad[po + nw:po + nw + nb] = gb
        grad[po + nw + nb:po + 2 * nw + nb] = grW.reshape(-1)
        grad[po + 2 * nw + nb:po + 2 * (nw + nb)] = grb
    return data + kl, grad


# ------------------------------------------------------------- full-cov MLP
def mvn_dense_L(sd, corr, n):
    L = np.zeros((n, n))
    L[np.arange(n), np.arange(n)] = softplus(sd)
    r, c = tril_rows_cols(n)
    L[r, c] = corr
    return L


def mvn_elbo_grad(layers, params, u, z, w, eps, S, prior_sd=1.0):
    """Negative inner ELBO and gradient for a VILinearMultivariateNormal stack
    (make_fc2net / logistic_regression_fullcov)."""
    params = np.asarray(params, dtype=np.float64)
    eps = np.asarray(eps, dtype=np.float64)
    s0 = float(prior_sd)
    Ws, bs, Es, views = [], [], [], []
    po = eo = 0
    kl = 0.0
    for din, dout in layers:
        n = mvn_n(din, dout)
        nc = mvn_ncorr(n)
        mean = params[po:po + n]
        sd = params[po + n:po + 2 * n]
        corr = params[po + 2 * n:po + 2 * n + nc]
        views.append((po, n, nc, mean, sd, corr))
        po += 2 * n + nc
        E = eps[eo:eo + S * n].reshape(S, n)
        eo += S * n
        L = mvn_dense_L(sd, corr, n)
        X = mean[None] + E @ L.T
        Ws.append(X[:, :din * dout].reshape(S, dout, din))
        bs.append(X[:, din * dout:])
        Es.append(E)
        spd = softplus(sd)
        kl += (n * np.log(s0) - np.log(spd).sum()
               + 0.5 * ((spd ** 2).sum() / s0 ** 2 + (corr ** 2).sum() / s0 ** 2
                        + (mean ** 2).sum() / s0 ** 2 - n))
    data, dWs, dbs = net_forward_backward(np.asarray(u, np.float64), np.asarray(z),
                                          np.asarray(w, np.float64), Ws, bs)
    grad = np.zeros_like(params)
    for l, (po, n, nc, mean, sd, corr) in enumerate(views):
        G = np.concatenate([dWs[l].reshape(S, -1), dbs[l]], axis=1)  # (S, n)
        E = Es[l]
        spd = softplus(sd)
        grad[po:po + n] = G.sum(0) + mean / s0 ** 2
        dsd = (G * E).sum(0)
        grad[po + n:po + 2 * n] = (dsd + spd / s0 ** 2 - 1.0 / spd) * sigmoid(sd)
        r, c = tril_rows_cols(n)
        dL = G.T @ E
        grad[po + 2 * n:po + 2 * n + nc] = dL[r, c] + corr / s0 ** 2
    return data + kl, grad


# --------------------------------------------------------------- trajectory
def run_inner_loop(family, layers, params0, u, z, w, eps_steps, S, lr, adam_kind,
                   prior_sd=1.0, t0=1):
    """T inner steps (one per eps_steps row): returns (elbos, grads, params, m, v).
    nested trainer: fresh higher-Adam state at t=1 (psvi_classes.py:549-555);
    hyper trainer: hypergrad step_cnt from 1 (psvi_classes.py:622-647)."""
    f = {"mf": mf_elbo_grad, "mvn": mvn_elbo_grad,
         "lenet": lambda _l, p, u, z, w, e, S, sd: lenet_elbo_grad(p, u, z, w, e, S, sd)}[family]
    p = np.asarray(params0, dtype=np.float64).copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    elbos, grads, traj = [], [], []
    for k, e in enumerate(eps_steps):
        val, g = f(layers, p, u, z, w, e, S, prior_sd)
        elbos.append(val)
        grads.append(g)
        p, m, v = adam(adam_kind, p, g, m, v, t0 + k, lr)
        traj.append(p.copy())
    return np.array(elbos), grads, traj, m, v


# ------------------------------------------------- outer objective (psvi_elbo)
def _net_rows_forward(X, Ws, bs):
    """Per-sample MLP forward over rows X (R, D): returns (nll-ready logits,
    the layer inputs hs[l] (S, R, in_l) and pre-activations acts[l])."""
    S = Ws[0].shape[0]
    L = len(Ws)
    hs = [np.broadcast_to(X[None], (S,) + X.shape)]
    acts = []
    for l in range(L):
        a = np.einsum("smi,soi->smo", hs[-1], Ws[l]) + bs[l][:, None, :]
        acts.append(a)
        hs.append(np.maximum(a, 0.0) if l < L - 1 else a)
    return hs, acts


def _net_rows_backward(coef, probs_minus_onehot, hs, acts, Ws):
    """Backward of sum_{s,r} coef[s,r] NLL_sr: per-sample dW, db and the input
    gradient dX (S, R, D)."""
    L = len(Ws)
    g = probs_minus_onehot * coef[..., None]
    dWs, dbs = [None] * L, [None] * L
    for l in range(L - 1, -1, -1):
        dWs[l] = np.einsum("smo,smi->soi", g, hs[l])
        dbs[l] = g.sum(1)
        g = np.einsum("smo,soi->smi", g, Ws[l])
        if l > 0:
            g = g * (acts[l - 1] > 0)
    return dWs, dbs, g


def outer_elbo_grad(family, layers, params, X, z, w, n_pseudo, eps, S, prior_sd=1.0,
                    mode="iw"):
    if family == "lenet":
        X = np.asarray(X)
        loss, g, gu, gw = lenet_outer_elbo_grad(params, X.reshape(-1, 1, 28, 28), z, w,
                                                n_pseudo, eps, S, prior_sd, mode)
        return loss, g, gu.reshape((int(n_pseudo),) + X.shape[1:]), gw
    """Negative PSVI-ELBO (PSVI.psvi_elbo, psvi/inference/psvi_classes.py:445-486)
    and its first-order gradient.

    X (R, D) = cat(u, xbatch) with the first n_pseudo rows the pseudopoints;
    z (R,) class ids; w (R,) row weights: N f(v)_m for the pseudopoints
    (``.matmul(self.N * self.f(self.v, 0))``, 478-480) and N / Nx for the data
    rows (``self.N / Nx * all_nlls[:, Nu:].sum(-1)``, 481); eps the reference
    draw order of ``model(all_data)``.
      pseudo_s = sum_{m<Mu} w_m NLL_sm,  data_s = sum_{m>=Mu} w_m NLL_sm
      nkl_s    = log p(w_s) - log q(w_s)       (sampled_nkl, neural_net.py:110-115
                                                mean-field, 438-442 full-cov)
               = sum_i [-x_si^2/(2 s0^2) - log s0 + eps_si^2/2 + log sigma_i]
      (x_s = mean + L eps_s, so L^-1 (x_s - mean) = eps_s; sigma_i = softplus(sd_i),
       the diagonal of L, or the mean-field scales)
      lw_s = -pseudo_s + nkl_s,  W = softmax_s(lw)
      loss = sum_s W_s (data_s - pseudo_s) - mean_s lw_s
    Returns (loss, d loss/d params, d loss/d X[:n_pseudo], d loss/d w[:n_pseudo]).
    The pathwise gradient of nkl_s is -x_s/s0^2 on the sampled weights; the
    explicit one is +1/sigma_i on every scale (the eps^2/2 term is constant).
    mode="ablated": PSVI_Ablated.psvi_elbo (psvi_classes.py:1397-1408),
      loss = mean_s data_s - mean_s nkl_s  (no pseudo rows: n_pseudo = 0), with
      nkl over the VILinear layers only -- a full-covariance model has none, and
      the reference fails there (sum() of nothing is the int 0, 0.mean())."""
    if mode == "ablated" and family != "mf":
        raise AttributeError("'int' object has no attribute 'mean' (PSVI_Ablated.psvi_elbo "
                             "on a model without VILinear layers)")
    params = np.asarray(params, np.float64)
    eps = np.asarray(eps, np.float64)
    X = np.asarray(X, np.float64)
    w = np.asarray(w, np.float64)
    s0 = float(prior_sd)
    Ws, bs, lay = [], [], []
    po = eo = 0
    sumlog = 0.0
    xsq = np.zeros(S)
    esq = np.zeros(S)
    for din, dout in layers:
        n = din * dout + dout
        if family == "mf":
            mu = params[po:po + n]
            rho = params[po + n:po + 2 * n]
            E = np.concatenate([eps[eo:eo + S * din * dout].reshape(S, din * dout),
                                eps[eo + S * din * dout:eo + S * n].reshape(S, dout)], axis=1)
            sd = softplus(rho)
            Xs = mu[None] + sd[None] * E
            lay.append((po, n, E, rho, sd, None))
            po += 2 * n
        else:
            nc = mvn_ncorr(n)
            mean = params[po:po + n]
            sdr = params[po + n:po + 2 * n]
            corr = params[po + 2 * n:po + 2 * n + nc]
            E = eps[eo:eo + S * n].reshape(S, n)
            Lm = mvn_dense_L(sdr, corr, n)
            Xs = mean[None] + E @ Lm.T
            sd = softplus(sdr)
            lay.append((po, n, E, sdr, sd, nc))
            po += 2 * n + nc
        eo += S * n
        sumlog += float(np.log(sd).sum())
        xsq += (Xs ** 2).sum(1)
        esq += (E ** 2).sum(1)
        Ws.append(Xs[:, :din * dout].reshape(S, dout, din))
        bs.append(Xs[:, din * dout:])
    n_tot = sum(i * o + o for i, o in layers)
    hs, acts = _net_rows_forward(X, Ws, bs)
    logits = hs[-1]
    R = X.shape[0]
    mx = logits.max(-1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(-1, keepdims=True)))[..., 0]
    zi = np.asarray(z).astype(np.int64)
    nll = lse - logits[:, np.arange(R), zi]  # (S, R)
    Mu = int(n_pseudo)
    pseudo = nll[:, :Mu] @ w[:Mu]
    data = nll[:, Mu:] @ w[Mu:]
    nkl = -xsq / (2 * s0 ** 2) - n_tot * np.log(s0) + 0.5 * esq + sumlog
    loss, cp, cd, ck = _outer_coef(pseudo, data, nkl, S, mode)
    coef = np.concatenate([cp[:, None] * w[None, :Mu], cd[:, None] * w[None, Mu:]], axis=1)
    pmo = np.exp(logits - lse[..., None])
    pmo[:, np.arange(R), zi] -= 1.0
    dWs, dbs, dX = _net_rows_backward(coef, pmo, hs, acts, Ws)
    grad = np.zeros_like(params)
    sck = float(ck.sum())
    for l, (po, n, E, sdr, sd, nc) in enumerate(lay):
        din, dout = layers[l]
        Xs = np.concatenate([Ws[l].reshape(S, -1), bs[l]], axis=1)
        G = np.concatenate([dWs[l].reshape(S, -1), dbs[l]], axis=1) - ck[:, None] * Xs / s0 ** 2
        grad[po:po + n] = G.sum(0)
        grad[po + n:po + 2 * n] = ((G * E).sum(0) + sck / sd) * sigmoid(sdr)
        if family != "mf":
            r, c = tril_rows_cols(n)
            grad[po + 2 * n:po + 2 * n + nc] = (G.T @ E)[r, c]
    gX = dX.sum(0)[:Mu]
    gw = (cp[:, None] * nll[:, :Mu]).sum(0)
    return loss, grad, gX, gw


def _outer_coef(pseudo, data, nkl, S, mode):
    """loss and its derivatives w.r.t. each sample's pseudo, data and nkl terms.
    iw (PSVI.psvi_elbo, psvi_classes.py:476-486): lw = -pseudo + nkl,
    W = softmax_s(lw), loss = sum_s W_s (data_s - pseudo_s) - mean_s lw_s.
    ablated (PSVI_Ablated.psvi_elbo, 1397-1408): loss = mean data - mean nkl."""
    if mode == "ablated":
        loss = float(data.mean() - nkl.mean())
        return loss, np.zeros(S), np.full(S, 1.0 / S), np.full(S, -1.0 / S)
    if mode != "iw":
        raise ValueError(mode)
    lw = -pseudo + nkl
    W = np.exp(lw - lw.max())
    W /= W.sum()
    a = data - pseudo
    abar = float((W * a).sum())
    loss = abar - float(lw.mean())
    ck = W * (a - abar) - 1.0 / S          # d loss / d lw_s = d loss / d nkl_s
    return loss, -W - ck, W, ck            # cp = d loss / d pseudo_s, cd = d / d data_s


# ------------------------------------- second order: HVP of the inner ELBO
def _sample(family, layers, params, eps, S):
    """Per-layer sampled weights and reparameterisation pieces."""
    out = []
    po = eo = 0
    for din, dout in layers:
        n = din * dout + dout
        if family == "mf":
            mu, rho = params[po:po + n], params[po + n:po + 2 * n]
            E = np.concatenate([eps[eo:eo + S * din * dout].reshape(S, din * dout),
                                eps[eo + S * din * dout:eo + S * n].reshape(S, dout)], axis=1)
            X = mu[None] + softplus(rho)[None] * E
            out.append(dict(po=po, n=n, E=E, mean=mu, sd=rho, corr=None, X=X))
            po += 2 * n
        else:
            nc = mvn_ncorr(n)
            mean, sdr, corr = params[po:po + n], params[po + n:po + 2 * n], params[po + 2 * n:po + 2 * n + nc]
            E = eps[eo:eo + S * n].reshape(S, n)
            X = mean[None] + E @ mvn_dense_L(sdr, corr, n).T
            out.append(dict(po=po, n=n, E=E, mean=mean, sd=sdr, corr=corr, X=X))
            po += 2 * n + nc
        eo += S * n
    return out


def _split(layers, Xl):
    return ([x["X"][:, :i * o].reshape(-1, o, i) for x, (i, o) in zip(Xl, layers)],
            [x["X"][:, i * o:] for x, (i, o) in zip(Xl, layers)])


def inner_hvp(family, layers, params, u, z, w, eps, S, vec, prior_sd=1.0):
    if family == "lenet":
        u = np.asarray(u)
        val, g, hv, du, dw = lenet_inner_hvp(params, u.reshape(-1, 1, 28, 28), z, w, eps, S, vec,
                                             prior_sd)
        return val, g, hv, du.reshape(u.shape), dw
    """Hessian-vector product of the negative inner ELBO (psvi_classes.py:488-511)
    at fixed eps, H vec, and the mixed products d/du (vec . grad) and
    d/dw (vec . grad) -- what hypergrad's CG_normaleq takes from autograd
    (torch_grad / jvp of GradientDescent's fp_map, psvi/hypergrad/
    hypergradients.py:199-244, 308-311).  Forward-over-reverse (Pearlmutter
    R-op): tangent sample x_dot = J vec, tangent forward, R-backward; the
    ReLU masks are constant.  Returns (value, grad, Hv, d_u, d_w)."""
    params = np.asarray(params, np.float64)
    vec = np.asarray(vec, np.float64)
    eps = np.asarray(eps, np.float64)
    u = np.asarray(u, np.float64)
    w = np.asarray(w, np.float64)
    s0sq = float(prior_sd) ** 2
    Xl = _sample(family, layers, params, eps, S)
    Ws, bs = _split(layers, Xl)
    # tangent sample
    for x in Xl:
        po, n, E = x["po"], x["n"], x["E"]
        vm, vs_ = vec[po:po + n], vec[po + n:po + 2 * n]
        dsd = sigmoid(x["sd"]) * vs_
        if family == "mf":
            x["Xd"] = vm[None] + dsd[None] * E
        else:
            nc = mvn_ncorr(n)
            Lv = np.zeros((n, n))
            Lv[np.arange(n), np.arange(n)] = dsd
            r, c = tril_rows_cols(n)
            Lv[r, c] = vec[po + 2 * n:po + 2 * n + nc]
            x["Xd"] = vm[None] + E @ Lv.T
    Wd = [x["Xd"][:, :i * o].reshape(S, o, i) for x, (i, o) in zip(Xl, layers)]
    bd = [x["Xd"][:, i * o:] for x, (i, o) in zip(Xl, layers)]
    L = len(layers)
    M = u.shape[0]
    hs, acts = _net_rows_forward(u, Ws, bs)
    hd = [np.zeros_like(hs[0])]
    for l in range(L):
        ad = np.einsum("smi,soi->smo", hd[l], Ws[l]) + np.einsum("smi,soi->smo", hs[l], Wd[l]) \
            + bd[l][:, None, :]
        hd.append(ad * (acts[l] > 0) if l < L - 1 else ad)
    logits, ldot = hs[-1], hd[-1]
    mx = logits.max(-1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(-1, keepdims=True)))[..., 0]
    zi = np.asarray(z).astype(np.int64)
    nll = lse - logits[:, np.arange(M), zi]
    p = np.exp(logits - lse[..., None])
    pmo = p.copy()
    pmo[:, np.arange(M), zi] -= 1.0
    nll_dot = (pmo * ldot).sum(-1)                                   # (S, M)
    pdot = p * (ldot - (p * ldot).sum(-1, keepdims=True))
    g = pmo * w[None, :, None]
    gd = pdot * w[None, :, None]
    G, Gd = [None] * L, [None] * L
    for l in range(L - 1, -1, -1):
        dW = np.einsum("smo,smi->soi", g, hs[l])
        dWd = np.einsum("smo,smi->soi", gd, hs[l]) + np.einsum("smo,smi->soi", g, hd[l])
        G[l] = np.concatenate([dW.reshape(S, -1), g.sum(1)], axis=1)
        Gd[l] = np.concatenate([dWd.reshape(S, -1), gd.sum(1)], axis=1)
        g_new = np.einsum("smo,soi->smi", g, Ws[l])
        gd_new = np.einsum("smo,soi->smi", gd, Ws[l]) + np.einsum("smo,soi->smi", g, Wd[l])
        if l > 0:
            g, gd = g_new * (acts[l - 1] > 0), gd_new * (acts[l - 1] > 0)
        else:
            d_u = gd_new.sum(0)
    value = float((nll * w[None]).sum())
    grad = np.zeros_like(params)
    hv = np.zeros_like(params)
    for l, x in enumerate(Xl):
        po, n, E, sd = x["po"], x["n"], x["E"], x["sd"]
        sp, sg = softplus(sd), sigmoid(sd)
        vm, vsd = vec[po:po + n], vec[po + n:po + 2 * n]
        mean = x["mean"]
        ge = (G[l] * E).sum(0)
        value += float((0.5 * ((sp ** 2 + mean ** 2) / s0sq - 1.0 - np.log(sp ** 2 / s0sq))).sum())
        grad[po:po + n] = G[l].sum(0) + mean / s0sq
        grad[po + n:po + 2 * n] = (ge + sp / s0sq - 1.0 / sp) * sg
        hv[po:po + n] = Gd[l].sum(0) + vm / s0sq
        kl2 = (1.0 / sp ** 2 + 1.0 / s0sq) * sg ** 2 + (sp / s0sq - 1.0 / sp) * sg * (1.0 - sg)
        hv[po + n:po + 2 * n] = (Gd[l] * E).sum(0) * sg + ge * sg * (1.0 - sg) * vsd + kl2 * vsd
        if family != "mf":
            nc = mvn_ncorr(n)
            corr = x["corr"]
            r, c = tril_rows_cols(n)
            value += float(0.5 * (corr ** 2).sum() / s0sq)
            grad[po + 2 * n:po + 2 * n + nc] = (G[l].T @ E)[r, c] + corr / s0sq
            hv[po + 2 * n:po + 2 * n + nc] = (Gd[l].T @ E)[r, c] + vec[po + 2 * n:po + 2 * n + nc] / s0sq
    return value, grad, hv, d_u, nll_dot.sum(0)


def inner_grad_uw(family, layers, params, u, z, w, eps, S, prior_sd=1.0):
    """Negative inner ELBO, its parameter gradient and its gradients w.r.t. u
    and w (for finite-difference checks of inner_hvp)."""
    params = np.asarray(params, np.float64)
    Xl = _sample(family, layers, params, np.asarray(eps, np.float64), S)
    Ws, bs = _split(layers, Xl)
    u = np.asarray(u, np.float64)
    w = np.asarray(w, np.float64)
    M = u.shape[0]
    hs, acts = _net_rows_forward(u, Ws, bs)
    logits = hs[-1]
    mx = logits.max(-1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(-1, keepdims=True)))[..., 0]
    zi = np.asarray(z).astype(np.int64)
    nll = lse - logits[:, np.arange(M), zi]
    pmo = np.exp(logits - lse[..., None])
    pmo[:, np.arange(M), zi] -= 1.0
    dWs, dbs, dX = _net_rows_backward(np.broadcast_to(w[None], nll.shape), pmo, hs, acts, Ws)
    fn = mf_elbo_grad if family == "mf" else mvn_elbo_grad
    val, grad = fn(layers, params, u, z, w, eps, S, prior_sd)
    return val, grad, dX.sum(0), nll.sum(0)


def torch_adam_step(p, g, m, v, t, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam (the reference's optim_u / optim_v), t 1-based."""
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    denom = np.sqrt(v) / np.sqrt(1 - beta2 ** t) + eps
    return p - (lr / (1 - beta1 ** t)) * m / denom, m, v


class Variant:
    """What a PSVI plugin class changes in the outer step (hyper_step /
    nested_step), psvi_classes.py:1344-1884:
      f        "softmax" (PSVILearnV and subclasses) or "exp_alpha_softmax"
               (PSVIAV / PSVIAFixedU: w = N exp(alpha) softmax(v), 1486-1488);
      alpha    the starting alpha (exp_alpha_softmax), stepped by its own
               torch Adam with lr0alpha (1489, 1578, 1610);
      fixed_u  PSVIFixedU / PSVIAFixedU: u.requires_grad_(False), optim_u never
               stepped (1631-1742, 1790-1884);
      outer    "iw" (PSVI.psvi_elbo) or "ablated" (PSVI_Ablated / PSVI_No_IW);
      noiw     PSVI_No_IW's single-sample inner objective: 2-d logits are
               unsqueezed to (M, 1, C) (psvi_classes.py:492-493), so
               Categorical.log_prob(z) broadcasts to (M, M) and the objective is
               sum_i sum_j w_j NLL(logits_i, z_j) = sum_i sum_c W_c NLL(logits_i, c),
               W_c = sum_{j: z_j = c} w_j: the standard objective over M*C
               expanded rows (u_i, class c, weight W_c)."""

    def __init__(self, f="softmax", alpha=None, fixed_u=False, outer="iw", noiw=False,
                 lr0alpha=1e-3):
        self.f, self.alpha, self.fixed_u = f, alpha, fixed_u
        self.outer, self.noiw, self.lr0alpha = outer, noiw, lr0alpha


def weights_vjp(v, alpha, dw, N, f="softmax"):
    """(d/dv, d/dalpha) of dw . w with w = N f(v) (coreset_weights)."""
    v = np.asarray(v, np.float64)
    e = np.exp(v - v.max())
    sm = e / e.sum()
    scale = N * (np.exp(alpha) if f == "exp_alpha_softmax" else 1.0)
    gs = scale * np.asarray(dw, np.float64)
    dv = sm * (gs - (gs * sm).sum())
    dalpha = float((gs * sm).sum()) if f == "exp_alpha_softmax" else None
    return dv, dalpha


def inner_rows(u, z, w, C, noiw):
    """The rows the inner objective scores: (u, z, w) itself, or PSVI_No_IW's
    M*C expanded rows (Variant.noiw); fold(du, dw) maps row gradients back."""
    u = np.asarray(u, np.float64)
    if not noiw:
        return u, z, w, lambda du, dw: (du, dw)
    M = u.shape[0]
    zi = np.asarray(z).astype(np.int64)
    Wc = np.bincount(zi, weights=np.asarray(w, np.float64), minlength=C)
    ue = np.repeat(u, C, axis=0)                      # row i*C + c
    ze = np.tile(np.arange(C), M).astype(np.float64)
    we = np.tile(Wc, M)

    def fold(du, dw):
        return (np.asarray(du).reshape((M, C) + u.shape[1:]).sum(1),
                np.asarray(dw).reshape(M, C).sum(0)[zi])
    return ue, ze, we, fold


def _outer_rows(var, u, z, w, xb, yb, N):
    """Rows, labels, weights and pseudo count of the outer objective."""
    Nx = xb.shape[0]
    if var.outer == "ablated":   # model(xbatch) only (psvi_classes.py:1402)
        return np.asarray(xb, np.float64), np.asarray(yb), np.full(Nx, N / Nx), 0
    return (np.concatenate([u, xb]), np.concatenate([z, yb]),
            np.concatenate([w, np.full(Nx, N / Nx)]), u.shape[0])


def _outer(var, family, layers, p, u, z, w, xb, yb, N, eps, S, prior_sd):
    X, zz, ww, Mu = _outer_rows(var, u, z, w, xb, yb, N)
    loss, g, gu, gw = outer_elbo_grad(family, layers, p, X, zz, ww, Mu, eps, S, prior_sd,
                                      mode=var.outer)
    if Mu == 0:
        gu, gw = np.zeros_like(u), np.zeros(u.shape[0])
    return loss, g, gu.reshape(u.shape), gw


def _hparam_steps(var, u, v, u_grad, v_grad, a_grad, lr0u, lr0v):
    """The optim_u / optim_v / optim_alpha steps (first torch Adam step each)."""
    u_new = u if var.fixed_u else torch_adam_step(u, u_grad, 0 * u, 0 * u, 1, lr0u)[0]
    v_new = torch_adam_step(v, v_grad, 0 * v, 0 * v, 1, lr0v)[0]
    a_new = None
    if var.f == "exp_alpha_softmax":
        a = np.array([var.alpha], np.float64)
        a_new = float(torch_adam_step(a, np.array([a_grad]), 0 * a, 0 * a, 1, var.lr0alpha)[0][0])
    return u_new, v_new, a_new


def _n_classes(layers, family):
    return 10 if family == "lenet" else layers[-1][1]


def hyper_step(family, layers, params0, u, z, v, N, xb, yb, eps_inner, eps_outer, S, T, K,
               lr0net, lr0u, lr0v, linsys_lr=1e-4, prior_sd=1.0, cg_tol=1e-10,
               approx="CG_normaleq", variant=None):
    """PSVI.hyper_step with the CG_normaleq hypergradient (psvi_classes.py:602-687,
    psvi/hypergrad/hypergradients.py:199-244, CG_torch.py:9-45), PSVILearnV
    weights f = softmax (v learned, not clamped) unless ``variant`` (Variant:
    PSVIAV 1504-1581, PSVIAFixedU 1774-1850, PSVI_Ablated / PSVI_No_IW through
    the base method) says otherwise.  eps_inner: the draws of the
    inner-objective calls in order -- T inner Adam steps, fp_map, the initial
    jvp (2: the first only sizes its dummy), then 2 per CG iteration;
    eps_outer: the outer objective's draws (hypergradient, returned loss).
    approx="fixed_point": hypergrad's fixed_point with stochastic=True
    (hypergradients.py:83-140): vs <- J^T vs + g_w for K draws of fp_map, then
    one more draw for the final torch_grad.
    Returns dict(params, u, v, u_grad, v_grad, ll) (+ alpha, alpha_grad)."""
    var = variant or Variant()
    if var.fixed_u and var.f != "exp_alpha_softmax":
        # PSVIFixedU.hyper_step hands hypergrad a DifferentiableAdam as fp_map
        # (psvi_classes.py:1710): it splits the plain parameter list in three
        # and the model call fails (Appendix B #24 of SURVEY.md)
        raise IndexError("list index out of range (PSVIFixedU.hyper_step: 3-way "
                         "DifferentiableAdam fp_map)")
    u = np.asarray(u, np.float64)
    v = np.asarray(v, np.float64)
    C = _n_classes(layers, family)

    def wts(vv, aa=var.alpha):
        return coreset_weights(vv, N, var.f, aa)

    w = wts(v)
    ui, zi, wi, fold = inner_rows(u, z, w, C, var.noiw)
    if family == "lenet":
        _, _, traj, _, _ = lenet_inner_loop(params0, ui, zi, wi, eps_inner[:T], S, lr0net,
                                            "hypergrad", prior_sd)
    else:
        _, _, traj, _, _ = run_inner_loop(family, layers, params0, ui, zi, wi, eps_inner[:T], S,
                                          lr0net, "hypergrad")
    p = traj[-1]
    ei = list(eps_inner[T:])
    o_loss, g_w, g_u, g_wts = _outer(var, family, layers, p, u, z, w, xb, yb, N, eps_outer[0],
                                     S, prior_sd)
    lr = linsys_lr

    def hv(e, x):
        val, g, h, du, dw = inner_hvp(family, layers, p, ui, zi, wi, e, S, x, prior_sd)
        du, dw = fold(du, dw)
        return val, g, h, du, dw

    if approx == "fixed_point":
        vs = np.zeros_like(g_w)
        for _ in range(K):
            prev = vs
            vs = vs - lr * hv(ei.pop(0), vs)[2] + g_w   # stochastic: a fresh fp_map each time
            if float(np.linalg.norm(vs - prev)) < cg_tol:
                break
        xk, eA = vs, ei.pop(0)
    else:
        eA = ei.pop(0)                              # w_mapped = fp_map(params, hparams)

        def jvp(x):                                 # J x = x - lr H x at a fresh draw
            ei.pop(0)                               # the dummy's fp_map call
            return x - lr * hv(ei.pop(0), x)[2]

        def A(x):                                   # dfp_map_dw
            vmj = lr * hv(eA, x)[2]                 # x - J^T x
            return vmj - jvp(vmj)

        b = g_w - jvp(g_w)
        xk = np.zeros_like(b)
        r = b.copy()
        pk = r.copy()
        for _ in range(K):
            Ap = A(pk)
            rTr = float(r @ r)
            alpha = rTr / float(pk @ Ap)
            xn = xk + alpha * pk
            rn = r - alpha * Ap
            if float(np.linalg.norm(rn)) < cg_tol:
                break
            beta = float(rn @ rn) / rTr
            pk = rn + beta * pk
            xk, r = xn, rn
    # grads = torch_grad(w_mapped, hparams, vs) = -lr d/dhp (vs . grad_p inner)
    _, _, _, du, dw = hv(eA, xk)
    u_grad = -lr * du + g_u
    dw_tot = -lr * dw + g_wts
    v_grad, a_grad = weights_vjp(v, var.alpha, dw_tot, N, var.f)
    u_new, v_new, a_new = _hparam_steps(var, u, v, u_grad, v_grad, a_grad, lr0u, lr0v)
    ll = _outer(var, family, layers, p, u_new, z, wts(v_new, a_new), xb, yb, N, eps_outer[1], S,
                prior_sd)[0]
    out = dict(params=p, u=u_new, v=v_new, u_grad=None if var.fixed_u else u_grad,
               v_grad=v_grad, ll=ll)
    if a_new is not None:
        out.update(alpha=a_new, alpha_grad=a_grad)
    return out


def adam_higher_adjoint(lt, lm, lv, m, v, g, t, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """Reverse of one robust_higher DifferentiableAdam step (optim.py:318-367)
        m' = b1 m + (1-b1) g,  v' = b2 v + (1-b2) g^2,
        p' = p - (lr/bc1) m' / (sqrt(v' + 1e-8)/sqrt(bc2) + eps):
    given the adjoints (lt, lm, lv) of (p', m', v') and the step's (m', v', g),
    returns (adjoint of g, adjoint of m, adjoint of v); p's adjoint is lt
    plus H^T (adjoint of g)."""
    bc1, bc2 = 1.0 - beta1 ** t, 1.0 - beta2 ** t
    c = lr / bc1
    sq = np.sqrt(v + 1e-8)
    D = sq / np.sqrt(bc2) + eps
    lm2 = lm - lt * c / D
    lv2 = lv + lt * c * m / (D * D) / (2.0 * sq * np.sqrt(bc2))
    lg = lm2 * (1.0 - beta1) + lv2 * 2.0 * (1.0 - beta2) * g
    return lg, beta1 * lm2, beta2 * lv2



def nested_step(family, layers, params0, u, z, v, N, xb, yb, eps_inner, eps_outer, S, T,
                lr0net, lr0u, lr0v, prior_sd=1.0, variant=None):
    """PSVI.nested_step (psvi_classes.py:541-600), PSVILearnV (f = softmax, v not
    clamped) unless ``variant`` (Variant: PSVIAV 1583-1620, PSVIFixedU
    1631-1657, PSVIAFixedU 1852-1884, PSVI_Ablated / PSVI_No_IW through the
    base method): T higher-Adam steps from params0 with fresh state, the outer
    objective at the result, its gradient w.r.t. u and v (and alpha) back
    through the unrolled steps (reverse-mode through Adam, one Hessian-vector
    product and mixed product per step), then the hparam Adam steps.
    Returns dict(params, u, v, u_grad, v_grad, loss) (+ alpha, alpha_grad)."""
    var = variant or Variant()
    u = np.asarray(u, np.float64)
    v = np.asarray(v, np.float64)
    C = _n_classes(layers, family)
    w = coreset_weights(v, N, var.f, var.alpha)
    ui, zi, wi, fold = inner_rows(u, z, w, C, var.noiw)
    if family == "lenet":
        f = lambda _l, p, uu, zz, ww, e, S, sd: lenet_elbo_grad(p, uu, zz, ww, e, S, sd)
    else:
        f = mf_elbo_grad if family == "mf" else mvn_elbo_grad
    p = np.asarray(params0, np.float64).copy()
    m = np.zeros_like(p)
    vv = np.zeros_like(p)
    hist = []
    for t in range(T):
        _, g = f(layers, p, ui, zi, wi, eps_inner[t], S, prior_sd)
        pn, m, vv = adam_higher(p, g, m, vv, t + 1, lr0net)
        hist.append((p, m.copy(), vv.copy(), g))
        p = pn
    loss, lt, gu, gw = _outer(var, family, layers, p, u, z, w, xb, yb, N, eps_outer[0], S,
                              prior_sd)
    lm = np.zeros_like(p)
    lv = np.zeros_like(p)
    for t in range(T - 1, -1, -1):
        pt, mt, vt, gt = hist[t]
        lg, lm, lv = adam_higher_adjoint(lt, lm, lv, mt, vt, gt, t + 1, lr0net)
        _, _, hv, du, dw = inner_hvp(family, layers, pt, ui, zi, wi, eps_inner[t], S, lg,
                                     prior_sd)
        du, dw = fold(du, dw)
        lt = lt + hv
        gu = gu + du
        gw = gw + dw
    v_grad, a_grad = weights_vjp(v, var.alpha, gw, N, var.f)
    u_new, v_new, a_new = _hparam_steps(var, u, v, gu, v_grad, a_grad, lr0u, lr0v)
    out = dict(params=p, u=u_new, v=v_new, u_grad=None if var.fixed_u else gu, v_grad=v_grad,
               loss=loss)
    if a_new is not None:
        out.update(alpha=a_new, alpha_grad=a_grad)
    return out


def evaluate_batch(family, layers, params, X, z, w_pseudo, n_pseudo, eps, S, correction=True,
                   prior_sd=1.0, clamp_eps=np.finfo(np.float64).eps):
    """One test batch of PSVI.evaluate (psvi_classes.py:1031-1108): X = cat(u, xt),
    z = cat(z, yt).  The weights use the reference's sign: its pseudo_nll there
    is log_prob(z).matmul(N f(v)) (a log-likelihood), so
    lw_s = +sum_m w_m NLL_sm + sampled_nkl_s.  Returns (correct, summed NLL,
    entropy of W, normalised ESS, probs (Nt, C)); the NLL is
    -Categorical(probs).log_prob(yt) with torch's clamp to [eps, 1 - eps]."""
    if family == "lenet":
        return lenet_evaluate_batch(params, np.asarray(X).reshape(-1, 1, 28, 28), z, w_pseudo,
                                    n_pseudo, eps, S, correction, prior_sd, clamp_eps)
    params = np.asarray(params, np.float64)
    eps = np.asarray(eps, np.float64)
    X = np.asarray(X, np.float64)
    s0 = float(prior_sd)
    Xl = _sample(family, layers, params, eps, S)
    Ws, bs = _split(layers, Xl)
    n_tot = sum(i * o + o for i, o in layers)
    sumlog = sum(float(np.log(softplus(x["sd"])).sum()) for x in Xl)
    xsq = sum((x["X"] ** 2).sum(1) for x in Xl)
    esq = sum((x["E"] ** 2).sum(1) for x in Xl)
    nkl = -xsq / (2 * s0 ** 2) - n_tot * np.log(s0) + 0.5 * esq + sumlog
    hs, _ = _net_rows_forward(X, Ws, bs)
    logits = hs[-1]
    R = X.shape[0]
    mx = logits.max(-1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(-1, keepdims=True)))[..., 0]
    zi = np.asarray(z).astype(np.int64)
    nll = lse - logits[:, np.arange(R), zi]
    Mu = int(n_pseudo)
    lw = nll[:, :Mu] @ np.asarray(w_pseudo, np.float64)[:Mu] + nkl
    W = np.exp(lw - lw.max())
    W /= W.sum()
    p = np.exp(logits[:, Mu:] - lse[:, Mu:, None])           # (S, Nt, C)
    probs = np.einsum("s,snc->nc", W, p) if correction else p.mean(0)
    yt = zi[Mu:]
    correct = float((probs.argmax(-1) == yt).sum())
    pn = probs / probs.sum(-1, keepdims=True)
    q = np.clip(pn[np.arange(len(yt)), yt], clamp_eps, 1 - clamp_eps)
    ent = float(-(W[W > 0] * np.log(W[W > 0])).sum())
    ness = float(W.sum() ** 2 / (W ** 2).sum() / S)
    return correct, float(-np.log(q).sum()), ent, ness, probs


# ------------------------------------------------------------------ LeNet
# make_lenet (psvi/models/neural_net.py:334-359) with the default VI classes:
#   VIConv2d(1,6,5,pad 2) ReLU BatchMaxPool2d(2)  VIConv2d(6,16,5) ReLU BatchMaxPool2d(2)
#   Flatten  VILinear(400,120) ReLU  VILinear(120,84) ReLU  VILinear(84,10)
# The convs and the first two linears carry the model's mc_samples (S weight
# sets); the last linear keeps the default mc_samples=1: ONE shared sample
# (weight batch shape (), neural_net.py:164-170).  inner_elbo's KL sums over
# VILinear modules only (psvi_classes.py:506-510): the conv layers have none.
LENET_LAYERS = [  # (n_weight, n_bias, batched over S, has KL)
    (150, 6, True, False), (2400, 16, True, False),
    (48000, 120, True, True), (10080, 84, True, True), (840, 10, False, True)]


def lenet_param_count():
    return 2 * sum(nw + nb for nw, nb, _, _ in LENET_LAYERS)


def lenet_eps_count(S):
    return sum((S if bat else 1) * (nw + nb) for nw, nb, bat, _ in LENET_LAYERS)


def _windows(x, k):
    """(..., H, W) -> (..., H-k+1, W-k+1, k, k) sliding views."""
    return np.lib.stride_tricks.sliding_window_view(x, (k, k), axis=(-2, -1))


def _conv(x, W, b, pad):
    """Per-sample conv: x (S,M,Ci,H,W), W (S,Co,Ci,k,k), b (S,Co).  Equal to
    VIConv2d.forward's grouped conv over the S-repeated input (neural_net.py:202-246)."""
    k = W.shape[-1]
    xp = np.pad(x, [(0, 0)] * 3 + [(pad, pad)] * 2)
    return (np.einsum("smchwij,socij->smohw", _windows(xp, k), W, optimize=True)
            + b[:, None, :, None, None])


def _relu_pool(a):
    """relu then 2x2/2 max-pool (BatchMaxPool2d, neural_net.py:249-255); returns
    the pooled map and the gradient route: flat window index (row-major, the
    first maximum, as torch's max_pool2d) or -1 where relu kills it."""
    S, M, C, H, W = a.shape
    win = a.reshape(S, M, C, H // 2, 2, W // 2, 2).transpose(0, 1, 2, 3, 5, 4, 6)
    win = win.reshape(S, M, C, H // 2, W // 2, 4)
    r = np.maximum(win, 0.0)
    arg = r.argmax(-1)
    out = np.take_along_axis(r, arg[..., None], -1)[..., 0]
    arg = np.where(out > 0, arg, -1)
    return out, arg


def _unpool(g, arg, H, W):
    S, M, C, h, w = g.shape
    full = np.zeros((S, M, C, h, w, 4))
    ok = arg >= 0
    np.put_along_axis(full, np.where(ok, arg, 0)[..., None], np.where(ok, g, 0.0)[..., None], -1)
    full = full.reshape(S, M, C, h, w, 2, 2).transpose(0, 1, 2, 3, 5, 4, 6)
    return full.reshape(S, M, C, H, W)


def lenet_sample(params, eps, S):
    """W_s = mu + softplus(rho) eps_s per layer (VIMixin.rsample, neural_net.py:155-162)."""
    params = np.asarray(params, np.float64)
    eps = np.asarray(eps, np.float64)
    out, po, eo = [], 0, 0
    for nw, nb, bat, _ in LENET_LAYERS:
        n = nw + nb
        mu, rho = params[po:po + n], params[po + n:po + 2 * n]
        ns = S if bat else 1
        e_w = eps[eo:eo + ns * nw].reshape(ns, nw)
        e_b = eps[eo + ns * nw:eo + ns * n].reshape(ns, nb)
        E = np.concatenate([e_w, e_b], 1)
        out.append(dict(po=po, n=n, nw=nw, mu=mu, rho=rho, E=E, bat=bat,
                        X=mu[None] + softplus(rho)[None] * E))
        po += 2 * n
        eo += ns * n
    return out


def lenet_forward(Xl, u, S):
    """LeNet forward over (S, M) images u (M,1,28,28); returns (logits, cache)."""
    u = np.asarray(u, np.float64).reshape(-1, 1, 28, 28)
    M = u.shape[0]
    c1, c2, f1, f2, f3 = Xl
    W1, b1 = c1["X"][:, :150].reshape(S, 6, 1, 5, 5), c1["X"][:, 150:]
    W2, b2 = c2["X"][:, :2400].reshape(S, 16, 6, 5, 5), c2["X"][:, 2400:]
    x0 = np.broadcast_to(u[None], (S, M, 1, 28, 28))
    a1 = _conv(x0, W1, b1, 2)
    p1, g1 = _relu_pool(a1)
    a2 = _conv(p1, W2, b2, 0)
    p2, g2 = _relu_pool(a2)
    x = p2.reshape(S, M, 400)
    Wf = [f1["X"][:, :48000].reshape(S, 120, 400), f2["X"][:, :10080].reshape(S, 84, 120),
          np.broadcast_to(f3["X"][:, :840].reshape(1, 10, 84), (S, 10, 84))]
    bf = [f1["X"][:, 48000:], f2["X"][:, 10080:], np.broadcast_to(f3["X"][:, 840:], (S, 10))]
    hs = [x]
    for l in range(3):
        a = np.einsum("smi,soi->smo", hs[-1], Wf[l]) + bf[l][:, None, :]
        hs.append(np.maximum(a, 0.0) if l < 2 else a)
    cache = dict(x0=x0, W1=W1, W2=W2, p1=p1, g1=g1, g2=g2, Wf=Wf, hs=hs)
    return hs[-1], cache


def _lenet_backward(c, d, S, M, want_dx=False):
    """Backward of the LeNet forward (cache c) from d logits (S, M, 10): per-layer
    per-sample weight gradients G[l] (S, n_l) in parameter order (the last
    layer's too), and, with want_dx, d input (S, M, 784) through the conv1
    transpose."""
    hs, Wf = c["hs"], c["Wf"]
    G = [None] * 5
    for l in (2, 1, 0):
        dW = np.einsum("smo,smi->soi", d, hs[l])
        db = d.sum(1)
        G[2 + l] = np.concatenate([dW.reshape(S, -1), db], 1)
        d = np.einsum("smo,soi->smi", d, Wf[l])
        if l > 0:
            d = d * (hs[l] > 0)
    dp2 = d.reshape(S, M, 16, 5, 5)
    da2 = _unpool(dp2, c["g2"], 10, 10)
    dW2 = np.einsum("smohw,smchwij->socij", da2, _windows(c["p1"], 5), optimize=True)
    G[1] = np.concatenate([dW2.reshape(S, -1), da2.sum((1, 3, 4))], 1)
    da2p = np.pad(da2, [(0, 0)] * 3 + [(4, 4)] * 2)
    dp1 = np.einsum("smohwij,socij->smchw", _windows(da2p, 5), c["W2"][..., ::-1, ::-1],
                    optimize=True)
    da1 = _unpool(dp1, c["g1"], 28, 28)
    x0p = np.pad(c["x0"], [(0, 0)] * 3 + [(2, 2)] * 2)
    dW1 = np.einsum("smohw,smchwij->socij", da1, _windows(x0p, 5), optimize=True)
    G[0] = np.concatenate([dW1.reshape(S, -1), da1.sum((1, 3, 4))], 1)
    dx = None
    if want_dx:
        da1p = np.pad(da1, [(0, 0)] * 3 + [(2, 2)] * 2)
        dx = np.einsum("smchwij,scij->smhw", _windows(da1p, 5), c["W1"][:, :, 0, ::-1, ::-1],
                       optimize=True).reshape(S, M, 784)
    return G, dx


def _lenet_param_grad(Xl, G, s0, kl_layers=True, sck=0.0):
    """d / d (mu, rho) from per-sample weight gradients; the VILinear layers
    add the analytic KL gradient (kl_layers) and/or the explicit sum_s ck_s /
    sigma of the sampled KL (sck).  Returns (grad, kl)."""
    P = sum(2 * (nw + nb) for nw, nb, _, _ in LENET_LAYERS)
    grad = np.zeros(P)
    kl = 0.0
    for (nw, nb, bat, has_kl), x, g in zip(LENET_LAYERS, Xl, G):
        po, n, mu, rho = x["po"], x["n"], x["mu"], x["rho"]
        if not bat:
            g = g.sum(0, keepdims=True)                           # shared sample
        sp = softplus(rho)
        gmu = g.sum(0)
        grho = (g * x["E"]).sum(0)
        if has_kl and kl_layers:
            vr = (sp / s0) ** 2
            kl += float((0.5 * (vr + (mu / s0) ** 2 - 1.0 - np.log(vr))).sum())
            gmu = gmu + mu / s0 ** 2
            grho = grho + sp / s0 ** 2 - 1.0 / sp
        if has_kl and sck:
            grho = grho + sck / sp
        grad[po:po + n] = gmu
        grad[po + n:po + 2 * n] = grho * sigmoid(rho)
    return grad, kl


def lenet_elbo_grad(params, u, z, w, eps, S, prior_sd=1.0):
    """Negative inner ELBO (psvi_classes.py:488-511) of a make_lenet model and
    its gradient w.r.t. the flat parameter vector (parameters_to_vector order:
    per layer weight, bias, _weight_sd, _bias_sd)."""
    params = np.asarray(params, np.float64)
    s0 = float(prior_sd)
    Xl = lenet_sample(params, eps, S)
    logits, c = lenet_forward(Xl, u, S)
    M = logits.shape[1]
    w = np.asarray(w, np.float64)
    zi = np.asarray(z).astype(np.int64)
    mx = logits.max(-1, keepdims=True)
    e = np.exp(logits - mx)
    lse = mx[..., 0] + np.log(e.sum(-1))
    nll = lse - logits[:, np.arange(M), zi]
    data = float((nll @ w).sum())
    P = e / e.sum(-1, keepdims=True)
    P[:, np.arange(M), zi] -= 1.0
    G, _ = _lenet_backward(c, P * w[None, :, None], S, M)
    grad, kl = _lenet_param_grad(Xl, G, s0)
    return data + kl, grad


def lenet_outer_elbo_grad(params, X, z, w, n_pseudo, eps, S, prior_sd=1.0, mode="iw"):
    """PSVI.psvi_elbo (psvi_classes.py:445-486) of a make_lenet model on rows
    X = cat(u, xbatch) (R, 1, 28, 28): sampled_nkl over the VILinear layers
    only (the last one's single shared sample enters every s), W = softmax_s(lw),
    loss = sum_s W_s (data_s - pseudo_s) - mean_s lw_s.  w: per-row weights
    (N f(v) for the pseudo rows, N / Nx for the data rows).  Returns
    (loss, d params, d u (n_pseudo, 784), d w (n_pseudo))."""
    params = np.asarray(params, np.float64)
    s0 = float(prior_sd)
    Xl = lenet_sample(params, eps, S)
    logits, c = lenet_forward(Xl, X, S)
    R = logits.shape[1]
    w = np.asarray(w, np.float64)
    zi = np.asarray(z).astype(np.int64)
    mx = logits.max(-1, keepdims=True)
    e = np.exp(logits - mx)
    lse = mx[..., 0] + np.log(e.sum(-1))
    nll = lse - logits[:, np.arange(R), zi]
    Mu = int(n_pseudo)
    pseudo = nll[:, :Mu] @ w[:Mu]
    data = nll[:, Mu:] @ w[Mu:]
    nkl = np.zeros(S)
    for x in Xl[2:]:
        n = x["n"]
        nkl = nkl + ((-(x["X"] ** 2).sum(1) / (2 * s0 ** 2) - n * np.log(s0)
                      + 0.5 * (x["E"] ** 2).sum(1) + np.log(softplus(x["rho"])).sum()))
    loss, cp, Wt, ck = _outer_coef(pseudo, data, nkl, S, mode)
    grad, gu, gw = _lenet_outer_backward(Xl, c, e, zi, w, Mu, nll, cp, Wt, ck, S, s0)
    return float(loss), grad, gu, gw


def lenet_outer_coef_grad(params, X, z, w, n_pseudo, eps, S, cp, cd, ck, prior_sd=1.0):
    """The sample-sharded outer objective's two passes on these S samples
    (psvi_outer_elbo_grad sample_out, psvi_outer_elbo_grad_coef): the
    per-sample terms (S, 3) [pseudo_s, data_s, nkl_s] and the gradients of
    sum_s (cp_s pseudo_s + cd_s data_s + ck_s nkl_s) w.r.t. params, u and w
    for caller-given coefficients (psvi_classes.py:463-486 split over ranks)."""
    params = np.asarray(params, np.float64)
    s0 = float(prior_sd)
    Xl = lenet_sample(params, eps, S)
    logits, c = lenet_forward(Xl, X, S)
    R = logits.shape[1]
    w = np.asarray(w, np.float64)
    zi = np.asarray(z).astype(np.int64)
    mx = logits.max(-1, keepdims=True)
    e = np.exp(logits - mx)
    lse = mx[..., 0] + np.log(e.sum(-1))
    nll = lse - logits[:, np.arange(R), zi]
    Mu = int(n_pseudo)
    nkl = np.zeros(S)
    for x in Xl[2:]:
        nkl = nkl + ((-(x["X"] ** 2).sum(1) / (2 * s0 ** 2) - x["n"] * np.log(s0)
                      + 0.5 * (x["E"] ** 2).sum(1) + np.log(softplus(x["rho"])).sum()))
    terms = np.stack([nll[:, :Mu] @ w[:Mu], nll[:, Mu:] @ w[Mu:], nkl], 1)
    cp, cd, ck = (np.asarray(a, np.float64) for a in (cp, cd, ck))
    grad, gu, gw = _lenet_outer_backward(Xl, c, e, zi, w, Mu, nll, cp, cd, ck, S, s0)
    return terms, grad, gu, gw


def _lenet_outer_backward(Xl, c, e, zi, w, Mu, nll, cp, Wt, ck, S, s0):
    """d/d(params, u, w) of sum_s (cp_s pseudo_s + Wt_s data_s + ck_s nkl_s)."""
    R = nll.shape[1]
    coef = np.where(np.arange(R)[None, :] < Mu, cp[:, None], Wt[:, None]) * w[None, :]
    Pm = e / e.sum(-1, keepdims=True)
    Pm[:, np.arange(R), zi] -= 1.0
    G, dx = _lenet_backward(c, Pm * coef[..., None], S, R, want_dx=True)
    for l in (2, 3, 4):                   # pathwise sampled-KL: -ck_s x_s / s0^2
        G[l] = G[l] - ck[:, None] * np.broadcast_to(Xl[l]["X"], (S, Xl[l]["n"])) / s0 ** 2
    grad, _ = _lenet_param_grad(Xl, G, s0, kl_layers=False, sck=float(ck.sum()))
    gu = dx[:, :Mu].sum(0)
    gw = cp @ nll[:, :Mu]
    return grad, gu, gw


def lenet_inner_loop(params0, u, z, w, eps_steps, S, lr, adam_kind, prior_sd=1.0, t0=1):
    """T lenet inner steps (run_inner_loop's contract)."""
    p = np.asarray(params0, dtype=np.float64).copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    elbos, grads, traj = [], [], []
    for k, e in enumerate(eps_steps):
        val, g = lenet_elbo_grad(p, u, z, w, e, S, prior_sd)
        elbos.append(val)
        grads.append(g)
        p, m, v = adam(adam_kind, p, g, m, v, t0 + k, lr)
        traj.append(p.copy())
    return np.array(elbos), grads, traj, m, v


# ------------------------------------------------------- MFVI baselines
def mfvi_run(family, layers, params0, x, y, xt, yt, draws, S, iters, log_every, lr, scale,
             eval_last=True, prior_sd=1.0):
    """run_mfvi / run_mfvi_subset (psvi/inference/baselines.py:824-914, 917-1062):
    per iteration loss = scale * sum_{s,b} NLL + KL(VILinear modules only: none
    for a full-covariance stack, baselines.py:889), torch.optim.Adam; every
    log_every iterations (and the last one for run_mfvi: eval_last) the
    predictive of the MEAN LOGITS over S: accuracy and mean NLL.  ``draws`` is
    the flat noise stream in consumption order (training and evaluation
    forwards interleaved).  Returns (elbos, accs, nlls, params)."""
    f = mf_elbo_grad if family == "mf" else mvn_elbo_grad
    n_eps = (mf_eps_count if family == "mf" else mvn_eps_count)(layers, S)
    p = np.asarray(params0, np.float64).copy()
    m, v = np.zeros_like(p), np.zeros_like(p)
    x = np.asarray(x, np.float64)
    w = np.full(x.shape[0], float(scale))
    o = 0
    elbos, accs, nlls = [], [], []
    for i in range(iters):
        e = np.asarray(draws[o:o + n_eps], np.float64)
        o += n_eps
        val, g = f(layers, p, x, y, w, e, S, prior_sd)
        if family != "mf":
            k, gk = f(layers, p, x, y, 0 * w, e, S, prior_sd)
            val, g = val - k, g - gk
        elbos.append(-val)
        p, m, v = torch_adam_step(p, g, m, v, i + 1, lr)
        if i % log_every == 0 or (eval_last and i == iters - 1):
            e = np.asarray(draws[o:o + n_eps], np.float64)
            o += n_eps
            Ws, bs = _split(layers, _sample(family, layers, p, e, S))
            hs, _ = _net_rows_forward(np.asarray(xt, np.float64), Ws, bs)
            lg = hs[-1].mean(0)
            yi = np.asarray(yt).astype(np.int64)
            mx = lg.max(-1, keepdims=True)
            ls = lg - mx - np.log(np.exp(lg - mx).sum(-1, keepdims=True))
            accs.append(float((lg.argmax(-1) == yi).mean()))
            nlls.append(float(-ls[np.arange(len(yi)), yi].mean()))
    assert o == len(draws), (o, len(draws))
    return np.array(elbos), np.array(accs), np.array(nlls), p


def lenet_evaluate_batch(params, X, z, w_pseudo, n_pseudo, eps, S, correction=True,
                         prior_sd=1.0, clamp_eps=np.finfo(np.float64).eps):
    """evaluate_batch for make_lenet: sampled_nkl over the VILinear layers only."""
    params = np.asarray(params, np.float64)
    s0 = float(prior_sd)
    Xl = lenet_sample(params, eps, S)
    logits, _ = lenet_forward(Xl, X, S)
    nkl = np.zeros(S)
    for x in Xl[2:]:
        nkl = nkl + ((-(x["X"] ** 2).sum(1) / (2 * s0 ** 2) - x["n"] * np.log(s0)
                      + 0.5 * (x["E"] ** 2).sum(1) + np.log(softplus(x["rho"])).sum()))
    R = logits.shape[1]
    mx = logits.max(-1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(-1, keepdims=True)))[..., 0]
    zi = np.asarray(z).astype(np.int64)
    nll = lse - logits[:, np.arange(R), zi]
    Mu = int(n_pseudo)
    lw = nll[:, :Mu] @ np.asarray(w_pseudo, np.float64)[:Mu] + nkl
    W = np.exp(lw - lw.max())
    W /= W.sum()
    p = np.exp(logits[:, Mu:] - lse[:, Mu:, None])
    probs = np.einsum("s,snc->nc", W, p) if correction else p.mean(0)
    yt = zi[Mu:]
    correct = float((probs.argmax(-1) == yt).sum())
    pn = probs / probs.sum(-1, keepdims=True)
    q = np.clip(pn[np.arange(len(yt)), yt], clamp_eps, 1 - clamp_eps)
    ent = float(-(W[W > 0] * np.log(W[W > 0])).sum())
    ness = float(W.sum() ** 2 / (W ** 2).sum() / S)
    return correct, float(-np.log(q).sum()), ent, ness, probs


def _route(a, arg):
    """Gather a (S,M,C,H,W) at the pool routes (0 where relu zeroes the window)."""
    S, M, C, H, W = a.shape
    win = a.reshape(S, M, C, H // 2, 2, W // 2, 2).transpose(0, 1, 2, 3, 5, 4, 6)
    win = win.reshape(S, M, C, H // 2, W // 2, 4)
    out = np.take_along_axis(win, np.maximum(arg, 0)[..., None], -1)[..., 0]
    return np.where(arg >= 0, out, 0.0)


def lenet_inner_hvp(params, u, z, w, eps, S, vec, prior_sd=1.0):
    """Hessian-vector product of the LeNet negative inner ELBO at fixed eps and
    the mixed products d/du, d/dw of vec . grad (inner_hvp's contract):
    forward-over-reverse with the relu masks and pool routes held constant.
    Returns (value, grad, Hv, d_u (M, 784), d_w (M,))."""
    params = np.asarray(params, np.float64)
    vec = np.asarray(vec, np.float64)
    s0 = float(prior_sd)
    val, grad = lenet_elbo_grad(params, u, z, w, eps, S, prior_sd)
    Xl = lenet_sample(params, eps, S)
    logits, c = lenet_forward(Xl, u, S)
    M = logits.shape[1]
    w = np.asarray(w, np.float64)
    zi = np.asarray(z).astype(np.int64)
    # tangent weights W_dot = v_mu + sigmoid(rho) v_rho eps
    Td = []
    for x in Xl:
        po, n = x["po"], x["n"]
        Td.append(vec[po:po + n][None] + (sigmoid(x["rho"]) * vec[po + n:po + 2 * n])[None] * x["E"])
    W1d, b1d = Td[0][:, :150].reshape(-1, 6, 1, 5, 5), Td[0][:, 150:]
    W2d, b2d = Td[1][:, :2400].reshape(-1, 16, 6, 5, 5), Td[1][:, 2400:]
    # primal activations (recomputed with pre-activations) and tangent forward
    W1, W2 = c["W1"], c["W2"]
    b1, b2 = Xl[0]["X"][:, 150:], Xl[1]["X"][:, 2400:]
    x0 = c["x0"]
    a1d = _conv(x0, W1d, b1d, 2)
    p1d = _route(a1d, c["g1"])
    a2d = _conv(p1d, W2, np.zeros_like(b2), 0) + _conv(c["p1"], W2d, b2d, 0)
    xd = _route(a2d, c["g2"]).reshape(S, M, 400)
    hs, Wf = c["hs"], c["Wf"]
    Wfd = [Td[2][:, :48000].reshape(S, 120, 400), Td[3][:, :10080].reshape(S, 84, 120),
           np.broadcast_to(Td[4][:, :840].reshape(1, 10, 84), (S, 10, 84))]
    bfd = [Td[2][:, 48000:], Td[3][:, 10080:], np.broadcast_to(Td[4][:, 840:], (S, 10))]
    hds = [xd]
    for l in range(3):
        ad = (np.einsum("smi,soi->smo", hds[-1], Wf[l]) + np.einsum("smi,soi->smo", hs[l], Wfd[l])
              + bfd[l][:, None, :])
        hds.append(ad * (hs[l + 1] > 0) if l < 2 else ad)
    ld = hds[-1]
    mx = logits.max(-1, keepdims=True)
    e = np.exp(logits - mx)
    P = e / e.sum(-1, keepdims=True)
    Pm = P.copy()
    Pm[:, np.arange(M), zi] -= 1.0
    nlld = (Pm * ld).sum(-1)                                     # tangent of NLL_sm
    d = Pm * w[None, :, None]
    dd = w[None, :, None] * (P * ld - P * (P * ld).sum(-1, keepdims=True))
    Gd = [None] * 5
    for l in (2, 1, 0):
        dW = np.einsum("smo,smi->soi", dd, hs[l]) + np.einsum("smo,smi->soi", d, hds[l])
        Gd[2 + l] = np.concatenate([dW.reshape(S, -1), dd.sum(1)], 1)
        dd_new = np.einsum("smo,soi->smi", dd, Wf[l]) + np.einsum("smo,soi->smi", d, Wfd[l])
        d = np.einsum("smo,soi->smi", d, Wf[l])
        if l > 0:
            dd_new = dd_new * (hs[l] > 0)
            d = d * (hs[l] > 0)
        dd = dd_new
    da2 = _unpool(d.reshape(S, M, 16, 5, 5), c["g2"], 10, 10)
    da2d = _unpool(dd.reshape(S, M, 16, 5, 5), c["g2"], 10, 10)
    dW2d = (np.einsum("smohw,smchwij->socij", da2d, _windows(c["p1"], 5), optimize=True)
            + np.einsum("smohw,smchwij->socij", da2, _windows(p1d, 5), optimize=True))
    Gd[1] = np.concatenate([dW2d.reshape(S, -1), da2d.sum((1, 3, 4))], 1)
    pad4 = [(0, 0)] * 3 + [(4, 4)] * 2
    dp1 = np.einsum("smohwij,socij->smchw", _windows(np.pad(da2, pad4), 5), W2[..., ::-1, ::-1],
                    optimize=True)
    dp1d = (np.einsum("smohwij,socij->smchw", _windows(np.pad(da2d, pad4), 5),
                      W2[..., ::-1, ::-1], optimize=True)
            + np.einsum("smohwij,socij->smchw", _windows(np.pad(da2, pad4), 5),
                        W2d[..., ::-1, ::-1], optimize=True))
    da1 = _unpool(dp1, c["g1"], 28, 28)
    da1d = _unpool(dp1d, c["g1"], 28, 28)
    pad2 = [(0, 0)] * 3 + [(2, 2)] * 2
    dW1d = np.einsum("smohw,smchwij->socij", da1d, _windows(np.pad(x0, pad2), 5), optimize=True)
    Gd[0] = np.concatenate([dW1d.reshape(S, -1), da1d.sum((1, 3, 4))], 1)
    dud = (np.einsum("smchwij,scij->smhw", _windows(np.pad(da1d, pad2), 5),
                     W1[:, :, 0, ::-1, ::-1], optimize=True)
           + np.einsum("smchwij,scij->smhw", _windows(np.pad(da1, pad2), 5),
                       W1d[:, :, 0, ::-1, ::-1], optimize=True))
    # primal per-sample G (for the softplus curvature) from the backward helper
    Pw = Pm * w[None, :, None]
    G, _ = _lenet_backward(c, Pw, S, M)
    hv = np.zeros_like(params)
    for (nw, nb, bat, has_kl), x, g, gd in zip(LENET_LAYERS, Xl, G, Gd):
        po, n, mu, rho = x["po"], x["n"], x["mu"], x["rho"]
        if not bat:
            g, gd = g.sum(0, keepdims=True), gd.sum(0, keepdims=True)
        sp, sg = softplus(rho), sigmoid(rho)
        vm, vr = vec[po:po + n], vec[po + n:po + 2 * n]
        E = x["E"]
        hm = gd.sum(0)
        hr = (gd * E).sum(0) * sg + (g * E).sum(0) * sg * (1 - sg) * vr
        if has_kl:
            hm = hm + vm / s0 ** 2
            hr = hr + ((1 / sp ** 2 + 1 / s0 ** 2) * sg * sg + (sp / s0 ** 2 - 1 / sp) * sg * (1 - sg)) * vr
        hv[po:po + n] = hm
        hv[po + n:po + 2 * n] = hr
    return val, grad, hv, dud.sum(0).reshape(M, 784), nlld.sum(0)
