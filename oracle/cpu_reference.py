"""Op-faithful CPU restatement of the reference inner step -- TEST / BASELINE
INFRASTRUCTURE ONLY (imported by tests/ and by bench.py's cpu_baseline leg;
never by the product path).

It replays the reference's torch op sequence for one inner step of
``PSVI.nested_step`` (psvi/inference/psvi_classes.py:549-555):
  forward through torch.distributions (Normal / Independent / MultivariateNormal
  rsample with a dense scale_tril assembled by index_put,
  neural_net.py:117-179, 452-476), Categorical(logits).log_prob(z)
  .matmul(N f(v)) + sum of kl_divergence terms (psvi_classes.py:488-511),
  torch.autograd.grad(create_graph=True) (robust_higher/optim.py:224-229) and
  the higher-Adam update built from tensor ops (optim.py:318-367),
so its wall time on the host is the reference's CPU cost (checked against the
reference's own timing in tests/test_cpu_reference.py).  Numerics are pinned to
tests/golden/*.npz like the oracle.
"""
import math

import torch
import torch.distributions as D
import torch.nn.functional as F


def _inv_softplus(x):
    return math.log(math.expm1(x))


class _MFLayer:
    """One VILinear: params [mu_W, mu_b, rho_W, rho_b] (reference order)."""

    def __init__(self, din, dout, flat, off):
        nw, nb = din * dout, dout
        self.shapes = [(dout, din), (dout,), (dout, din), (dout,)]
        self.sizes = [nw, nb, nw, nb]
        self.din, self.dout = din, dout

    def forward(self, h, p, S, prior_sd):
        muW, mub, rW, rb = p
        qW = D.Independent(D.Normal(muW, F.softplus(rW)), 2)
        qb = D.Independent(D.Normal(mub, F.softplus(rb)), 1)
        W = qW.rsample((S,))
        b = qb.rsample((S, 1))
        out = h.matmul(W.transpose(-2, -1)) + b
        pW = D.Independent(D.Normal(torch.zeros_like(muW), prior_sd), 2)
        pb = D.Independent(D.Normal(torch.zeros_like(mub), prior_sd), 1)
        kl = D.kl_divergence(qW, pW) + D.kl_divergence(qb, pb)
        # VIMixin.sampled_nkl (neural_net.py:110-115) of this draw
        bs = b.squeeze(1)
        self.nkl = (pW.log_prob(W) - qW.log_prob(W)) + (pb.log_prob(bs) - qb.log_prob(bs))
        return out, kl


class _MVNLayer:
    """One VILinearMultivariateNormal: params [mean, _sd, _corr]."""

    def __init__(self, din, dout):
        n = din * dout + dout
        self.n, self.din, self.dout = n, din, dout
        self.shapes = [(n,), (n,), ((n - 1) * (n - 2) // 2,)]
        self.sizes = [n, n, (n - 1) * (n - 2) // 2]
        self.tril = torch.tril_indices(n - 1, n - 1, offset=-1)

    def _dist(self, mean, sd, corr):
        # scale_tril / param_dist are properties in the reference: the dense L
        # is re-assembled on every access (rsample and kl each access it).
        n = self.n
        L = mean.new_zeros(n, n)
        ar = torch.arange(n)
        L[ar, ar] = F.softplus(sd)
        L[self.tril[0], self.tril[1]] = corr
        return D.MultivariateNormal(mean, scale_tril=L)

    def forward(self, h, p, S, prior_sd):
        mean, sd, corr = p
        q = self._dist(mean, sd, corr)
        x = q.rsample((S,))
        W = x[:, :self.din * self.dout].reshape(S, self.dout, self.din)
        b = x[:, self.din * self.dout:].reshape(S, self.dout)
        out = h.matmul(W.transpose(-1, -2)) + b.unsqueeze(-2)
        prior = D.MultivariateNormal(torch.zeros_like(mean),
                                     scale_tril=torch.full_like(mean, prior_sd).diag_embed())
        # MultivariateNormalVIMixin.sampled_nkl (neural_net.py:438-442): triangular solves
        self.nkl = prior.log_prob(x) - self._dist(mean, sd, corr).log_prob(x)
        return out, D.kl_divergence(self._dist(mean, sd, corr), prior)


class RefInnerStep:
    """family 'mf' | 'mvn'; layers [(in, out), ...]."""

    def __init__(self, family, layers, S, prior_sd=1.0):
        self.family, self.S, self.prior_sd = family, S, prior_sd
        self.layers = [(_MFLayer(i, o, None, 0) if family == "mf" else _MVNLayer(i, o))
                       for i, o in layers]

    def split(self, flat):
        out, o = [], 0
        for lay in self.layers:
            ps = []
            for shp, sz in zip(lay.shapes, lay.sizes):
                ps.append(flat[o:o + sz].view(shp))
                o += sz
            out.append(ps)
        return out

    def elbo(self, params_list, u, z, w):
        h = u
        kl = 0.0
        nl = len(self.layers)
        for i, lay in enumerate(self.layers):
            h, k = lay.forward(h, params_list[i], self.S, self.prior_sd)
            kl = kl + k
            if i < nl - 1:
                h = torch.relu(h)
        torch.nn.LogSoftmax(dim=-1)(h).permute(1, 2, 0)  # computed, unused (psvi_classes.py:495)
        nll = -D.Categorical(logits=h).log_prob(z)
        return nll.matmul(w).sum() + kl

    def psvi_elbo(self, params_list, u, z, w, xb, yb, N):
        """PSVI.psvi_elbo (psvi_classes.py:445-486) with the reference's op sequence."""
        X = torch.cat((u, xb))
        labels = torch.cat((z, yb))
        h = X
        nl = len(self.layers)
        for i, lay in enumerate(self.layers):
            h, _ = lay.forward(h, params_list[i], self.S, self.prior_sd)
            if i < nl - 1:
                h = torch.relu(h)
        torch.nn.LogSoftmax(dim=-1)(h).permute(1, 2, 0)
        nlls = -D.Categorical(logits=h).log_prob(labels)
        Nu, Nx = u.shape[0], xb.shape[0]
        pseudo = nlls[:, :Nu].matmul(w)
        data = N / Nx * nlls[:, Nu:].sum(-1)
        lw = -pseudo + sum(lay.nkl for lay in self.layers)
        return lw.softmax(0).mul(data - pseudo).sum() - lw.mean()

    def nested_step(self, params0, u, z, v, N, xb, yb, T, lr, seed=0, eps_inner=None,
                    eps_outer=None):
        """PSVI.nested_step (psvi_classes.py:541-600) for PSVILearnV: T higher-Adam
        steps with create_graph, psvi_elbo, backward to u and v.  eps_inner /
        eps_outer replay recorded draws (flat, reference order)."""
        torch.manual_seed(seed)
        u = u.detach().clone().requires_grad_(True)
        v = v.detach().clone().requires_grad_(True)
        p = [t.detach().clone().requires_grad_(True)
             for ps in self.split(params0.detach().clone()) for t in ps]
        m = [torch.zeros_like(t) for t in p]
        s2 = [torch.zeros_like(t) for t in p]
        for t in range(T):
            w = N * torch.softmax(v, 0)
            with _patched_normal(_EpsReplay(eps_inner[t]) if eps_inner is not None else None):
                loss = self.elbo(self._group(p), u, z, w)
            gs = torch.autograd.grad(loss, p, create_graph=True)
            bc1, bc2 = 1 - 0.9 ** (t + 1), 1 - 0.999 ** (t + 1)
            newp = []
            for i, (pi, gi) in enumerate(zip(p, gs)):
                m[i] = m[i] * 0.9 + 0.1 * gi
                s2[i] = s2[i] * 0.999 + 0.001 * gi * gi
                newp.append(pi - (lr / bc1) * m[i] / ((s2[i] + 1e-8).sqrt() / math.sqrt(bc2) + 1e-8))
            p = newp
        with _patched_normal(_EpsReplay(eps_outer) if eps_outer is not None else None):
            out = self.psvi_elbo(self._group(p), u, z, N * torch.softmax(v, 0), xb, yb, N)
        out.backward()
        return float(out.detach()), u.grad, v.grad

    def run(self, params0, u, z, w, T, lr, eps_list=None, seed=0, adam="higher",
            create_graph=True):
        """T inner steps; eps_list[t] (flat, reference draw order) replaces the
        RNG when given.  Returns (elbos, params)."""
        flat = params0.detach().clone().requires_grad_(True)
        p = [t for ps in self.split(flat) for t in ps]
        p = [t.detach().clone().requires_grad_(True) for t in p]
        m = [torch.zeros_like(t) for t in p]
        v = [torch.zeros_like(t) for t in p]
        elbos = []
        for t in range(T):
            gen = _EpsReplay(eps_list[t]) if eps_list is not None else None
            if gen is None:
                torch.manual_seed(seed + t)
            with _patched_normal(gen):
                grouped = self._group(p)
                loss = self.elbo(grouped, u, z, w)
            elbos.append(float(loss.detach()))
            gs = torch.autograd.grad(loss, p, create_graph=create_graph)
            newp = []
            for i, (pi, gi) in enumerate(zip(p, gs)):
                if adam == "higher":
                    m[i] = m[i] * 0.9 + 0.1 * gi
                    v[i] = v[i] * 0.999 + 0.001 * gi * gi
                    bc1, bc2 = 1 - 0.9 ** (t + 1), 1 - 0.999 ** (t + 1)
                    denom = (v[i] + 1e-8).sqrt() / math.sqrt(bc2) + 1e-8
                    newp.append(pi - (lr / bc1) * m[i] / denom)
                else:
                    m[i] = 0.9 * m[i] + 0.1 * gi
                    v[i] = 0.999 * v[i] + 0.001 * gi ** 2 + 1e-12
                    newp.append(pi - lr * (m[i] / (1 - 0.9 ** (t + 1)))
                                / (torch.sqrt(v[i] / (1 - 0.999 ** (t + 1))) + 1e-8))
            p = newp
        return elbos, torch.cat([x.detach().reshape(-1) for x in p])

    def _group(self, p):
        out, o = [], 0
        for lay in self.layers:
            k = len(lay.shapes)
            out.append(p[o:o + k])
            o += k
        return out


class _LenetLayer:
    """One make_lenet variational layer: [weight, bias, _weight_sd, _bias_sd]."""

    def __init__(self, wshape, batched):
        nw = 1
        for d in wshape:
            nw *= d
        nb = wshape[0]
        self.shapes = [wshape, (nb,), wshape, (nb,)]
        self.sizes = [nw, nb, nw, nb]
        self.batched = batched


class RefLenetStep(RefInnerStep):
    """make_lenet (neural_net.py:334-359) with the reference's op sequence:
    VIConv2d's grouped conv over the S-repeated input (202-246), BatchMaxPool2d
    on the flattened (S*M) maps (249-255), batched VILinear matmuls, the last
    layer one shared sample (mc_samples=1), KL over the VILinear layers only
    (psvi_classes.py:506-510).  run() / nested-step machinery inherited."""

    def __init__(self, S, prior_sd=1.0):
        self.family, self.S, self.prior_sd = "lenet", S, prior_sd
        self.layers = [_LenetLayer((6, 1, 5, 5), True), _LenetLayer((16, 6, 5, 5), True),
                       _LenetLayer((120, 400), True), _LenetLayer((84, 120), True),
                       _LenetLayer((10, 84), False)]

    def _q(self, p):
        W, b, rW, rb = p
        return (D.Independent(D.Normal(W, F.softplus(rW)), W.ndim),
                D.Independent(D.Normal(b, F.softplus(rb)), 1))

    def elbo(self, params_list, u, z, w):
        S = self.S
        x = u.reshape(-1, 1, 28, 28)
        for li, pad in ((0, 2), (1, 0)):
            qW, qb = self._q(params_list[li])
            Ws = qW.rsample((S,))
            bs = qb.rsample((S, 1))
            x = x.repeat(1, S, 1, 1) if x.ndim == 4 else x.transpose(0, 1).flatten(1, 2)
            a = F.conv2d(x, Ws.flatten(0, 1), bs.flatten(), padding=pad, groups=S)
            a = a.view(-1, S, Ws.shape[1], *a.shape[-2:]).transpose(0, 1)
            a = torch.relu(a)
            d0, d1 = a.shape[:2]
            pooled = F.max_pool2d(a.flatten(0, 1), 2, 2)
            x = pooled.view(d0, d1, *pooled.shape[1:])
        h = x.flatten(-3, -1)
        kl = 0.0
        for li in (2, 3, 4):
            W, b, _, _ = params_list[li]
            qW, qb = self._q(params_list[li])
            if li < 4:
                Ws, bs = qW.rsample((S,)), qb.rsample((S, 1))
            else:
                Ws, bs = qW.rsample(), qb.rsample()
            h = h.matmul(Ws.transpose(-2, -1)) + bs
            if li < 4:
                h = torch.relu(h)
            pW = D.Independent(D.Normal(torch.zeros_like(W), self.prior_sd), 2)
            pb = D.Independent(D.Normal(torch.zeros_like(b), self.prior_sd), 1)
            kl = kl + D.kl_divergence(qW, pW) + D.kl_divergence(qb, pb)
        torch.nn.LogSoftmax(dim=-1)(h).permute(1, 2, 0)  # computed, unused (psvi_classes.py:495)
        nll = -D.Categorical(logits=h).log_prob(z)
        return nll.matmul(w).sum() + kl


class _EpsReplay:
    def __init__(self, flat):
        self.flat = torch.as_tensor(flat)
        self.o = 0

    def __call__(self, shape, dtype, device):
        n = 1
        for s in shape:
            n *= s
        out = self.flat[self.o:self.o + n].reshape(shape).to(dtype=dtype, device=device)
        self.o += n
        return out


class _patched_normal:
    """Route Normal/MultivariateNormal rsample noise through a replay source."""

    def __init__(self, gen):
        self.gen = gen

    def __enter__(self):
        if self.gen is None:
            return
        import torch.distributions.multivariate_normal as mv
        import torch.distributions.normal as nm
        self.mods = (nm, mv)
        self.orig = (nm._standard_normal, mv._standard_normal)
        nm._standard_normal = self.gen
        mv._standard_normal = self.gen

    def __exit__(self, *a):
        if self.gen is None:
            return
        nm, mv = self.mods
        nm._standard_normal, mv._standard_normal = self.orig


def reference_init(family, layers, init_sd=1e-6, seed=0):
    """Parameter vector at the reference's initialisation: VILinear mu from
    nn.Linear's uniform(-1/sqrt(in), 1/sqrt(in)), rho = inv_softplus(init_sd);
    full-cov mean = 0, _sd = inv_softplus(init_sd), _corr = 0
    (neural_net.py:61-96, 408-431)."""
    g = torch.Generator().manual_seed(seed)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        if family == "mf":
            bound = 1.0 / math.sqrt(din)
            parts += [(torch.rand(n, generator=g) * 2 - 1) * bound,
                      torch.full((n,), _inv_softplus(init_sd))]
        else:
            parts += [torch.zeros(n), torch.full((n,), _inv_softplus(init_sd)),
                      torch.zeros((n - 1) * (n - 2) // 2)]
    return torch.cat(parts)
