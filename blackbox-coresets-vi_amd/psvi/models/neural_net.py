"""Variational layers: the model API of the reference's psvi/models/neural_net.py.

These modules are the parameter containers the inner loop runs on.  Their
parameter names, shapes, registration order and initialisation follow the
reference, so ``parameters_to_vector(model.parameters())`` is exactly the flat
vector the HIP library reads and updates:

  VILinear                    [weight (out,in), bias (out), _weight_sd, _bias_sd]
                              (neural_net.py:61-91, 176-179)
  VILinearMultivariateNormal  [mean (n), _sd (n), _corr ((n-1)(n-2)/2)],
                              n = out*in + out, _corr packed row-major strict
                              lower of the top-left (n-1)x(n-1) block
                              (neural_net.py:408-491)

Their torch ``forward`` / ``kl`` / ``sampled_nkl`` / ``rsample`` keep the
reference semantics for code that uses the modules directly (prediction,
the outer objective); the inner loop itself never calls them -- it runs in
libpsvi_hip (see psvi.inference.psvi_classes).  The full-covariance ``kl`` is
the closed form  n log s0 - sum log diag L + (|L|_F^2 + |mean|^2)/(2 s0^2) - n/2,
equal to torch's triangular-solve evaluation (neural_net.py:435-436) in O(n^2).
"""
import math

import numpy as np
import torch
import torch.distributions as dist
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "VIMixin", "VILinear", "MultivariateNormalVIMixin", "VILinearMultivariateNormal",
    "make_fcnet", "make_fc2net", "make_logreg", "set_mc_samples", "inverse_softplus",
    "categorical_fn", "gaussian_fn", "vi_layers", "model_spec",
    "VIConv2d", "BatchMaxPool2d", "make_lenet", "LENET_LAYERS",
]


def gaussian_fn(loc=None, scale=None):
    return dist.Normal(loc, scale)


def categorical_fn(logits=None, probs=None):
    return dist.Categorical(logits=logits, probs=probs)


def inverse_softplus(x):
    """log(exp(x) - 1) (neural_net.py:32-35)."""
    if torch.is_tensor(x):
        return x.expm1().log()
    return np.log(np.expm1(x))


def set_mc_samples(net, mc_samples):
    """Set the number of MC samples of every mean-field layer (neural_net.py:26-29:
    VIMixin modules only -- full-covariance layers keep theirs)."""
    for m in net.modules():
        if isinstance(m, VIMixin):
            m.mc_samples = mc_samples


# ------------------------------------------------------------ mean-field
class VIMixin(nn.Module):
    """Factorised Gaussian q(W) = N(weight, softplus(_weight_sd)^2) with prior
    N(0, prior_sd^2) (neural_net.py:61-173)."""

    def __init__(self, *args, init_sd=0.01, prior_sd=1.0, mc_samples=1, **kwargs):
        super().__init__(*args, **kwargs)
        self._weight_sd = nn.Parameter(inverse_softplus(torch.full_like(self.weight, init_sd)))
        if self.bias is not None:
            self._bias_sd = nn.Parameter(inverse_softplus(torch.full_like(self.bias, init_sd)))
        else:
            self.register_parameter("_bias_sd", None)
        self.prior_sd = prior_sd
        self.mc_samples = mc_samples
        self._init_sd = init_sd
        self._cached_weight = None
        self._cached_bias = None
        self.reset_parameters_variational()

    def reset_parameters_variational(self):
        super().reset_parameters()  # nn.Linear's init for the means
        with torch.no_grad():
            self._weight_sd.copy_(inverse_softplus(torch.full_like(self.weight, self._init_sd)))
            if self.bias is not None:
                self._bias_sd.copy_(inverse_softplus(torch.full_like(self.bias, self._init_sd)))
        self._cached_weight = self._cached_bias = None

    @property
    def weight_sd(self):
        return F.softplus(self._weight_sd)

    @property
    def bias_sd(self):
        return F.softplus(self._bias_sd) if self.bias is not None else None

    @property
    def weight_dist(self):
        return dist.Independent(dist.Normal(self.weight, self.weight_sd), self.weight.ndim)

    @property
    def prior_weight_dist(self):
        return dist.Independent(dist.Normal(torch.zeros_like(self.weight), self.prior_sd),
                                self.weight.ndim)

    @property
    def bias_dist(self):
        if self.bias is None:
            return None
        return dist.Independent(dist.Normal(self.bias, self.bias_sd), self.bias.ndim)

    @property
    def prior_bias_dist(self):
        if self.bias is None:
            return None
        return dist.Independent(dist.Normal(torch.zeros_like(self.bias), self.prior_sd),
                                self.bias.ndim)

    @property
    def weight_batch_shape(self):
        return torch.Size((self.mc_samples,) if self.mc_samples > 1 else ())

    @property
    def bias_batch_shape(self):
        return torch.Size((self.mc_samples, 1) if self.mc_samples > 1 else ())

    def rsample(self):
        w = self.weight_dist.rsample(self.weight_batch_shape)
        b = self.bias_dist.rsample(self.bias_batch_shape) if self.bias is not None else None
        return w, b

    def kl(self):
        """KL(q || prior), closed form (torch _kl_normal_normal)."""
        out = dist.kl_divergence(self.weight_dist, self.prior_weight_dist)
        if self.bias is not None:
            out = out + dist.kl_divergence(self.bias_dist, self.prior_bias_dist)
        return out

    def sampled_nkl(self):
        """log p(w_s) - log q(w_s) of the last forward's samples (neural_net.py:110-115)."""
        w = self._cached_weight
        out = self.prior_weight_dist.log_prob(w) - self.weight_dist.log_prob(w)
        if self.bias is not None:
            b = self._cached_bias.squeeze(1) if self.mc_samples > 1 else self._cached_bias
            out = out + self.prior_bias_dist.log_prob(b) - self.bias_dist.log_prob(b)
        return out

    def extra_repr(self):
        return f"{super().extra_repr()}, mc_samples={self.mc_samples}"


class VILinear(VIMixin, nn.Linear):
    """Mean-field Bayesian linear layer: x @ W_s^T + b_s per MC sample."""

    def forward(self, x):
        self._cached_weight, self._cached_bias = self.rsample()
        out = x.matmul(self._cached_weight.transpose(-2, -1))
        return out + self._cached_bias if self._cached_bias is not None else out


# -------------------------------------------------------- full covariance
class MultivariateNormalVIMixin(nn.Module):
    """Full-covariance Gaussian over all of a layer's weights (neural_net.py:408-482).

    The wrapped layer's own parameters are removed and replaced by
    ``mean``/``_sd``/``_corr``; each forward samples them per MC sample.
    """

    def __init__(self, *args, init_sd=0.01, prior_sd=1.0, mc_samples=1, **kwargs):
        super().__init__(*args, **kwargs)
        self.mc_samples = mc_samples
        self.prior_sd = prior_sd
        self.param_names, self.param_shapes = [], []
        proto = None
        for name, p in list(self.named_parameters()):
            self.param_names.append(name)
            self.param_shapes.append(p.shape)
            proto = p
            delattr(self, name)
        self.param_numels = [int(np.prod(s)) for s in self.param_shapes]
        n = sum(self.param_numels)
        self.num_params = n
        self.mean = nn.Parameter(proto.new_zeros(n))
        self._sd = nn.Parameter(inverse_softplus(proto.new_full((n,), init_sd)))
        self._corr = nn.Parameter(proto.new_zeros(max(n - 1, 0) * max(n - 2, 0) // 2))

    def reset_parameters_variational(self):
        raise NotImplementedError  # as in the reference

    @property
    def scale_tril(self):
        """Dense L = diag(softplus(_sd)) + _corr scattered into the strict lower
        triangle of the top-left (n-1)x(n-1) block (neural_net.py:452-461)."""
        n = self.num_params
        k = torch.diag_embed(F.softplus(self._sd))
        if n > 2:
            i = torch.tril_indices(n - 1, n - 1, offset=-1, device=self.mean.device)
            k = k.index_put((i[0], i[1]), self._corr, accumulate=True)
        return k

    @property
    def param_dist(self):
        return dist.MultivariateNormal(self.mean, scale_tril=self.scale_tril)

    @property
    def prior_dist(self):
        m = torch.zeros_like(self.mean)
        return dist.MultivariateNormal(m, scale_tril=torch.full_like(self.mean,
                                                                     self.prior_sd).diag_embed())

    def rsample(self):
        x = self.param_dist.rsample((self.mc_samples,))
        return [xx.reshape(self.mc_samples, *shape)
                for xx, shape in zip(x.split(self.param_numels, dim=-1), self.param_shapes)]

    def cached_rsample(self):
        for name, sample in zip(self.param_names, self.rsample()):
            setattr(self, name, sample)

    def kl(self):
        """KL(N(mean, LL^T) || N(0, s0^2 I)) in O(n^2)."""
        n, s0 = self.num_params, float(self.prior_sd)
        sp = F.softplus(self._sd)
        fro = (sp * sp).sum() + (self._corr * self._corr).sum()
        return (n * math.log(s0) - torch.log(sp).sum()
                + 0.5 * (fro + (self.mean * self.mean).sum()) / (s0 * s0) - 0.5 * n)

    def sampled_nkl(self):
        x = torch.cat([getattr(self, name).flatten(1) for name in self.param_names], dim=1)
        return self.prior_dist.log_prob(x) - self.param_dist.log_prob(x)


class VILinearMultivariateNormal(MultivariateNormalVIMixin, nn.Linear):
    def forward(self, x, **kwargs):
        self.cached_rsample()
        out = x.matmul(self.weight.transpose(-1, -2))
        if self.bias is not None:
            out = out + self.bias.unsqueeze(-2)
        return out


class VIConv2d(VIMixin, nn.Conv2d):
    """Mean-field Bayesian conv layer (neural_net.py:194-246): S weight samples,
    each convolving its own copy of the input (one grouped conv with
    groups=S).  Input (M, C, H, W) or (S, M, C, H, W); output (S, M, K, H', W')
    when mc_samples > 1."""

    def __init__(self, *args, **kwargs):
        if "groups" in kwargs:
            raise ValueError("groups is reserved: it parallelises the conv over samples")
        super().__init__(*args, **kwargs)

    def forward(self, x):
        S = self.mc_samples
        if S > 1:
            x = x.repeat(1, S, 1, 1) if x.ndim == 4 else x.transpose(0, 1).flatten(1, 2)
        self._cached_weight, self._cached_bias = self.rsample()
        wt = self._cached_weight.flatten(0, 1) if S > 1 else self._cached_weight
        b = self._cached_bias.flatten() if self.bias is not None else None
        a = F.conv2d(x, wt, b, stride=self.stride, padding=self.padding,
                     dilation=self.dilation, groups=S)
        if S > 1:
            return a.view(-1, S, self.out_channels, *a.shape[-2:]).transpose(0, 1)
        return a


class BatchMaxPool2d(nn.MaxPool2d):
    """Max-pool over the trailing (C, H, W) of an (S, M, C, H, W) map
    (neural_net.py:249-255; its ``x.shape == 4`` guard is never true, so 5-d
    input always takes the flattening path -- kept)."""

    def forward(self, x):
        d0, d1 = x.shape[:2]
        x = super().forward(x.flatten(0, 1))
        return x.view(d0, d1, *x.shape[1:])


def make_lenet(conv_class=None, linear_class=None, pool_class=None, nonl_class=None, **kwargs):
    """LeNet-5 BNN (neural_net.py:334-359).  kwargs (mc_samples, init_sd,
    prior_sd) go to every layer but the last, which keeps the VILinear defaults:
    mc_samples=1 (one weight sample shared by all S) and init_sd=0.01."""
    conv_class = conv_class or VIConv2d
    linear_class = linear_class or VILinear
    pool_class = pool_class or BatchMaxPool2d
    nonl_class = nonl_class or nn.ReLU
    return nn.Sequential(
        conv_class(1, 6, 5, padding=2, **kwargs), nonl_class(), pool_class(2, 2),
        conv_class(6, 16, 5, padding=0, **kwargs), nonl_class(), pool_class(2, 2),
        nn.Flatten(-3, -1),
        linear_class(400, 120, **kwargs), nonl_class(),
        linear_class(120, 84, **kwargs), nonl_class(),
        linear_class(84, 10))


# (weight elements / out channels, out) of make_lenet's variational layers as
# the HIP library lays them out (n = in*out + out per layer)
LENET_LAYERS = [(25, 6), (150, 16), (400, 120), (120, 84), (84, 10)]


# ------------------------------------------------------------ builders
def _stack(in_dim, h_dim, out_dim, n_layers, linear_class, nonl_class, mc_samples, kwargs):
    net = nn.Sequential()
    for i in range(n_layers):
        net.add_module(f"lin{i}", linear_class(in_dim if i == 0 else h_dim, h_dim, **kwargs))
        net.add_module(f"nonl{i}", nonl_class())
    net.add_module("classifier", linear_class(h_dim if n_layers else in_dim, out_dim, **kwargs))
    for m in net.modules():
        m.mc_samples = mc_samples
    return net


def make_fcnet(in_dim, h_dim, out_dim, n_layers=2, linear_class=None, nonl_class=None,
               mc_samples=4, residual=False, **kwargs):
    """Mean-field MLP ('fn' architecture, neural_net.py:267-297)."""
    if residual:
        raise NotImplementedError("residual_fn is commented out in the reference builder too")
    return _stack(in_dim, h_dim, out_dim, n_layers, linear_class or VILinear,
                  nonl_class or nn.ReLU, mc_samples, kwargs)


def make_fc2net(in_dim, h_dim, out_dim, n_layers=2, linear_class=None, nonl_class=None,
                mc_samples=4, residual=False, **kwargs):
    """Full-covariance MLP ('fn2' architecture, neural_net.py:494-525)."""
    if residual:
        raise NotImplementedError("residual_fn is commented out in the reference builder too")
    return _stack(in_dim, h_dim, out_dim, n_layers, linear_class or VILinearMultivariateNormal,
                  nonl_class or nn.ReLU, mc_samples, kwargs)


def make_logreg(in_dim, out_dim, fullcov=False, mc_samples=4, **kwargs):
    """'logistic_regression' / 'logistic_regression_fullcov' (psvi_classes.py:693-705)."""
    cls = VILinearMultivariateNormal if fullcov else VILinear
    net = nn.Sequential(cls(in_dim, out_dim, mc_samples=mc_samples, **kwargs))
    set_mc_samples(net, mc_samples)
    return net


# --------------------------------------------- inner-loop (HIP) model spec
def vi_layers(model):
    return [m for m in model.modules() if isinstance(m, (VIMixin, MultivariateNormalVIMixin))]


def _lenet_spec(mods):
    """("lenet", LENET_LAYERS, prior_sd, S) for make_lenet's exact stack."""
    kinds = [VIConv2d, nn.ReLU, BatchMaxPool2d, VIConv2d, nn.ReLU, BatchMaxPool2d, nn.Flatten,
             VILinear, nn.ReLU, VILinear, nn.ReLU, VILinear]
    if len(mods) != len(kinds) or not all(isinstance(m, k) for m, k in zip(mods, kinds)):
        raise ValueError("only make_lenet's exact stack runs on the HIP LeNet path")
    c1, c2, f1, f2, f3 = mods[0], mods[3], mods[7], mods[9], mods[11]
    for c, (ci, co, pad) in ((c1, (1, 6, 2)), (c2, (6, 16, 0))):
        if (c.in_channels, c.out_channels, c.kernel_size, c.padding, c.stride, c.dilation) != \
                (ci, co, (5, 5), (pad, pad), (1, 1), (1, 1)) or c.bias is None:
            raise ValueError("LeNet conv layers must be make_lenet's (5x5, stride 1, bias)")
    for p in (mods[2], mods[5]):
        if p.kernel_size not in (2, (2, 2)) or p.stride not in (2, (2, 2)) or \
                p.padding not in (0, (0, 0)) or p.dilation not in (1, (1, 1)) or p.ceil_mode:
            raise ValueError("LeNet pools must be 2x2 / stride 2")
    if (mods[6].start_dim, mods[6].end_dim) != (-3, -1):
        raise ValueError("LeNet flatten must be Flatten(-3, -1)")
    for f, (i, o) in ((f1, (400, 120)), (f2, (120, 84)), (f3, (84, 10))):
        if (f.in_features, f.out_features) != (i, o) or f.bias is None:
            raise ValueError("LeNet linear layers must be 400-120-84-10 with bias")
    S = int(c1.mc_samples)
    if any(int(m.mc_samples) != S for m in (c2, f1, f2)) or S < 2:
        raise ValueError("LeNet: the convs and the first two linears share mc_samples > 1")
    if int(f3.mc_samples) != 1:
        raise ValueError("LeNet: the last layer keeps one shared sample (mc_samples=1)")
    prior = float(c1.prior_sd)
    if any(float(m.prior_sd) != prior for m in (c2, f1, f2, f3)):
        raise ValueError("all layers must share prior_sd")
    return "lenet", list(LENET_LAYERS), prior, S


def model_spec(model):
    """(family, [(in, out), ...], prior_sd, mc_samples) of a model the HIP inner
    loop can run: an nn.Sequential of variational linear layers of one family
    with ReLU between them, or make_lenet's stack (family "lenet").  Raises
    ValueError otherwise.  A functional view (psvi.robust_higher's fmodel)
    reports the spec of the module it wraps."""
    model = getattr(model, "_psvi_module", model)
    if not isinstance(model, nn.Sequential):
        raise ValueError("the HIP inner loop runs nn.Sequential VI stacks (make_fcnet / "
                         "make_fc2net / make_logreg / make_lenet)")
    mods = list(model.children())
    if mods and isinstance(mods[0], VIConv2d):
        return _lenet_spec(mods)
    layers, fam, prior, S = [], None, None, None
    for i, m in enumerate(mods):
        if i % 2 == 1:
            if not isinstance(m, nn.ReLU):
                raise ValueError(f"module {i}: only ReLU between variational layers")
            continue
        if isinstance(m, VILinear):
            f = "meanfield"
            if m.bias is None:
                raise ValueError("VILinear without bias is not supported")
        elif isinstance(m, VILinearMultivariateNormal):
            f = "fullcov"
            if "bias" not in m.param_names:
                raise ValueError("VILinearMultivariateNormal without bias is not supported")
        else:
            raise ValueError(f"module {i} ({type(m).__name__}) is not a variational linear layer")
        if fam is not None and f != fam:
            raise ValueError("mixed mean-field / full-covariance stacks are not supported")
        fam = f
        if prior is not None and float(m.prior_sd) != prior:
            raise ValueError("all layers must share prior_sd")
        prior = float(m.prior_sd)
        if S is not None and m.mc_samples != S:
            raise ValueError("all layers must share mc_samples")
        S = int(m.mc_samples)
        layers.append((m.in_features, m.out_features))
    if not layers or len(mods) % 2 == 0:
        raise ValueError("the stack must end with a variational layer")
    return fam, layers, prior, S
