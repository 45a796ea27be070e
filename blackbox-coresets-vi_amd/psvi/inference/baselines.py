"""Mean-field VI baselines of the reference's psvi/inference/baselines.py on the
HIP inner-step kernels:

  run_mfvi         baselines.py:824-914   VI on data minibatches (weights N/B)
  run_mfvi_subset  baselines.py:917-1062  VI on a fixed random subset (weights N/M)

Each iteration is the inner ELBO of the HIP library with uniform coreset
weights -- psvi_elbo_grad on the batch, then torch.optim.Adam's update
(PSVI_ADAM_TORCH, psvi_adam_update) -- with the reference's quirks kept: the
loss sums the NLL over the S samples too, and its KL term sums over
``VILinear`` modules only (baselines.py:889, 1033), so a full-covariance stack
trains without KL.  The predictive evaluation every ``log_every`` iterations
averages the LOGITS over samples (baselines.py:898-906) and runs the model's
torch forward on the device (not the hot path).  There is no CPU fallback:
the training step raises without the HIP library or a device.
"""
import random
import time

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from ..models import (VILinear, VILinearMultivariateNormal, categorical_fn, make_fc2net,
                      make_fcnet, make_lenet, model_spec)
from ..runtime import InnerLoopPlan, adam_update_, randn_

__all__ = ["set_up_model", "pseudo_subsample_init", "pseudo_rand_init", "run_mfvi",
           "run_mfvi_subset"]


def set_up_model(D=None, n_hidden=None, nc=None, mc_samples=None, architecture=None,
                 **kwargs):
    """experiments_utils.set_up_model (psvi/experiments/experiments_utils.py:346-413)
    for the architectures the HIP path runs.  As there, kwargs (init_sd) reach
    fn / fn2 only; lenet and the logistic regressions take their defaults."""
    if architecture == "fn":
        return make_fcnet(D, n_hidden, nc, linear_class=VILinear, nonl_class=nn.ReLU,
                          mc_samples=mc_samples, **kwargs)
    if architecture == "fn2":
        return make_fc2net(D, n_hidden, nc, linear_class=VILinearMultivariateNormal,
                           nonl_class=nn.ReLU, mc_samples=mc_samples, **kwargs)
    if architecture == "lenet":
        return make_lenet(linear_class=VILinear, nonl_class=nn.ReLU, mc_samples=mc_samples)
    if architecture == "logistic_regression":
        return nn.Sequential(VILinear(D, nc, mc_samples=mc_samples))
    if architecture == "logistic_regression_fullcov":
        return nn.Sequential(VILinearMultivariateNormal(D, nc, mc_samples=mc_samples))
    raise NotImplementedError(f"architecture {architecture!r} is not on the HIP path "
                              "(residual_fn / regressor_net / alexnet / resnet)")


def pseudo_subsample_init(x, y, num_pseudo=20, nc=2, seed=0):
    """psvi/inference/utils.py:33-50: a random subset with num_pseudo // nc points
    per class (the remainder on the last class)."""
    torch.manual_seed(seed)
    N = x.shape[0]
    cnt = 0
    u, z = torch.Tensor([]), torch.Tensor([])
    for c in range(nc):
        idx_c = torch.arange(N)[y == c]
        k = num_pseudo // nc if c < nc - 1 else num_pseudo - cnt
        u = torch.cat((u, x[idx_c[torch.randperm(len(idx_c))[:k]]]))
        z = torch.cat((z, c * torch.ones(k)))
        cnt += num_pseudo // nc
    return u.requires_grad_(True), z


def pseudo_rand_init(x, y, num_pseudo=20, nc=2, seed=0, variance=0.1):
    """psvi/inference/utils.py:53-77: noisy data mean, labels split over classes."""
    torch.manual_seed(seed)
    D = x.shape[1]
    u = (x[:, :].mean() + variance * torch.randn(num_pseudo, D)).clone().requires_grad_(True)
    z = torch.Tensor([])
    for c in range(nc):
        k = num_pseudo // nc if c < nc - 1 else num_pseudo - (nc - 1) * (num_pseudo // nc)
        z = torch.cat((z, c * torch.ones(k)))
    return u, z


class _MFVIStepper:
    """One MFVI iteration on the HIP library for a fixed model: plans cached per
    batch size, parameters and torch-Adam state resident on the device."""

    def __init__(self, net, device, lr, seed, eps_source=None):
        self.net = net
        self.fam, self.layers, self.prior_sd, self.S = model_spec(net)
        self.device = device
        self.lr = float(lr)
        self.plist = list(net.parameters())
        with torch.no_grad():
            self.params = nn.utils.parameters_to_vector(self.plist).detach().to(
                device, torch.float32).clone()
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.t = 0
        self.plans = {}
        self.eps_source = eps_source
        self.seed, self.offset = int(seed), 0

    def _plan(self, B):
        if B not in self.plans:
            self.plans[B] = InnerLoopPlan(self.fam, self.layers, self.S, B,
                                          prior_sd=self.prior_sd)
        return self.plans[B]

    def step(self, xb, yb, scale):
        """loss = scale * sum_{s,b} NLL + KL (VILinear modules) and one
        torch.optim.Adam step; returns the loss (device float64)."""
        B = int(xb.shape[0])
        plan = self._plan(B)
        u = xb.detach().to(self.device, torch.float32).reshape(B, -1).contiguous()
        z = yb.detach().to(self.device)
        if z.is_floating_point() and not torch.equal(z, z.round()):
            raise ValueError("labels must hold class ids")
        z = z.to(torch.int32).contiguous()
        w = torch.full((B,), float(scale), device=self.device)
        if self.eps_source is not None:
            eps = self.eps_source(plan.eps_count).to(self.device, torch.float32).contiguous()
        else:
            eps = torch.empty(plan.eps_count, device=self.device)
            randn_(eps, self.seed, self.offset)
            self.offset += plan.eps_stride
        loss, grad = plan.elbo_grad(u, z, w, eps, self.params,
                                    include_kl=self.fam != "fullcov")
        self.t += 1
        adam_update_(self.params, grad, self.m, self.v, step=self.t, lr=self.lr, kind="torch")
        return loss

    def sync_model(self):
        with torch.no_grad():
            nn.utils.vector_to_parameters(self.params.to(self.plist[0].dtype), self.plist)


def _evaluate(net, test_loader, device, distr_fn):
    """Mean-logit predictive (baselines.py:892-906): accuracy and mean NLL."""
    total, test_nll, corrects = 0, 0.0, 0.0
    with torch.no_grad():
        for xt, yt in test_loader:
            xt, yt = xt.to(device, non_blocking=True), yt.to(device, non_blocking=True)
            logits = net(xt).squeeze(-1).mean(0)
            corrects += logits.argmax(-1).float().eq(yt).float().sum()
            total += yt.size(0)
            test_nll += -distr_fn(logits=logits).log_prob(yt).sum()
    return float(corrects / float(total)), float(test_nll / float(total))


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("the MFVI baselines run on the HIP library: no HIP device")
    return torch.device("cuda")


def run_mfvi(xt=None, yt=None, mc_samples=4, data_minibatch=128, num_epochs=100, log_every=10,
             N=None, D=None, lr0net=1e-3, mul_fact=2, seed=0, distr_fn=categorical_fn,
             architecture=None, n_hidden=None, nc=2, log_pseudodata=False,
             train_dataset=None, test_dataset=None, init_sd=None, eps_source=None, **kwargs):
    """Mean-field VI on the full training set (baselines.py:824-914): each
    iteration draws a fresh shuffled minibatch, loss = N/B * sum NLL + KL.
    Returns the reference's results dict {accs, nlls, times, elbos, csizes}.
    ``eps_source(n)`` (optional) supplies each training step's noise in the
    library's eps layout; default: the library's Philox stream."""
    if log_pseudodata:
        raise NotImplementedError("log_pseudodata (grid predictions) is not on the HIP path")
    device = _device()
    random.seed(seed), np.random.seed(seed), torch.manual_seed(seed)
    nlls, accs, times, elbos = [], [], [0], []
    t_start = time.time()
    net = set_up_model(architecture=architecture, D=D, n_hidden=n_hidden, nc=nc,
                       mc_samples=mc_samples, init_sd=init_sd).to(device)
    train_loader = DataLoader(train_dataset, batch_size=data_minibatch, pin_memory=True,
                              shuffle=True)
    n_train = len(train_loader.dataset)
    test_loader = DataLoader(test_dataset, batch_size=data_minibatch, pin_memory=True,
                             shuffle=True)
    stepper = _MFVIStepper(net, device, lr0net, seed, eps_source)
    total_iterations = mul_fact * num_epochs
    for i in range(total_iterations):
        xbatch, ybatch = next(iter(train_loader))
        loss = stepper.step(xbatch, ybatch, n_train / xbatch.shape[0])
        elbos.append(-loss.item())
        if i % log_every == 0 or i == total_iterations - 1:
            stepper.sync_model()
            a, n = _evaluate(net, test_loader, device, distr_fn)
            times.append(times[-1] + time.time() - t_start)
            accs.append(a)
            nlls.append(n)
    stepper.sync_model()
    return {"accs": accs, "nlls": nlls, "times": times[1:], "elbos": elbos, "csizes": None}


def run_mfvi_subset(x=None, y=None, xt=None, yt=None, mc_samples=4, data_minibatch=128,
                    num_epochs=100, log_every=10, D=None, lr0net=1e-3, mul_fact=2, seed=0,
                    distr_fn=categorical_fn, log_pseudodata=False, train_dataset=None,
                    test_dataset=None, num_pseudo=100, init_args="subsample", architecture=None,
                    n_hidden=None, nc=2, dnm=None, init_sd=None, eps_source=None, **kwargs):
    """Mean-field VI on a fixed random subset of num_pseudo training points
    (baselines.py:917-1062), loss = N/num_pseudo * sum NLL + KL.  The MNIST
    per-class loader branch (dnm="MNIST") needs torchvision datasets and is not
    supported; the subset comes from pseudo_subsample_init / pseudo_rand_init."""
    if log_pseudodata:
        raise NotImplementedError("log_pseudodata (grid predictions) is not on the HIP path")
    if dnm == "MNIST":
        raise NotImplementedError("the torchvision MNIST subset loader is not available")
    device = _device()
    random.seed(seed), np.random.seed(seed), torch.manual_seed(seed)
    nlls, accs, times, elbos = [], [], [0], []
    t_start = time.time()
    net = set_up_model(architecture=architecture, D=D, n_hidden=n_hidden, nc=nc,
                       mc_samples=mc_samples, init_sd=init_sd).to(device)
    init = pseudo_rand_init if init_args == "random" else pseudo_subsample_init
    xbatch, ybatch = init(x, y, num_pseudo=num_pseudo, seed=seed, nc=nc)
    n_train = len(train_dataset)
    test_loader = DataLoader(test_dataset, batch_size=data_minibatch, pin_memory=True,
                             shuffle=True)
    stepper = _MFVIStepper(net, device, lr0net, seed, eps_source)
    sum_scaling = n_train / num_pseudo
    for i in range(mul_fact * num_epochs):
        loss = stepper.step(xbatch, ybatch, sum_scaling)
        elbos.append(-loss.item())
        if i % log_every == 0:
            stepper.sync_model()
            a, n = _evaluate(net, test_loader, device, distr_fn)
            times.append(times[-1] + time.time() - t_start)
            accs.append(a)
            nlls.append(n)
    stepper.sync_model()
    return {"accs": accs, "nlls": nlls, "times": times[1:], "elbos": elbos,
            "csizes": [num_pseudo] * (mul_fact * num_epochs)}
