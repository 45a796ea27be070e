"""The experiment driver's entry point on the HIP trainers: called exactly as
flow_psvi.py's inf_dict does (psvi/experiments/flow_psvi.py:306-354, 401-454):
Class(**kwargs).run_psvi(**kwargs) on a halfmoon-shaped dataset."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _DS(torch.utils.data.Dataset):
    """x / y tensors with the .data / .targets attributes the reference's
    datasets carry (experiments_utils.py:81-105)."""

    def __init__(self, x, y):
        self.data, self.targets = x, y

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        return self.data[i], self.targets[i]


def halfmoon():
    from sklearn.datasets import make_moons

    X, Y = make_moons(1000, noise=0.1, random_state=42)  # experiments_utils.py:759-767
    X, Y = torch.tensor(X, dtype=torch.float32), torch.tensor(Y, dtype=torch.float32)
    return _DS(X[:800], Y[:800]), _DS(X[800:], Y[800:])


def flow_kwargs(**over):
    tr, te = halfmoon()
    kw = dict(mc_samples=4, num_epochs=4, data_minibatch=128, D=2, N=800, tr=0, diagonal=None,
              x=tr.data, y=tr.targets, xt=te.data, yt=te.targets, inner_it=3, outer_it=100,
              scatterplot_coreset=None, logistic_regression=False, trainer="nested", log_every=2,
              register_elbos=True, lr0u=1e-4, lr0net=1e-3, lr0v=1e-3, lr0z=1e-3, lr0alpha=1e-3,
              init_args="subsample", init_sd=1e-6, num_pseudo=10, seed=0,
              compute_weights_entropy=True, reset=None, reset_interval=None,
              architecture="fn2", log_pseudodata=True, n_hidden=8, n_layers=1,
              train_dataset=tr, test_dataset=te, dnm="halfmoon", nc=2, prune=None,
              prune_interval=None, prune_sizes=None, increment=None, increment_interval=None,
              increment_sizes=None, retrain_on_coreset=None, learn_z=False, device_id=0)
    kw.update(over)
    return kw


@pytest.mark.parametrize("trainer,arch,cls", [
    ("nested", "fn2", "PSVILearnV"),
    ("hyper", "fn2", "PSVILearnV"),
    ("joint", "fn", "PSVIAV"),
    ("alternating", "logistic_regression_fullcov", "PSVILearnV"),
    ("nested", "logistic_regression", "PSVI"),
])
def test_run_psvi_like_flow_psvi(trainer, arch, cls):
    import psvi.inference as I

    kw = flow_kwargs(trainer=trainer, architecture=arch,
                     logistic_regression=arch == "logistic_regression")
    torch.manual_seed(0)
    res = getattr(I, cls)(**kw).run_psvi(**kw)
    n_log = len(range(0, kw["num_epochs"], kw["log_every"]))
    for key in ("accs", "nlls", "csizes", "times", "elbos", "went", "ness", "vent", "vs",
                "avg_epoch_time", "gpu_memory", "chosen_indices", "us", "zs", "grid_preds"):
        assert key in res, key
    assert len(res["accs"]) == len(res["nlls"]) == n_log
    assert all(0.0 <= a <= 1.0 for a in res["accs"])
    assert all(math.isfinite(x) for x in res["nlls"])
    assert res["csizes"] == [10] * n_log
    assert res["grid_preds"][0].shape == (2, 250 * 250)
    assert np.asarray(res["us"][0]).shape == (10, 2)


@pytest.mark.parametrize("trainer", ["joint", "alternating", "hyper", "nested"])
def test_run_psvi_lenet_trainers(trainer):
    """make_lenet through run_psvi on an MNIST-shaped synthetic set with every
    trainer: psvi_elbo, evaluate, and for hyper / nested the LeNet HVP (C5's
    bilevel outer) on the LeNet kernels."""
    import psvi.inference as I
    from psvi.experiments import make_mnist_shaped

    x, y, xt, yt = make_mnist_shaped(n_train=256, n_test=64, seed=1)
    tr, te = _DS(x, y), _DS(xt, yt)
    kw = flow_kwargs(trainer=trainer, architecture="lenet", logistic_regression=False,
                     D=28, N=256, x=None, y=None, xt=None, yt=None, train_dataset=tr,
                     test_dataset=te, nc=10, num_pseudo=10, mc_samples=3, data_minibatch=32,
                     log_pseudodata=False, init_sd=0.05, dnm="mnist_shaped")
    torch.manual_seed(0)
    res = I.PSVILearnV(**kw).run_psvi(**kw)
    assert len(res["accs"]) == 2 and all(math.isfinite(x) for x in res["nlls"])
