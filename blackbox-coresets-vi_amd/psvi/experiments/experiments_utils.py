"""Datasets and results files of psvi/experiments/experiments_utils.py and
flow_psvi.py, for the datasets that need no download (halfmoon, four_blobs,
synth_lr_<D>, normal_mvn, and the MNIST-shaped synthetic set of config C5).
The UCI / LIBSVM / torchvision loaders fetch remote files and are refused
here (no network): read_dataset raises for them."""
import json
import os
import pickle
from collections import defaultdict

import numpy as np
import torch
from torch.utils.data import Dataset

__all__ = ["SynthDataset", "split_data", "make_four_class_dataset", "make_synthetic",
           "make_synthetic_normal", "make_mnist_shaped", "read_dataset", "rec_dd",
           "write_to_files"]


class SynthDataset(Dataset):
    """experiments_utils.py:81-105: (data, targets) tensors as a Dataset."""

    def __init__(self, x, y=None, transforms=None):
        self.data = x
        self.targets = y
        self.transforms = transforms

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        return self.data[index], self.targets[index]

    def subset_where(self, cs=(0, 1)):
        keep = torch.isin(self.targets, torch.tensor(list(cs)))
        return SynthDataset(self.data[keep], self.targets[keep])

    def concatenate(self, u, z):
        return SynthDataset(torch.cat((self.data, u)), y=torch.cat((self.targets, z)))


def split_data(N, p_split=(0.6, 0.2, 0.2), n_split=None, shuffle=True, seed=None):
    """experiments_utils.py:107-141: index split into train / val / test."""
    if seed is not None:
        np.random.seed(seed)
    if n_split is None:
        p = np.array(p_split, dtype=np.float64)
        assert np.sum(p == -1) <= 1
        p[p == -1] = 1 - (np.sum(p) + 1)
        assert np.sum(p) == 1.0
        train_idx = int(np.ceil(p[0] * N))
        val_idx = int(np.ceil(train_idx + p[1] * N))
    else:
        n = np.array(n_split)
        assert np.sum(n == -1) <= 1
        n[n == -1] = N - (np.sum(n) + 1)
        assert np.sum(n) == N
        train_idx = int(n[0])
        val_idx = int(train_idx + n[1])
    idx = np.arange(N)
    if shuffle:
        np.random.shuffle(idx)
    return {"train": idx[:train_idx], "val": idx[train_idx:val_idx], "test": idx[val_idx:]}


def make_four_class_dataset(N_K=250):
    """experiments_utils.py:299-343: four 2-d Gaussian blobs (torch RNG),
    shifted, rows shuffled."""
    X1 = torch.cat([0.8 + 0.4 * torch.randn(N_K, 1), 1.5 + 0.4 * torch.randn(N_K, 1)], dim=-1)
    X2 = torch.cat([0.5 + 0.6 * torch.randn(N_K, 1), -0.2 - 0.1 * torch.randn(N_K, 1)], dim=-1)
    X3 = torch.cat([2.5 - 0.1 * torch.randn(N_K, 1), 1.0 + 0.6 * torch.randn(N_K, 1)], dim=-1)
    X4 = torch.distributions.MultivariateNormal(
        torch.Tensor([-0.5, 1.5]),
        covariance_matrix=torch.Tensor([[0.2, 0.1], [0.1, 0.1]])).sample(torch.Size([N_K]))
    X = torch.cat([X1, X2, X3, X4], dim=0)
    X[:, 1] -= 1
    X[:, 0] -= 0.5
    Y = torch.cat([c * torch.ones(N_K).long() for c in range(4)])
    perm = torch.randperm(X.size()[0])
    return X[perm, :], Y[perm]


def make_synthetic(num_datapoints=1000, D=2):
    """experiments_utils.py:666-677: X ~ N(0, I_D), y ~ Bernoulli(sigmoid(5 sum x))
    in {-1, 1} (numpy RNG)."""
    X = np.random.multivariate_normal(np.zeros(D, dtype=int), np.eye(D), num_datapoints)
    ps = 1.0 / (1.0 + np.exp(-(X * np.full(D, 5)).sum(axis=1)))
    y = (np.random.rand(num_datapoints) <= ps).astype(int)
    y[y == 0] = -1
    return torch.from_numpy(X.astype(np.float32)), torch.from_numpy(y.astype(np.float32))


def make_synthetic_normal(num_datapoints=1000):
    """experiments_utils.py:679-702: two correlated Gaussians (seed 43), {-1, 1}."""
    np.random.seed(43)
    cov = 8.0 * np.eye(2)
    cov[0, 1] = cov[1, 0] = 2.5
    pts_1 = np.random.multivariate_normal(np.array([-1, 1]), cov, num_datapoints)
    pts_2 = np.random.multivariate_normal(np.array([1, -1]), cov, num_datapoints)
    X = np.vstack((pts_1, pts_2))
    y = np.concatenate([np.zeros(num_datapoints), np.ones(num_datapoints)])
    y[y == 0] = -1
    idx = np.random.permutation(X.shape[0])
    return torch.from_numpy(X[idx].astype(np.float32)), torch.from_numpy(y[idx].astype(np.float32))


def make_mnist_shaped(n_train=60000, n_test=10000, seed=0):
    """The C5 workload's stand-in for MNIST (no download): images ~ N(0, 1) of
    shape (1, 28, 28), labels uniform over 10 classes."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n_train, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (n_train,), generator=g).float()
    xt = torch.randn(n_test, 1, 28, 28, generator=g)
    yt = torch.randint(0, 10, (n_test,), generator=g).float()
    return x, y, xt, yt


def read_dataset(dnm, method_args):
    """experiments_utils.py:752-836 for the offline datasets; returns
    (x, y, xt, yt, N, D, train_dataset, test_dataset, num_classes).  The last
    test_ratio of the rows is the test split; labels -1 become 0."""
    if dnm == "mnist_shaped":
        x, y, xt, yt = make_mnist_shaped(seed=method_args.get("seed", 0))
        return (None, None, None, None, x.shape[0], 28, SynthDataset(x, y),
                SynthDataset(xt, yt), 10)
    if dnm == "halfmoon":
        from sklearn.datasets import make_moons

        X, Y = make_moons(n_samples=1000, noise=0.1, random_state=42)
        X, Y, nc = torch.from_numpy(X.astype(np.float32)), torch.from_numpy(Y.astype(np.float32)), 2
    elif dnm == "four_blobs":
        (X, Y), nc = make_four_class_dataset(N_K=250), 4
    elif dnm.startswith("synth_lr"):
        (X, Y), nc = make_synthetic(D=int(dnm.split("_")[-1]), num_datapoints=1000), 2
    elif dnm == "normal_mvn":
        (X, Y), nc = make_synthetic_normal(num_datapoints=1000), 2
    else:
        raise NotImplementedError(f"dataset {dnm!r} is a remote download (UCI / LIBSVM / "
                                  "torchvision): not available offline")
    Y[Y == -1] = 0
    test_size = int(method_args["test_ratio"] * X.shape[0])
    x, y, xt, yt = X[:-test_size], Y[:-test_size], X[-test_size:], Y[-test_size:]
    N, D = x.shape
    return x, y, xt, yt, N, D, SynthDataset(x, y), SynthDataset(xt, yt), nc


def rec_dd():
    """flow_psvi.py:299-300: the recursive results dict
    results[dataset][method][coreset size][trial] = run's results."""
    return defaultdict(rec_dd)


def _plain(obj):
    if isinstance(obj, dict):
        return {str(k): _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    if torch.is_tensor(obj):
        return obj.detach().cpu().tolist()
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, (np.floating, np.integer)):
        return obj.item()
    return obj


def write_to_files(results, fnm, results_folder="results"):
    """flow_psvi.py:552-564: <fnm>.pk (pickle of the results dict) and
    <fnm>.json.  Tensors are converted to lists first (the reference's
    json.dump fails on them after writing the pickle)."""
    os.makedirs(results_folder, exist_ok=True)
    plain = _plain(results)
    with open(os.path.join(results_folder, f"{fnm}.pk"), "wb") as f:
        pickle.dump(plain, f)
    with open(os.path.join(results_folder, f"{fnm}.json"), "w") as f:
        json.dump(plain, f)
    return plain
