"""Data / results plumbing (psvi.experiments): the offline
datasets equal the reference's read_dataset output (tests/golden/d1_datasets.npz
from tools/gen_golden_data.py); the results dict round-trips through its files."""
import json
import os
import pickle

import numpy as np
import pytest
import torch

from golden_util import GOLDEN


@pytest.mark.parametrize("dnm,seed", [("halfmoon", None), ("four_blobs", 0),
                                      ("synth_lr_5", 0), ("normal_mvn", None)])
def test_read_dataset_matches_reference(dnm, seed):
    from psvi.experiments import read_dataset

    g = np.load(os.path.join(GOLDEN, "d1_datasets.npz"))
    if seed is not None:
        torch.manual_seed(seed)
        np.random.seed(seed)
    x, y, xt, yt, N, D, tr, te, nc = read_dataset(dnm, {"test_ratio": 0.2})
    for k, v in (("x", x), ("y", y), ("xt", xt), ("yt", yt)):
        assert np.array_equal(v.numpy(), g[f"{dnm}_{k}"]), (dnm, k)
    assert [N, D, nc] == list(g[f"{dnm}_meta"])
    assert len(tr) == N and len(te) == xt.shape[0] and tr[3][1] == y[3]


def test_offline_only_datasets():
    from psvi.experiments import read_dataset

    with pytest.raises(NotImplementedError, match="offline"):
        read_dataset("phishing", {"test_ratio": 0.2})
    x, y, xt, yt, N, D, tr, te, nc = read_dataset("mnist_shaped", {})
    assert (N, D, nc) == (60000, 28, 10) and tr[0][0].shape == (1, 28, 28)


def test_split_data_partitions():
    from psvi.experiments import split_data

    s = split_data(100, seed=1)
    idx = np.concatenate([s["train"], s["val"], s["test"]])
    assert sorted(idx.tolist()) == list(range(100)) and len(s["train"]) == 60


def test_results_dict_files(tmp_path):
    from psvi.experiments import rec_dd, write_to_files

    r = rec_dd()
    r["halfmoon"]["mfvi"][-1][0] = {"accs": [0.5, torch.tensor(0.75)], "elbos": np.arange(3.0)}
    plain = write_to_files(r, "res", str(tmp_path))
    with open(tmp_path / "res.pk", "rb") as f:  # our own file
        back = pickle.load(f)
    assert back == plain == json.load(open(tmp_path / "res.json"))
    assert back["halfmoon"]["mfvi"]["-1"]["0"]["accs"] == [0.5, 0.75]
