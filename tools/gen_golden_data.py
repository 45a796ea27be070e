#!/usr/bin/env python3
"""Golden datasets for the data plumbing: the
reference's own read_dataset (psvi/experiments/experiments_utils.py:752-836)
for the offline datasets -- halfmoon, four_blobs (torch seed 0), synth_lr_5
(numpy seed 0), normal_mvn -- with test_ratio 0.2.  Runs only in the
development container (child interpreter with the reference on sys.path, like
tools/gen_golden.py); writes tests/golden/d1_datasets.npz (arrays only)."""
import os
import subprocess
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _child():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gen_golden import _install_stubs

    _install_stubs()
    import numpy as np
    import torch

    from psvi.experiments.experiments_utils import read_dataset

    out = {}
    for dnm, seed in (("halfmoon", None), ("four_blobs", 0), ("synth_lr_5", 0),
                      ("normal_mvn", None)):
        if seed is not None:
            torch.manual_seed(seed)
            np.random.seed(seed)
        x, y, xt, yt, N, D, tr, te, nc = read_dataset(dnm, {"test_ratio": 0.2})
        for k, v in (("x", x), ("y", y), ("xt", xt), ("yt", yt)):
            out[f"{dnm}_{k}"] = v.numpy()
        out[f"{dnm}_meta"] = np.array([N, D, nc])
        print(dnm, N, D, nc)
    np.savez_compressed(os.path.join(OUT, "d1_datasets.npz"), **out)


def main():
    if "--child" in sys.argv:
        _child()
        return
    env = dict(os.environ)
    env["PYTHONPATH"] = REF
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    subprocess.run([sys.executable, "-B", os.path.abspath(__file__), "--child"],
                   env=env, check=True, cwd="/tmp")


if __name__ == "__main__":
    main()
