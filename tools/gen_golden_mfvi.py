#!/usr/bin/env python3
"""Golden vectors for the MFVI baselines:
``run_mfvi`` (psvi/inference/baselines.py:824-914) and ``run_mfvi_subset``
(baselines.py:917-1062) -- the inner ELBO with uniform weights N/B on data
minibatches (resp. on a fixed random subset), torch.optim.Adam, and the
mean-logit predictive evaluation every log_every iterations.

Runs ONLY in the development container.  Like tools/gen_golden.py, the parent
re-launches this script in a child whose sys.path holds the reference and not
this repo; the child calls the reference's run_mfvi / run_mfvi_subset
themselves on small in-memory datasets and records every Normal /
MultivariateNormal draw in order (training forwards and evaluation forwards
interleaved, as the reference consumes them), the initial parameters (by
wrapping the set_up_model the baselines module calls), and the returned
results (elbos, accs, nlls).  The minibatch is the whole training set, so a
step's loss does not depend on the DataLoader's shuffle order.

Usage:  python tools/gen_golden_mfvi.py      (writes tests/golden/b*.npz)
"""
import json
import os
import subprocess
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def _child():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gen_golden import _install_stubs, _Recorder

    _install_stubs()
    import numpy as np
    import torch
    from torch.nn.utils import parameters_to_vector
    from torch.utils.data import TensorDataset

    import psvi.inference.baselines as B

    torch.set_default_dtype(torch.float32)
    rec = _Recorder()
    captured = {}
    orig_setup = B.set_up_model

    def setup_wrapper(**kw):
        net = orig_setup(**kw)
        captured["p0"] = parameters_to_vector(net.parameters()).detach().clone()
        return net

    B.set_up_model = setup_wrapper
    gen = torch.Generator().manual_seed(99)

    def dataset(n, D, nc):
        x = torch.randn(n, D, generator=gen)
        Wt = torch.randn(D, nc, generator=gen)
        y = (x @ Wt).argmax(1).float()
        return x, y

    def run(name, fn, arch, D, nc, n_hidden, S, n_train, n_test, iters, log_every, lr,
            init_sd, extra):
        x, y = dataset(n_train, D, nc)
        xt, yt = dataset(n_test, D, nc)
        kw = dict(mc_samples=S, data_minibatch=n_train, num_epochs=iters, mul_fact=1,
                  log_every=log_every, D=D, lr0net=lr, seed=0, architecture=arch,
                  n_hidden=n_hidden, nc=nc, train_dataset=TensorDataset(x, y),
                  test_dataset=TensorDataset(xt, yt), init_sd=init_sd, **extra)
        if fn == "run_mfvi_subset":
            kw.update(x=x, y=y)
        rec.start()
        res = getattr(B, fn)(**kw)
        draws = rec.stop()
        cfg = dict(fn=fn, arch=arch, D=D, nc=nc, n_hidden=n_hidden, S=S, n_train=n_train,
                   iters=iters, log_every=log_every, lr=lr, init_sd=init_sd,
                   num_pseudo=extra.get("num_pseudo"))
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"), config=np.array(json.dumps(cfg)),
            x=x.numpy(), y=y.numpy(), xt=xt.numpy(), yt=yt.numpy(),
            params0=captured["p0"].numpy(), draws=draws.numpy().astype(np.float32),
            elbos=np.array(res["elbos"], np.float64), accs=np.array(res["accs"], np.float64),
            nlls=np.array(res["nlls"], np.float64))
        print(f"wrote {name}: {len(res['elbos'])} iterations, elbos {res['elbos'][:2]}..., "
              f"accs {res['accs']}, draws {draws.numel()}")

    run("b1_mfvi_fn", "run_mfvi", "fn", 2, 3, 20, 4, 60, 30, 4, 2, 1e-2, 0.05, {})
    run("b2_mfvi_fn2", "run_mfvi", "fn2", 3, 2, 4, 4, 40, 20, 3, 2, 1e-2, 0.05, {})
    run("b3_mfvi_subset_logreg", "run_mfvi_subset", "logistic_regression", 2, 2, None, 4,
        50, 20, 4, 2, 1e-2, None, dict(num_pseudo=10))


def main():
    if "--child" in sys.argv:
        _child()
        return
    os.makedirs(OUT, exist_ok=True)
    env = dict(os.environ)
    env["PYTHONPATH"] = REF
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    subprocess.run([sys.executable, "-B", os.path.abspath(__file__), "--child"],
                   env=env, check=True, cwd="/tmp")


if __name__ == "__main__":
    main()
