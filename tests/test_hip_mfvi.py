"""MFVI baselines on the HIP path (psvi.inference.baselines.run_mfvi /
run_mfvi_subset) replaying the reference's own runs (fixtures b*): the
training steps take the recorded noise through ``eps_source``; the
evaluation forwards draw theirs through torch.distributions, patched to the
same recorded stream.  ELBOs within 1e-5 relative, accuracies exact."""
import numpy as np
import pytest
import torch
from torch.utils.data import TensorDataset

from golden_util import fixture_names, load_fixture

pytestmark = pytest.mark.gpu


class _Stream:
    def __init__(self, flat):
        self.flat = torch.tensor(flat)
        self.o = 0

    def take(self, n):
        out = self.flat[self.o:self.o + n]
        assert out.numel() == n, "draw stream exhausted"
        self.o += n
        return out


@pytest.mark.parametrize("name", fixture_names("b"))
def test_mfvi_replays_reference(name):
    import torch.distributions.multivariate_normal as mv
    import torch.distributions.normal as nm

    from psvi.inference.baselines import run_mfvi, run_mfvi_subset

    f = load_fixture(name)
    cfg = f["cfg"]
    st = _Stream(f["draws"])

    def std_normal(shape, dtype, device):
        n = int(np.prod(shape)) if len(shape) else 1
        return st.take(n).reshape(shape).to(dtype=dtype, device=device)

    kw = dict(mc_samples=cfg["S"], data_minibatch=cfg["n_train"], num_epochs=cfg["iters"],
              mul_fact=1, log_every=cfg["log_every"], D=cfg["D"], lr0net=cfg["lr"], seed=0,
              architecture=cfg["arch"], n_hidden=cfg["n_hidden"], nc=cfg["nc"],
              train_dataset=TensorDataset(torch.tensor(f["x"]), torch.tensor(f["y"])),
              test_dataset=TensorDataset(torch.tensor(f["xt"]), torch.tensor(f["yt"])),
              init_sd=cfg["init_sd"], eps_source=st.take)
    orig = (nm._standard_normal, mv._standard_normal)
    nm._standard_normal = mv._standard_normal = std_normal
    try:
        if cfg["fn"] == "run_mfvi":
            res = run_mfvi(**kw)
        else:
            res = run_mfvi_subset(x=torch.tensor(f["x"]), y=torch.tensor(f["y"]),
                                  num_pseudo=cfg["num_pseudo"], **kw)
    finally:
        nm._standard_normal, mv._standard_normal = orig
    assert st.o == st.flat.numel()
    assert np.allclose(res["elbos"], f["elbos"], rtol=1e-5), (res["elbos"], f["elbos"])
    nt = len(f["yt"])
    assert np.array_equal(np.round(np.array(res["accs"]) * nt), np.round(f["accs"] * nt))
    assert np.allclose(res["nlls"], f["nlls"], rtol=1e-4)


def test_mfvi_lenet_step_runs_on_hip():
    """The same stepper drives the LeNet plan (KL on the VILinear layers only)."""
    from psvi.inference.baselines import run_mfvi

    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (64,), generator=g).float()
    res = run_mfvi(mc_samples=2, data_minibatch=32, num_epochs=3, mul_fact=1, log_every=2,
                   lr0net=1e-3, architecture="lenet", nc=10,
                   train_dataset=TensorDataset(x, y), test_dataset=TensorDataset(x[:16], y[:16]))
    assert len(res["elbos"]) == 3 and np.isfinite(res["elbos"]).all()
    assert len(res["accs"]) == 2


def test_experiment_driver_end_to_end(tmp_path):
    """flow_psvi-style driver on halfmoon: a PSVI method and the MFVI baseline,
    results dict in the reference's layout, written as .pk / .json."""
    from psvi.experiments import experiment_driver

    args = dict(mc_samples=4, num_epochs=2, data_minibatch=100, inner_it=2, trainer="nested",
                log_every=1, lr0u=1e-3, lr0net=1e-3, lr0v=1e-2, init_sd=1e-3,
                coreset_sizes=[10], num_trials=1, test_ratio=0.2, architecture="fn",
                logistic_regression=False, n_hidden=10, fnm="drv",
                results_folder=str(tmp_path))
    res = experiment_driver(["halfmoon"], ["psvi_learn_v", "mfvi"], args)
    assert len(res["halfmoon"]["psvi_learn_v"]["10"]["0"]["accs"]) >= 1
    assert len(res["halfmoon"]["mfvi"]["-1"]["0"]["elbos"]) == 4
    assert (tmp_path / "drv.pk").exists() and (tmp_path / "drv.json").exists()
