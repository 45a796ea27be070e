"""Device-side non-finite check (psvi_nonfinite) and the trainers' anomaly
mode: with torch.autograd.set_detect_anomaly(True) (the reference driver's
setting, psvi/experiments/flow_psvi.py:50) a non-finite objective or gradient
raises RuntimeError after the step, as the reference's anomaly detection does;
finite runs pass, and with anomaly mode off nothing is read back."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_nonfinite_flag():
    from psvi.runtime import nonfinite_

    for dt in (torch.float32, torch.float64):
        x = torch.randn(100003, device="cuda", dtype=dt)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        nonfinite_(flag, x)
        assert int(flag.item()) == 0
        for bad in (float("nan"), float("inf"), -float("inf")):
            y = x.clone()
            y[77777] = bad
            flag.zero_()
            nonfinite_(flag, x, y)
            assert int(flag.item()) == 1


def _ps():
    from psvi.inference import PSVILearnV
    from psvi.models import make_fcnet

    torch.manual_seed(0)
    model = make_fcnet(5, 7, 3, n_layers=2, mc_samples=6, init_sd=0.05).cuda()
    u = torch.randn(13, 5, device="cuda").requires_grad_(True)
    z = (torch.arange(13, device="cuda") % 3).float()
    ps = PSVILearnV(u=u, z=z, N=500, model=model, mc_samples=6, device_id=0, inner_it=3)
    ps.device = torch.device("cuda")
    ps.setup_optimizers()
    return ps, model


def test_anomaly_mode_raises_on_nonfinite_and_passes_finite():
    ps, model = _ps()
    xb, yb = torch.randn(9, 5, device="cuda"), (torch.arange(9, device="cuda") % 3).float()
    with torch.autograd.set_detect_anomaly(True):
        ps.inner_loop()
        ps.nested_step(xb, yb)
        ps.hyper_step(xb, yb, K=2)
        with torch.no_grad():
            next(model.parameters())[0, 0] = float("nan")
        with pytest.raises(RuntimeError, match="non-finite"):
            ps.inner_loop()
        with pytest.raises(RuntimeError, match="non-finite"):
            ps.nested_step(xb, yb)
    assert np.isnan(next(model.parameters()).detach().cpu().numpy()).any()
