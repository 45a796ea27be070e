"""The op-faithful CPU restatement (oracle/cpu_reference.py, bench.py's
cpu_baseline leg) reproduces the reference's numbers: inner loops on the g*
fixtures, whole nested_steps on the n* fixtures (float64, draws replayed)."""
import numpy as np
import pytest
import torch

from cpu_reference import RefInnerStep
from golden_util import adam_kind, fixture_names, l2rel, load_fixture, rel


@pytest.mark.parametrize("name", ["g1r_logreg_rand", "g3r_fn2_tiny_rand", "g2h_fn_c2_hyper"])
def test_cpu_inner_loop_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    r = RefInnerStep(cfg["family"], cfg["layers"], cfg["S"])
    elbos, p = r.run(torch.tensor(f["params0"]), torch.tensor(f["u"]), torch.tensor(f["z"]),
                     torch.tensor(f["w"]), cfg["T"], cfg["lr"], eps_list=list(f["eps"]),
                     adam=adam_kind(cfg), create_graph=False)
    assert rel(elbos, f["elbo"]) < 1e-5
    assert l2rel(p.numpy(), f["params"][-1]) < 1e-5


@pytest.mark.parametrize("name", fixture_names("n"))
def test_cpu_nested_step_matches_reference(name):
    f = load_fixture(name)
    cfg = f["cfg"]
    d = torch.float64
    prev = torch.get_default_dtype()
    torch.set_default_dtype(d)
    try:
        r = RefInnerStep(cfg["family"], cfg["layers"], cfg["S"])
        loss, gu, gv = r.nested_step(
            torch.tensor(f["params0"], dtype=d), torch.tensor(f["u0"], dtype=d),
            torch.tensor(f["z"], dtype=d), torch.tensor(f["v0"], dtype=d), cfg["N"],
            torch.tensor(f["xb"], dtype=d), torch.tensor(f["yb"], dtype=d), cfg["T"],
            cfg["lr0net"], eps_inner=[torch.tensor(e, dtype=d) for e in f["eps_inner"]],
            eps_outer=torch.tensor(f["eps_outer"][0], dtype=d))
    finally:
        torch.set_default_dtype(prev)
    assert rel(loss, f["loss"]) < 1e-10
    assert l2rel(gu.numpy(), f["u_grad"]) < 1e-8
    assert l2rel(gv.numpy(), f["v_grad"]) < 1e-8


def test_lenet_op_faithful_step_matches_reference_fixture():
    """RefLenetStep (the bench's C5 CPU baseline) replays make_lenet's inner
    loop: the reference's ELBOs and Adam trajectory on its own draws."""
    from cpu_reference import RefLenetStep

    f = load_fixture("l1_lenet_tiny")
    cfg = f["cfg"]
    r = RefLenetStep(cfg["S"])
    elbos, p = r.run(torch.tensor(f["params0"]), torch.tensor(f["u"]),
                     torch.tensor(f["z"]), torch.tensor(f["w"]), cfg["T"], cfg["lr"],
                     eps_list=[torch.tensor(e) for e in f["eps"]])
    assert np.allclose(elbos, f["elbo"], rtol=1e-5)
    assert np.linalg.norm(p.numpy() - f["params"][-1]) <= 1e-5 * np.linalg.norm(f["params"][-1])
