"""A/B of the C5 world-8 vs world-1 hyper_step agreement (tests/
test_hip_sharded_trainer.py::test_c5_lenet_hyper_step_world8_matches_world1)
with the LeNet conv towers on the VALU kernels (PSVI_DBG_LENET_CONV_VALU) and
on MFMA: the spread both give is fp32 summation-order noise amplified by CG."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]

from golden_util import l2rel, rel  # noqa: E402
from psvi.runtime import _lib  # noqa: E402
from test_hip_sharded_trainer import _run_ranks  # noqa: E402


def run(K):
    from psvi.inference import PSVILearnV
    from psvi.models import make_lenet

    S, M = 256, 500
    g = torch.Generator().manual_seed(3)
    u0 = torch.randn(M, 1, 28, 28, generator=g)
    z = torch.randint(0, 10, (M,), generator=g).float()
    xb = torch.randn(128, 1, 28, 28, generator=g).cuda()
    yb = torch.randint(0, 10, (128,), generator=g).float().cuda()
    torch.manual_seed(0)
    p0 = torch.nn.utils.parameters_to_vector(make_lenet(mc_samples=S, init_sd=0.05).parameters())

    def rank_fn(world):
        def fn(r, comm):
            net = make_lenet(mc_samples=S, init_sd=0.05).cuda()
            with torch.no_grad():
                torch.nn.utils.vector_to_parameters(p0.detach().cuda(), net.parameters())
            ps = PSVILearnV(u=u0.clone().cuda().requires_grad_(True), z=z.cuda(), N=60000,
                            model=net, mc_samples=S, device_id=0, inner_it=2, seed=7,
                            world=world, rank=r, comm=comm)
            ps.device = torch.device("cuda")
            ps.register_elbos = False
            ps.setup_optimizers()
            ll = ps.hyper_step(xb, yb, K=K)
            pv = torch.nn.utils.parameters_to_vector(net.parameters()).detach().cpu().numpy()
            return dict(ll=ll, u_grad=ps.u.grad.cpu().numpy(), v_grad=ps.v.grad.cpu().numpy(),
                        params=pv)
        return fn

    return _run_ranks(1, rank_fn(1))[0], _run_ranks(8, rank_fn(8))[0]


lib = _lib.load()
res = {}
for valu in (1, 0):
    lib.psvi_debug_set(16, valu)
    res[valu] = run(0)
names = {(1, 0): "VALU w1", (1, 1): "VALU w8", (0, 0): "MFMA w1", (0, 1): "MFMA w8"}
keys = list(names)
for i, a in enumerate(keys):
    for b in keys[i + 1:]:
        A, B = res[a[0]][a[1]], res[b[0]][b[1]]
        print(f"{names[a]} vs {names[b]}: params {l2rel(A['params'], B['params']):.2e} "
              f"u_grad {l2rel(A['u_grad'], B['u_grad']):.2e} "
              f"v_grad {l2rel(A['v_grad'], B['v_grad']):.2e}", flush=True)
