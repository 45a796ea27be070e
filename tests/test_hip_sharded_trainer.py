"""Sample-sharded second-order trainers on the GPU: PSVI.hyper_step /
nested_step with world > 1, the ranks emulated as threads of one process (one
PSVI instance per rank, all_reduce through a thread barrier).  Each rank's
inner objective, psvi_hvp_partial and outer passes run on a world-1 plan of its
own samples (SampleShardedPlan, ShardedOuter); every rank must reproduce the
reference's whole hyper_step / nested_step (y*, n*, v14 fixtures), and at
C5's size (make_lenet, S = 256, M = 500) the world-8 hyper_step must agree with
the world-1 one on the same Philox draws."""
import threading

import numpy as np
import pytest
import torch

from golden_util import l2rel, load_fixture, rel

pytestmark = pytest.mark.gpu


class _ThreadComm:
    def __init__(self, world):
        self.slots = [None] * world
        self.bar = threading.Barrier(world)

    def bind(self, rank):
        outer = self

        class _Rank:
            def all_reduce(self, t):
                outer.slots[rank] = t.clone()
                outer.bar.wait()
                total = sum(outer.slots[r] for r in range(len(outer.slots)))
                outer.bar.wait()
                t.copy_(total)

        return _Rank()


def _run_ranks(world, fn):
    comm = _ThreadComm(world)
    res, errs = [None] * world, []

    def run(r):
        try:
            res[r] = fn(r, comm.bind(r))
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not errs, errs
    return res


def _fixture_rank(name, cls, world, rank, comm):
    from test_host_api import build_model

    f = load_fixture(name)
    cfg = f["cfg"]
    model = build_model(cfg, f["params0"]).cuda()
    u = torch.tensor(f["u0"], device="cuda").requires_grad_(True)
    ps = cls(u=u, z=torch.tensor(f["z"], device="cuda"), N=cfg["N"], model=model,
             mc_samples=cfg["S"], device_id=0, inner_it=cfg["T"], world=world, rank=rank,
             comm=comm)
    ps.device = torch.device("cuda")
    ps.v = torch.tensor(f["v0"], device="cuda").requires_grad_(True)
    if getattr(ps, "alpha", None) is not None and "alpha0" in f:
        ps.alpha = torch.tensor(f["alpha0"], device="cuda").reshape(1).requires_grad_(True)
        ps.f = lambda *x: torch.exp(ps.alpha) * torch.softmax(x[0], x[1])
    ps.setup_optimizers(lr0net=cfg["lr0net"], lr0u=cfg["lr0u"], lr0v=cfg["lr0v"])
    ei = [torch.tensor(e, device="cuda") for e in f["eps_inner"]]
    eo = [torch.tensor(e, device="cuda") for e in f["eps_outer"]]
    xb, yb = torch.tensor(f["xb"], device="cuda"), torch.tensor(f["yb"], device="cuda")
    if "K" in cfg:
        ll = ps.hyper_step(xb, yb, K=cfg["K"], linsys_lr=cfg["linsys_lr"], eps_inner=ei,
                           eps_outer=eo, hypergrad_approx=cfg.get("approx", "CG_normaleq"))
    else:
        ll = ps.nested_step(xb, yb, eps_inner=ei, eps_outer=eo).item()
    p = torch.nn.utils.parameters_to_vector(model.parameters()).detach().cpu().numpy()
    return dict(ll=ll, params=p, u_grad=ps.u.grad.cpu().numpy(), v_grad=ps.v.grad.cpu().numpy())


@pytest.mark.parametrize("name,world", [("y1_fn2_tiny", 8), ("y2_fn_deep", 3), ("y5_lenet", 2),
                                        ("n1_fn2_tiny", 4), ("n2_fn_deep", 2)])
def test_sharded_trainer_matches_reference(name, world):
    from psvi.inference import PSVILearnV

    f = load_fixture(name)
    res = _run_ranks(world, lambda r, c: _fixture_rank(name, PSVILearnV, world, r, c))
    for g in res:
        assert l2rel(g["params"], f["params"]) < 1e-5
        for k in ("u_grad", "v_grad"):
            own = l2rel(f[k + "_fp32"], f[k]) if k + "_fp32" in f else 0.0
            assert l2rel(g[k], f[k]) < max(1e-4, 4 * own), (name, k, l2rel(g[k], f[k]))
        assert rel(g["ll"], f["ll"] if "ll" in f else f["loss"]) < 1e-5
        assert np.array_equal(g["params"], res[0]["params"])


def test_c5_lenet_hyper_step_world8_matches_world1():
    """C5's bilevel outer (make_lenet, S = 256, M = 500, a 128-image data
    batch) split over 8 ranks against one rank, same Philox draws."""
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
            ll = ps.hyper_step(xb, yb, K=3)
            pv = torch.nn.utils.parameters_to_vector(net.parameters()).detach().cpu().numpy()
            return dict(ll=ll, params=pv, u_grad=ps.u.grad.cpu().numpy(),
                        v_grad=ps.v.grad.cpu().numpy())
        return fn

    one = _run_ranks(1, rank_fn(1))[0]
    eight = _run_ranks(8, rank_fn(8))

    for g in eight:
        assert l2rel(g["params"], one["params"]) < 1e-5
        # d/du: the two runs' inner solutions differ in the last bits (the
        # weight gradients are summed over differently cut image chunks).  At
        # C5 the importance weights W_s = softmax_s(nkl_s - pseudo_s) see
        # pseudo_s ~ N sum_m f(v)_m NLL ~ 1e5, so fp32 noise of 1e-7 relative
        # moves the exponents by ~1e-2 and W (hence d/du) by ~1 %.  Bound here:
        # 1e-2 overall, the loss to 1e-5; the tight check of the two
        # decompositions at IDENTICAL parameters is
        # test_c5_outer_world8_decomposition_identical_params below.
        assert l2rel(g["u_grad"], one["u_grad"]) < 1e-2
        assert l2rel(g["v_grad"], one["v_grad"]) < 1e-2
        assert rel(g["ll"], one["ll"]) < 1e-5


def test_c5_outer_world8_decomposition_identical_params():
    """C5's outer objective (make_lenet, S = 256, M = 500 + a 128-image batch)
    at one parameter vector: the world-1 plan's gradients against the sum of 8
    sample shards of 32 (psvi_outer_elbo_grad_coef with the global softmax
    coefficients, as ShardedOuter runs it).  Same parameters, same draw: the
    two decompositions differ by fp32 summation order only, so d/du and the
    parameter gradient must agree tightly (measured 2e-7) -- the check the hyper_step comparison above
    cannot make through the softmax's sensitivity."""
    from psvi.models import LENET_LAYERS, make_lenet
    from psvi.runtime import InnerLoopPlan, randn_
    from psvi.runtime.sharded import local_eps, outer_coefficients, pack_coef, sample_split

    S, M, Nx = 256, 500, 128
    g = torch.Generator().manual_seed(3)
    u = torch.randn(M, 784, generator=g)
    xb = torch.randn(Nx, 784, generator=g)
    z = torch.randint(0, 10, (M + Nx,), generator=g).int()
    torch.manual_seed(0)
    p = torch.nn.utils.parameters_to_vector(
        make_lenet(mc_samples=S, init_sd=0.05).parameters()).detach().cuda()
    x_all = torch.cat([u, xb]).cuda().contiguous()
    z_all = z.cuda()
    w_all = torch.cat([torch.full((M,), 120.0), torch.full((Nx,), 60000.0 / Nx)]).cuda()
    one = InnerLoopPlan("lenet", LENET_LAYERS, S, M + Nx)
    e = torch.empty(one.eps_count, device="cuda")
    randn_(e, 5)
    o1 = one.outer_elbo_grad(M, x_all, z_all, w_all, e, p, sample_stats=True)
    loss, cp, cd, ck = outer_coefficients(o1["samples"][:, :3].contiguous())
    assert rel(float(loss), float(o1["loss"])) < 1e-9
    gu8 = torch.zeros_like(o1["grad_u"])
    g8 = torch.zeros_like(o1["grad"])
    gw8 = torch.zeros_like(o1["grad_w"])
    for off, cnt in sample_split(S, 8):
        pl = InnerLoopPlan("lenet", LENET_LAYERS, cnt, M + Nx)
        el = local_eps("lenet", LENET_LAYERS, S, off, cnt, e)
        gg = pl.outer_grad_coef(M, x_all, z_all, w_all, el, p,
                                pack_coef(cp, cd, ck, off, cnt).cuda())
        gu8 += gg["grad_u"]
        g8 += gg["grad"]
        gw8 += gg["grad_w"]
    assert l2rel(gu8.cpu().numpy(), o1["grad_u"].cpu().numpy()) < 1e-5
    assert l2rel(g8.cpu().numpy(), o1["grad"].cpu().numpy()) < 1e-5
    assert l2rel(gw8.cpu().numpy(), o1["grad_w"].cpu().numpy()) < 1e-5
