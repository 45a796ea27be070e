"""Multi-rank inner step on CPU: world_size 2 and 3 over gloo.

The sharded driver (psvi.runtime.sharded.ShardedInnerLoop: split sizes,
blocked-by-source layouts, the two all_to_all exchanges per full-cov step, the
mean-field all-reduce, reduce_elbo, owned_mask, gather_params) runs for real
over torch.distributed; only its three HIP phases are replaced by oracle
emulations that read and write the same buffers in the same layouts.  One
sharded step must reproduce the world-1 oracle step (negative ELBO, updated
params and Adam state)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _emulate_fullcov(loop, O, layers, S, prior_sd):
    """Install oracle versions of the three full-cov phases on `loop` (a
    rank's rows: whole 64-row bands, possibly several runs per layer, at the
    x-shard columns psvi_plan_shard_runs gives)."""
    from psvi.runtime.sharded import layer_rows

    infos, r = loop.info, loop.rank
    me = infos[r]
    n_l = [a * b + b for a, b in layers]
    woff = np.concatenate([[0], np.cumsum(n_l)]).astype(int)
    rc = [[layer_rows(i, l) for l in range(len(layers))] for i in infos]
    s0 = prior_sd

    def layer_views(params, eps):
        po = eo = 0
        for l, n in enumerate(n_l):
            nc = (n - 1) * (n - 2) // 2
            mean, sd, corr = params[po:po + n], params[po + n:po + 2 * n], params[po + 2 * n:po + 2 * n + nc]
            yield l, n, mean, sd, corr, eps[eo:eo + S * n].reshape(S, n)
            po += 2 * n + nc
            eo += S * n

    def phase_sample(eps, params):
        p = params.double().numpy()
        e = eps.double().numpy()
        X = np.zeros((S, me["rows"]))
        for l, n, mean, sd, corr, E in layer_views(p, e):
            rows, cols = rc[r][l]
            L = O.mvn_dense_L(sd, corr, n)
            X[:, cols] = mean[rows] + E @ L[rows].T
        loop.x_shard.copy_(torch.from_numpy(X.ravel()).float())

    def recv_to_full(buf):
        s_cnt = me["s_count"]
        full = np.zeros((s_cnt, woff[-1]))
        off = 0
        for p, q in enumerate(infos):
            blk = buf[off:off + s_cnt * q["rows"]].reshape(s_cnt, q["rows"])
            for l in range(len(layers)):
                rows, cols = rc[p][l]
                full[:, woff[l] + rows] = blk[:, cols]
            off += s_cnt * q["rows"]
        return full

    def full_to_send(full):
        s_cnt = me["s_count"]
        out = []
        for p, q in enumerate(infos):
            blk = np.zeros((s_cnt, q["rows"]))
            for l in range(len(layers)):
                rows, cols = rc[p][l]
                blk[:, cols] = full[:, woff[l] + rows]
            out.append(blk.ravel())
        return np.concatenate(out)

    def phase_net(u, z, w):
        loop.parts.zero_()
        X = recv_to_full(loop.x_recv.double().numpy())
        Ws, bs = O.mvn_split_x(layers, X)
        data, dWs, dbs = O.net_forward_backward(u.double().numpy(), z.numpy(),
                                                w.double().numpy(), Ws, bs)
        G = np.concatenate([np.concatenate([dWs[l].reshape(X.shape[0], -1), dbs[l]], 1)
                            for l in range(len(layers))], 1)
        loop.g_send.copy_(torch.from_numpy(full_to_send(G)).float())
        loop.parts[0] = data

    def phase_net_half(u, z, w, h, draw=None):
        # the same network on half h of the rank's samples: their rows of
        # g_send, their NLL added
        lo, n = loop._halves(r)[h]
        X = recv_to_full(loop.x_recv.double().numpy())[lo:lo + n]
        Ws, bs = O.mvn_split_x(layers, X)
        data, dWs, dbs = O.net_forward_backward(u.double().numpy(), z.numpy(),
                                                w.double().numpy(), Ws, bs)
        G = np.concatenate([np.concatenate([dWs[l].reshape(X.shape[0], -1), dbs[l]], 1)
                            for l in range(len(layers))], 1)
        full = np.zeros((me["s_count"], woff[-1]))
        full[lo:lo + n] = G
        send = full_to_send(full)
        cur = loop.g_send.double().numpy()
        off = 0
        for q in infos:
            blk_c = cur[off:off + me["s_count"] * q["rows"]].reshape(me["s_count"], q["rows"])
            blk_n = send[off:off + me["s_count"] * q["rows"]].reshape(me["s_count"], q["rows"])
            blk_c[lo:lo + n] = blk_n[lo:lo + n]
            off += me["s_count"] * q["rows"]
        loop.g_send.copy_(torch.from_numpy(cur).float())
        loop.parts[0] += data

    def phase_update(eps, params, m, v, step, lr, kind, grad_out=None):
        p = params.double().numpy()
        e = eps.double().numpy()
        Gs = loop.g_shard.double().numpy().reshape(S, me["rows"])
        G = np.zeros((S, woff[-1]))
        kl = 0.0
        for l, n, mean, sd, corr, E in layer_views(p, e):
            rows, cols = rc[r][l]
            G[:, woff[l] + rows] = Gs[:, cols]
            L = O.mvn_dense_L(sd, corr, n)[rows]
            sp = O.softplus(sd[rows])
            kl += float(np.sum(np.log(s0) - np.log(sp) - 0.5
                               + 0.5 * ((L * L).sum(1) + mean[rows] ** 2) / s0 ** 2))
        g = O.mvn_grad_from_G(layers, p, G, e, S, prior_sd=s0)
        own = loop.owned_mask().numpy()
        pn, mn, vn = O.adam(kind, p, g, m.double().numpy(), v.double().numpy(), step, lr)
        for t, new in ((params, pn), (m, mn), (v, vn)):
            cur = t.double().numpy()
            cur[own] = new[own]
            t.copy_(torch.from_numpy(cur).to(t.dtype))
        loop.parts[1] = kl

    def phase_update_sample(eps, params, m, v, step, lr, kind, eps_next):
        phase_update(eps, params, m, v, step, lr, kind)
        phase_sample(eps_next, params)

    loop.phase_sample, loop.phase_net, loop.phase_update = phase_sample, phase_net, phase_update
    loop.phase_update_sample = phase_update_sample
    loop.phase_net_half = phase_net_half


def _rank_main(rank, world, port, name, kind_override, out):
    import sys
    for p in (os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import psvi_oracle as O
    from golden_util import adam_kind, load_fixture
    from psvi.runtime.sharded import ShardedInnerLoop, TorchDistComm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = load_fixture(name)
        cfg = f["cfg"]
        layers, S, M = cfg["layers"], cfg["S"], cfg["M"]
        kind = kind_override or adam_kind(cfg)
        loop = ShardedInnerLoop("fullcov", layers, S, M, world, rank, prior_sd=cfg["prior_sd"],
                                device="cpu", comm=TorchDistComm())
        _emulate_fullcov(loop, O, layers, S, cfg["prior_sd"])
        t = lambda x, d=torch.float32: torch.tensor(np.ascontiguousarray(x), dtype=d)
        params = t(f["params0"]).double()
        m = torch.zeros_like(params)
        v = torch.zeros_like(params)
        parts = torch.zeros(1, 2, dtype=torch.float64)
        loop.step(t(f["u"]), t(f["z"].astype(np.int32), torch.int32), t(f["w"]), t(f["eps"][0]),
                  params, m, v, step=1, lr=cfg["lr"], kind=kind, elbo_parts=parts[0])
        negelbo = loop.reduce_elbo(parts)
        loop.gather_params(params, m, v)
        if rank == 0:
            out.put((float(negelbo[0]), params.numpy(), m.numpy(), v.numpy()))
        else:
            out.put(None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name,kind", [("g3r_fn2_tiny_rand", None), ("g4h_fn2_mid_hyper", None)])
def test_sharded_fullcov_step_matches_world1(world, name, kind):
    import psvi_oracle as O
    from golden_util import adam_kind, l2rel, load_fixture, rel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, kind, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    negelbo, params, m, v = next(x for x in res if x is not None)

    f = load_fixture(name)
    cfg = f["cfg"]
    o_elbo, _, o_traj, o_m, o_v = O.run_inner_loop(
        "mvn", cfg["layers"], f["params0"], f["u"], f["z"], f["w"], f["eps"][:1], cfg["S"],
        cfg["lr"], kind or adam_kind(cfg), prior_sd=cfg["prior_sd"])
    assert rel(negelbo, o_elbo[0]) < 1e-6, (negelbo, o_elbo[0])
    assert l2rel(params, o_traj[0]) < 1e-6
    assert l2rel(m, o_m) < 1e-5 and l2rel(v, o_v) < 1e-5


def _run_overlap_rank(rank, world, port, out):
    import sys
    for p in (os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import psvi_oracle as O
    from psvi.runtime.sharded import ShardedInnerLoop, TorchDistComm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        layers, S, M = [(8, 6), (6, 3)], 4 * world + 1, 7
        g = torch.Generator().manual_seed(5)
        u = torch.randn(M, 8, generator=g)
        z = torch.randint(0, 3, (M,), generator=g).to(torch.int32)
        w = torch.rand(M, generator=g) * 10 + 1

        def draw(t, seed, offset):
            gg = torch.Generator().manual_seed(int(seed) * 1000003 + int(offset))
            t.copy_(torch.randn(t.numel(), generator=gg))

        res = []
        for overlap in (False, True):
            loop = ShardedInnerLoop("fullcov", layers, S, M, world, rank, device="cpu",
                                    comm=TorchDistComm())
            _emulate_fullcov(loop, O, layers, S, 1.0)
            loop.draw = draw
            assert loop.plan.net_part_ok   # the overlapped schedule runs (no chunk slots)
            n = [a * b + b for a, b in layers]
            params = torch.cat([torch.cat([0.1 * torch.randn(k, generator=torch.Generator().manual_seed(k)),
                                           torch.full((k,), -4.0),
                                           0.05 * torch.randn((k - 1) * (k - 2) // 2,
                                                              generator=torch.Generator().manual_seed(k + 1))])
                                for k in n])
            m, v = torch.zeros_like(params), torch.zeros_like(params)
            parts = torch.zeros(3, 2, dtype=torch.float64)
            loop.run(u, z, w, params, m, v, 3, 1e-3, seed=9, elbo_parts=parts, overlap=overlap)
            negelbo = loop.reduce_elbo(parts)
            loop.gather_params(params, m, v)
            res.append((negelbo.numpy(), params.numpy(), m.numpy(), v.numpy()))
        out.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_run_overlap_matches_plain(world):
    """run(overlap=True) -- two sample halves, each exchange in two list
    all_to_alls of per-peer views, the network launched per half -- against
    the plain schedule on the same draws: the same steps (float64 oracle
    phases: equal up to the NLL's split sum)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_overlap_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, ((e0, p0, m0, v0), (e1, p1, m1, v1)) in res:
        assert np.allclose(e0, e1, rtol=1e-12, atol=0)
        for a, b in ((p0, p1), (m0, m1), (v0, v1)):
            assert np.allclose(a, b, rtol=1e-6, atol=1e-12)


def _emulate_lenet(loop, O, S):
    """Oracle versions of the LeNet (mean-field-style) phases on `loop`: the
    rank accumulates [sum_s G_s | sum_s G_s eps_s] over its own samples; the
    replicated update turns the all-reduced accumulator into the gradient
    (KL on the VILinear layers) and one Adam step."""
    s_lo, s_cnt = loop.plan.s_offset, loop.plan.s_local
    layers = O.LENET_LAYERS

    def accumulate(u, z, w, eps, params, acc, nll_out):
        p = params.double().numpy()
        Xl = O.lenet_sample(p, eps.double().numpy(), S)
        logits, c = O.lenet_forward(Xl, u.double().numpy(), S)
        M = logits.shape[1]
        zi = z.numpy().astype(np.int64)
        wd = w.double().numpy()
        mx = logits.max(-1, keepdims=True)
        e = np.exp(logits - mx)
        nll = mx[..., 0] + np.log(e.sum(-1)) - logits[:, np.arange(M), zi]
        P = e / e.sum(-1, keepdims=True)
        P[:, np.arange(M), zi] -= 1.0
        G, _ = O._lenet_backward(c, P * wd[None, :, None], S, M)
        sl = slice(s_lo, s_lo + s_cnt)
        g_mu = np.concatenate([G[l][sl].sum(0) for l in range(5)])
        g_e = np.concatenate([(G[l][sl] * Xl[l]["E"][sl if Xl[l]["bat"] else slice(0, 1)]).sum(0)
                              for l in range(5)])
        acc.copy_(torch.from_numpy(np.concatenate([g_mu, g_e])).float())
        nll_out += float((nll[sl] @ wd).sum())

    def update(acc, params, m, v, step, lr, kind, kl_out=None, grad_out=None):
        p = params.double().numpy()
        a = acc.double().numpy()
        n_tot = a.size // 2
        grad = np.zeros_like(p)
        kl, po, wo = 0.0, 0, 0
        for nw, nb, _, has_kl in layers:
            n = nw + nb
            mu, rho = p[po:po + n], p[po + n:po + 2 * n]
            sp, sg = O.softplus(rho), O.sigmoid(rho)
            gm, gr = a[wo:wo + n].copy(), a[n_tot + wo:n_tot + wo + n] * sg
            if has_kl:
                gm += mu
                gr += (sp - 1.0 / sp) * sg
                kl += float((0.5 * (sp ** 2 + mu ** 2 - 1.0 - np.log(sp ** 2))).sum())
            grad[po:po + n], grad[po + n:po + 2 * n] = gm, gr
            po += 2 * n
            wo += n
        pn, mn, vn = O.adam(kind, p, grad, m.double().numpy(), v.double().numpy(), step, lr)
        for t, new in ((params, pn), (m, mn), (v, vn)):
            t.copy_(torch.from_numpy(new).to(t.dtype))
        if kl_out is not None:
            kl_out += kl

    loop.plan.mf_accumulate = accumulate
    loop.plan.mf_update = update


def _rank_main_lenet(rank, world, port, out):
    import sys
    for p in (os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import psvi_oracle as O
    from golden_util import LENET_PLAN_LAYERS, adam_kind, load_fixture
    from psvi.runtime.sharded import ShardedInnerLoop, TorchDistComm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = load_fixture("l1_lenet_tiny")
        cfg = f["cfg"]
        S, M = cfg["S"], cfg["M"]
        loop = ShardedInnerLoop("lenet", LENET_PLAN_LAYERS, S, M, world, rank, device="cpu",
                                comm=TorchDistComm())
        _emulate_lenet(loop, O, S)
        t = lambda x, d=torch.float32: torch.tensor(np.ascontiguousarray(x), dtype=d)
        params = t(f["params0"]).double()
        m, v = torch.zeros_like(params), torch.zeros_like(params)
        parts = torch.zeros(1, 2, dtype=torch.float64)
        loop.step(t(f["u"]), t(f["z"].astype(np.int32), torch.int32), t(f["w"]), t(f["eps"][0]),
                  params, m, v, step=1, lr=cfg["lr"], kind=adam_kind(cfg), elbo_parts=parts[0])
        negelbo = loop.reduce_elbo(parts)
        out.put((rank, loop.plan.s_local, float(negelbo[0]), params.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_lenet_step_matches_world1(world):
    """C5's multi-GPU shape: LeNet samples sharded, one all-reduce of the
    accumulator per step; every rank ends with the world-1 oracle step."""
    import psvi_oracle as O
    from golden_util import adam_kind, l2rel, load_fixture, rel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main_lenet, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f = load_fixture("l1_lenet_tiny")
    cfg = f["cfg"]
    assert sum(r[1] for r in res) == cfg["S"]
    o_elbo, _, o_traj, _, _ = O.lenet_inner_loop(f["params0"], f["u"], f["z"], f["w"],
                                                 f["eps"][:1], cfg["S"], cfg["lr"],
                                                 adam_kind(cfg))
    for _, _, negelbo, params in res:
        assert rel(negelbo, o_elbo[0]) < 1e-9, (negelbo, o_elbo[0])
        assert l2rel(params, o_traj[0]) < 1e-9
