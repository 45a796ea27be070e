"""psvi_inner_loop_ex KEEP / RESUME: a run of inner steps split over several
calls gives the numbers of one call over all of them, bit for bit, and a
resumed call takes the loop's state from the workspace (not from the packed
arrays).  Reference: the inner loop of PSVI.nested_step / hyper_step
(psvi/inference/psvi_classes.py:549-555, 622-650), whose T steps one call
of psvi_inner_loop runs; the split only moves the fixed per-call work."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

C3 = [(64, 40), (40, 40), (40, 2)]


def _case(layers, M, seed):
    rng = np.random.default_rng(seed)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
                  (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
    p0 = torch.tensor(np.concatenate(parts).astype(np.float32), device=DEV)
    u = torch.tensor(rng.standard_normal((M, layers[0][0])).astype(np.float32), device=DEV)
    z = torch.tensor(rng.integers(0, layers[-1][1], M).astype(np.int32), device=DEV)
    w = torch.tensor(rng.uniform(1, 20, M).astype(np.float32), device=DEV)
    return p0, u, z, w


def _state(p0):
    return p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)


@pytest.mark.parametrize("layers,S", [(C3, 128), (C3, 64), ([(12, 20), (20, 4)], 128)])
@pytest.mark.parametrize("kind", ["higher", "hypergrad"])
def test_split_calls_equal_one_call(layers, S, kind):
    from psvi.runtime import InnerLoopPlan

    M, seed, lr = 40, 31, 1e-3
    plan = InnerLoopPlan("fullcov", layers, S, M)
    assert plan.tiled_floats > 0
    p0, u, z, w = _case(layers, M, 5)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=DEV)
    # one call of 2 + 5 + 3 steps
    p1, m1, v1 = _state(p0)
    e1 = plan.inner_loop(u, z, w, p1, m1, v1, 10, lr, kind=kind, seed=seed, ws=ws).clone()
    # three calls, each continuing the last (the last one plain)
    p2, m2, v2 = _state(p0)
    es, off, step = [], 0, 1
    for T, keep in ((2, True), (5, True), (3, False)):
        es.append(plan.inner_loop(u, z, w, p2, m2, v2, T, lr, kind=kind, step0=step, seed=seed,
                                  offset=off, ws=ws, keep=keep).clone())
        off += T * plan.eps_stride
        step += T
    torch.cuda.synchronize()
    for a, b, n in ((p1, p2, "params"), (m1, m2, "m"), (v1, v2, "v")):
        assert torch.equal(a, b), n
    assert torch.equal(e1, torch.cat(es))
    # a KEEP call's packed arrays after its fused last step: the plain call's
    # values up to fp32 rounding (Adam's step ~ lr sign(g) where g cancels)
    p3, m3, v3 = _state(p0)
    e3 = plan.inner_loop(u, z, w, p3, m3, v3, 10, lr, kind=kind, seed=seed, ws=ws, keep=True)
    torch.cuda.synchronize()
    # (the last step's KL term is summed by the other kernel too)
    assert torch.equal(e3[:-1], e1[:-1])
    assert abs(e3[-1].item() - e1[-1].item()) <= 1e-6 * abs(e1[-1].item())
    assert (p3 - p1).abs().max().item() <= 2 * lr
    assert ((p3 - p1).norm() / p1.norm()).item() < 1e-5


def test_resume_takes_the_resident_state():
    """After a KEEP call, the packed corr entries are overwritten behind the
    version counter (.data): a RESUME call ignores them (the tiled state in ws
    is the loop's), and copies its own back at the end."""
    from psvi.runtime import InnerLoopPlan

    layers, S, M, seed, lr = C3, 128, 40, 8, 1e-3
    plan = InnerLoopPlan("fullcov", layers, S, M)
    p0, u, z, w = _case(layers, M, 6)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=DEV)
    pr, mr, vr = _state(p0)
    er = plan.inner_loop(u, z, w, pr, mr, vr, 6, lr, seed=seed, ws=ws).clone()
    p, m, v = _state(p0)
    plan.inner_loop(u, z, w, p, m, v, 3, lr, seed=seed, ws=ws, keep=True)
    # corr entries of layer 0: after its mean and sd
    n0 = layers[0][0] * layers[0][1] + layers[0][1]
    p.data[2 * n0: 2 * n0 + 1000] = 7.0
    e = plan.inner_loop(u, z, w, p, m, v, 3, lr, step0=4, seed=seed, offset=3 * plan.eps_stride,
                        ws=ws)
    torch.cuda.synchronize()
    assert torch.equal(e, er[3:])
    assert torch.equal(p, pr) and torch.equal(m, mr) and torch.equal(v, vr)


def test_modified_state_starts_cold():
    """A torch write to params between the calls (version counter) or a call
    that does not continue the offset makes the next call start cold: its
    numbers are those of a plain call from the modified state."""
    from psvi.runtime import InnerLoopPlan

    layers, S, M, seed, lr = C3, 128, 40, 9, 1e-3
    plan = InnerLoopPlan("fullcov", layers, S, M)
    p0, u, z, w = _case(layers, M, 7)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=DEV)
    ws2 = torch.empty_like(ws)
    off = 3 * plan.eps_stride
    for case in ("written", "offset"):
        p, m, v = _state(p0)
        plan.inner_loop(u, z, w, p, m, v, 3, lr, seed=seed, ws=ws, keep=True)
        if case == "written":
            p.mul_(0.5)
            o = off
        else:
            o = 100 * plan.eps_stride
        ref = [t.clone() for t in (p, m, v)]
        e = plan.inner_loop(u, z, w, p, m, v, 4, lr, step0=4, seed=seed, offset=o, ws=ws).clone()
        e_ref = plan.inner_loop(u, z, w, *ref, 4, lr, step0=4, seed=seed, offset=o, ws=ws2)
        torch.cuda.synchronize()
        assert torch.equal(e, e_ref), case
        for a, b in zip((p, m, v), ref):
            assert torch.equal(a, b), case


@pytest.mark.parametrize("call", ["elbo_grad", "hvp", "elbo_grad_c"])
def test_other_calls_on_the_workspace_drop_the_state(call):
    """A KEEP loop, then another library call on the same workspace (it writes
    the draw / x / tiled scratch the state lives in), then a call that would
    continue the loop: it starts cold -- its numbers are those of a plain call
    from the packed state.  elbo_grad_c: through the C ABI alone (the
    library's own drop, not the host's version counter)."""
    import ctypes

    from psvi.runtime import InnerLoopPlan, randn_
    from psvi.runtime import _lib

    layers, S, M, seed, lr = C3, 128, 40, 12, 1e-3
    plan = InnerLoopPlan("fullcov", layers, S, M)
    p0, u, z, w = _case(layers, M, 8)
    ws = torch.empty(max(plan.loop_ws_bytes, plan.hvp_ws_bytes), dtype=torch.uint8, device=DEV)
    ws2 = torch.empty_like(ws)
    e = torch.empty(plan.eps_count, device=DEV)
    randn_(e, 99)
    p, m, v = _state(p0)
    plan.inner_loop(u, z, w, p, m, v, 3, lr, seed=seed, ws=ws, keep=True)
    if call == "elbo_grad":
        plan.elbo_grad(u, z, w, e, p, ws=ws)
    elif call == "hvp":
        plan.hvp(u, z, w, e, p, torch.randn_like(p), ws=ws)
    else:
        elbo = torch.empty(1, dtype=torch.float64, device=DEV)
        grad = torch.empty_like(p)
        f = lambda t: ctypes.c_void_p(t.data_ptr())
        rc = plan.lib.psvi_elbo_grad(plan.handle, f(u), f(z), f(w), f(e), f(p), 1, f(elbo),
                                     f(grad), f(ws), ws.numel(),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        # the host token still matches: RESUME is passed, the library refuses it
        assert plan._resident is not None
    ref = [t.clone() for t in (p, m, v)]
    off = 3 * plan.eps_stride
    got = plan.inner_loop(u, z, w, p, m, v, 4, lr, step0=4, seed=seed, offset=off, ws=ws).clone()
    want = plan.inner_loop(u, z, w, *ref, 4, lr, step0=4, seed=seed, offset=off, ws=ws2)
    torch.cuda.synchronize()
    assert torch.equal(got, want), call
    for a, b in zip((p, m, v), ref):
        assert torch.equal(a, b), call
