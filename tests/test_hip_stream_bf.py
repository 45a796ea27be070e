"""The bf16-piece streaming update (mvn_stream_bf_kernel): psvi_inner_loop in
Philox mode on a tiled S = 128 plan runs both GEMMs of the fused update --
dL = G^T eps and the next sample's x' = L' eps' -- on the bf16 matrix cores
with every operand split into three bf16 pieces (fp32-faithful).  Checked
against the same loop on the fp32 streaming kernel (PSVI_DBG_STREAM_BF_OFF)
and against the float64 oracle on the same Philox draws.  Reference: the
inner loop of PSVI.nested_step / hyper_step (psvi/inference/psvi_classes.py:
549-555, 622-650) over VILinearMultivariateNormal (psvi/models/neural_net.py:
408-491)."""
import numpy as np
import pytest
import torch

import psvi_oracle as O
from golden_util import l2rel, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF_OFF = 24  # PSVI_DBG_STREAM_BF_OFF


def _case(layers, seed):
    rng = np.random.default_rng(seed)
    parts = []
    for din, dout in layers:
        n = din * dout + dout
        parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
                  (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
    return rng, np.concatenate(parts).astype(np.float32)


def _loop(plan, u, z, w, p0, T, kind, seed, bf):
    from psvi.runtime import _lib as L

    lib = L.load()
    assert lib.psvi_debug_set(BF_OFF, 0 if bf else 1) == 0
    try:
        p = torch.tensor(p0, device=DEV)
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        e = plan.inner_loop(u, z, w, p, m, v, T, 1e-3, kind=kind, seed=seed)
        torch.cuda.synchronize()
    finally:
        lib.psvi_debug_set(BF_OFF, 0)
    return [x.cpu().numpy().astype(np.float64) for x in (e, p, m, v)]


SHAPES = [[(64, 40), (40, 40), (40, 2)],   # C3
          [(7, 5), (5, 3)],                 # n = 40, 18: one partial band each
          [(30, 33), (33, 2)],              # n = 1023, 68
          [(12, 20), (20, 4)]]              # n = 260, 84


@pytest.mark.parametrize("layers", SHAPES)
@pytest.mark.parametrize("kind", ["higher", "hypergrad"])
def test_bf_stream_loop_matches_fp32_stream_and_oracle(layers, kind):
    from psvi.runtime import InnerLoopPlan, randn_

    S, M, T, seed = 128, 24, 3, 77
    plan = InnerLoopPlan("fullcov", layers, S, M)
    assert plan.tiled_floats > 0
    rng, p0 = _case(layers, 3)
    u = rng.standard_normal((M, layers[0][0])).astype(np.float32)
    z = rng.integers(0, layers[-1][1], M).astype(np.int32)
    w = O.coreset_weights(0.3 * rng.standard_normal(M), 800).astype(np.float32)
    t = lambda a, d=torch.float32: torch.tensor(a, dtype=d, device=DEV)
    du, dz, dw = t(u), t(z, torch.int32), t(w)
    eb, pb, mb, vb = _loop(plan, du, dz, dw, p0, T, kind, seed, True)
    ef, pf, mf, vf = _loop(plan, du, dz, dw, p0, T, kind, seed, False)
    assert np.isfinite(pb).all() and np.isfinite(eb).all()
    # the float64 oracle on the same Philox draws; the fp32 streaming kernel's
    # loop beside it: both round differently, so each is held to the oracle
    draws = []
    for k in range(T):
        e = torch.empty(plan.eps_count, device=DEV)
        randn_(e, seed, k * plan.eps_stride)
        draws.append(e.cpu().numpy().astype(np.float64))
    o_e, _, o_traj, o_m, o_v = O.run_inner_loop("mvn", layers, p0, u, z, w, draws, S, 1e-3, kind)
    # (hypergrad's Adam steps sign(g) lr even for |g| at rounding level, so
    # after a step the fp32 trajectories themselves leave the float64 one by
    # more than 1e-5: each path is held to the oracle relative to the other)
    print(f"ELBO bf16 pieces {eb}, fp32 {ef}, oracle {o_e}")
    for k in range(T):
        assert abs(eb[k] - o_e[k]) <= 2 * abs(ef[k] - o_e[k]) + 1e-6 * abs(o_e[k]), k
    errs = {}
    for tag, (a_b, a_f, ref) in {"p": (pb, pf, o_traj[-1]), "m": (mb, mf, o_m),
                                 "v": (vb, vf, o_v)}.items():
        errs[tag] = (l2rel(a_b, ref), l2rel(a_f, ref))
    print(f"{layers} {kind}: l2 vs oracle (bf16 pieces, fp32): " +
          ", ".join(f"{k} {a:.1e} / {b:.1e}" for k, (a, b) in errs.items()))
    for k, (e_b, e_f) in errs.items():
        assert e_b < 2 * e_f + 1e-7, (k, e_b, e_f)
    assert errs["p"][0] < 1e-3
    # Adam's steps are ~ lr sign(g): entries whose gradient cancels to ~0 may
    # differ by up to ~2 lr per step between two fp32-level roundings
    assert np.abs(pb - pf).max() < 2 * T * 1e-3


def test_bf_stream_runs_in_the_loop():
    """The C3 loop in Philox mode takes the bf16-piece kernel (the plan carries
    the draw's planes) and is bitwise reproducible run to run."""
    from psvi.runtime import InnerLoopPlan

    layers, S, M = [(64, 40), (40, 40), (40, 2)], 128, 100
    plan = InnerLoopPlan("fullcov", layers, S, M)
    rng, p0 = _case(layers, 9)
    u = torch.tensor(rng.standard_normal((M, 64)).astype(np.float32), device=DEV)
    z = torch.tensor(rng.integers(0, 2, M).astype(np.int32), device=DEV)
    w = torch.full((M,), 8.0, device=DEV)
    a = _loop(plan, u, z, w, p0, 4, "higher", 5, True)
    b = _loop(plan, u, z, w, p0, 4, "higher", 5, True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    f = _loop(plan, u, z, w, p0, 4, "higher", 5, False)
    assert not np.array_equal(a[1], f[1]), "the bf16-piece kernel did not run"


@pytest.mark.parametrize("kind", ["higher", "hypergrad"])
def test_bf_stream_at_the_bench_inputs(kind):
    """The headline kernel at bench.py's own inputs: C3 (fn2 64-40-40-2, S =
    128, M = 100), bench.synthetic_inputs, the reference init (mean = 0, corr =
    0, sd = 1e-6: reference neural_net.py:425-428 with init_sd = 1e-6), the
    bench's Philox seed, T = 3 -- diagonal entries around 1e-6 beside corr
    entries around lr after the first step.  Held to the float64 oracle on the
    same draws as the generic shapes above."""
    import importlib.util
    import os

    from psvi.runtime import InnerLoopPlan, randn_

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    layers, S, M, T, seed = B.LAYERS, B.S_PER_GPU, B.M, 3, 20251015
    plan = InnerLoopPlan("fullcov", layers, S, M)
    du, dz, dw = B.synthetic_inputs(DEV)
    p0 = B.reference_init_params(layers, "cpu").numpy()
    eb, pb, mb, vb = _loop(plan, du, dz, dw, p0, T, kind, seed, True)
    ef, pf, mf, vf = _loop(plan, du, dz, dw, p0, T, kind, seed, False)
    assert np.isfinite(pb).all() and np.isfinite(eb).all()
    draws = []
    for k in range(T):
        e = torch.empty(plan.eps_count, device=DEV)
        randn_(e, seed, k * plan.eps_stride)
        draws.append(e.cpu().numpy().astype(np.float64))
    u, z, w = (x.cpu().numpy() for x in (du, dz, dw))
    o_e, _, o_traj, o_m, o_v = O.run_inner_loop("mvn", layers, p0, u.astype(np.float64), z,
                                                w.astype(np.float64), draws, S, 1e-3, kind)
    print(f"bench inputs {kind}: ELBO bf16 pieces {eb}, fp32 {ef}, oracle {o_e}")
    for k in range(T):
        assert abs(eb[k] - o_e[k]) <= 2 * abs(ef[k] - o_e[k]) + 1e-6 * abs(o_e[k]), k
        assert rel(eb[k], o_e[k]) < 1e-4, k      # the north star's ELBO bar
    for tag, (a_b, a_f, ref) in {"p": (pb, pf, o_traj[-1]), "m": (mb, mf, o_m),
                                 "v": (vb, vf, o_v)}.items():
        e_b, e_f = l2rel(a_b, ref), l2rel(a_f, ref)
        print(f"  {tag}: l2 vs oracle bf16 pieces {e_b:.2e}, fp32 {e_f:.2e}")
        assert e_b < 2 * e_f + 1e-7, (tag, e_b, e_f)
    assert l2rel(pb, o_traj[-1]) < 1e-4
    assert np.abs(pb - pf).max() < 2 * T * 1e-3


FOLD_OFF = 32  # PSVI_DBG_STREAM_FOLD_OFF


@pytest.mark.parametrize("layers", SHAPES)
@pytest.mark.parametrize("kind", ["higher", "hypergrad"])
def test_band_combine_in_kernel_equals_reduce(layers, kind):
    """The streaming update's in-kernel band combine (the last segment of a
    band to arrive adds the band's slots into x') against the separate
    mvn_fwd_reduce_kernel: bitwise equal (same sum order), T = 4 steps so the
    combined x' feeds three later steps, and run twice so the arrival counters
    are seen to reset."""
    from psvi.runtime import InnerLoopPlan
    from psvi.runtime import _lib as L

    lib = L.load()
    S, M, T, seed = 128, 24, 4, 31
    plan = InnerLoopPlan("fullcov", layers, S, M)
    rng, p0 = _case(layers, 5)
    t = lambda a, d=torch.float32: torch.tensor(a, dtype=d, device=DEV)
    u = t(rng.standard_normal((M, layers[0][0])).astype(np.float32))
    z = t(rng.integers(0, layers[-1][1], M).astype(np.int32), torch.int32)
    w = t(O.coreset_weights(0.3 * rng.standard_normal(M), 800).astype(np.float32))
    fold = _loop(plan, u, z, w, p0, T, kind, seed, True)
    fold2 = _loop(plan, u, z, w, p0, T, kind, seed, True)
    assert lib.psvi_debug_set(FOLD_OFF, 1) == 0
    try:
        red = _loop(plan, u, z, w, p0, T, kind, seed, True)
    finally:
        lib.psvi_debug_set(FOLD_OFF, 0)
    for a, b, c in zip(fold, fold2, red):
        assert np.array_equal(a, b)
        assert np.array_equal(a, c)
