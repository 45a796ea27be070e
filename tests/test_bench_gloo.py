"""bench.py's N > 1 control flow on CPU: world_size 2 and 3 over gloo.

The driver's scaling run launches ``bench.py --gpus N`` under torchrun; this
test runs bench's own N > 1 code -- ``run()``: the C4 strong-scaling headline
and the weak-scaled C3 side line (``sharded_timed``), the one-GPU C4 reference
of rank 0 (stubbed: it is a HIP loop) and the C5
leg (``lenet_timings``: LeNet samples split over ranks) with their barriers,
max-over-ranks timing and the rank-0 JSON line -- over torch.distributed
(gloo, host-staged comm) on small stand-in shapes.  Only the HIP phases are
replaced by the oracle emulations of tests/test_sharded_gloo.py (same buffers,
same layouts) and the Philox draw by a seeded torch draw.  The sharded steps
bench times must reproduce the world-1 oracle inner loop bit for bit up to
fp32 (params, Adam state, negative ELBO)."""
import argparse
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FN2 = [(8, 6), (6, 3)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_draw(t, seed, offset):
    g = torch.Generator().manual_seed(int(seed) * 1000003 + int(offset))
    t.copy_(torch.randn(t.numel(), generator=g))


def _rank_main(rank, world, port, out):
    import sys
    for p in (os.path.join(ROOT, "blackbox-coresets-vi_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests"), ROOT):
        sys.path.insert(0, p)
    import bench
    import psvi_oracle as O
    from psvi.runtime.sharded import HostStagedComm, ShardedInnerLoop
    from test_sharded_gloo import _emulate_fullcov, _emulate_lenet

    def make_loop(family, layers, S, M, rt):
        loop = ShardedInnerLoop(family, layers, S, M, rt.world, rt.rank, device=rt.dev,
                                comm=rt.comm)
        if family == "fullcov":
            _emulate_fullcov(loop, O, layers, S, 1.0)
        else:
            _emulate_lenet(loop, O, S)
        loop.draw = _fake_draw
        return loop

    bench.make_sharded_loop = make_loop
    # the one-GPU C4 reference runs psvi_inner_loop on rank 0's device
    bench.c4_single_gpu = lambda rt, **kw: {"config": "stub", "inner_steps_per_s": 123.0,
                                            "ms_per_step": 8.13}
    bench.draw_eps = _fake_draw
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rt = bench.Runtime(torch.device("cpu"), world, rank, HostStagedComm())
        args = argparse.Namespace(steps=3, warmup=1, no_c4=False, no_cpu_baseline=True,
                                  no_c2=True, no_trainers=True, no_lenet=False, cpu_budget=1.0,
                                  no_dp=True)
        shapes = dict(layers=FN2, s_per_gpu=4, M=5,
                      c4=dict(layers=FN2, S=7, M=6, steps=2, warmup=1),
                      c5=dict(S=world + 1, M=3, T=2, second_order=False))
        line = bench.run(rt, args, shapes)
        # the steps bench times, against the world-1 oracle loop on the same draws
        layers, S, M = FN2, 4 * world, 5
        loop = make_loop("fullcov", layers, S, M, rt)
        u, z, w = bench.fn2_inputs(layers, M, rt.dev, 0)
        params = bench.reference_init_params(layers, rt.dev)
        g = torch.Generator().manual_seed(9)
        params += 0.05 * torch.randn(params.shape, generator=g)  # off the zero init
        p0 = params.clone()
        m, v = torch.zeros_like(params), torch.zeros_like(params)
        parts = torch.zeros(3, 2, dtype=torch.float64)
        bench.sharded_steps(rt, loop, u, z, w, params, m, v, 77, 0, 3, parts)
        negelbo = loop.reduce_elbo(parts)
        loop.gather_params(params, m, v)
        out.put((rank, line, p0.numpy(), params.numpy(), m.numpy(), v.numpy(),
                 negelbo.numpy(), u.numpy(), z.numpy(), w.numpy(), loop.plan.eps_count))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_multi_rank_control_flow(world):
    import psvi_oracle as O
    from golden_util import l2rel, rel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    line = res[0][1]
    assert all(r[1] is None for r in res[1:]), "only rank 0 prints the JSON line"
    # the headline at N > 1 is C4 itself (stand-in S = 7, M = 6), strong
    # scaling: value = timed steps / elapsed, not multiplied by N
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    assert line["config"]["S_total"] == 7 and line["config"]["M"] == 6
    assert line["config"]["workload"].startswith("C4") and "S=7, M=6" in line["config"]["workload"]
    assert line["config"]["elbo_finite"]
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert abs(line["value"] - 1e3 / line["ms_per_step"]) <= 1e-3 * line["value"] + 0.01
    assert line["config"]["comm"].startswith("gloo")
    ks = line["roofline"]["kernels"]
    assert set(ks) == {"mvn_kstream_kernel + mvn_fwd_seg_kernel + reduce (update + next-step sample)",
                       "net_kernel(+exchange)"}
    assert all(d["avg_us"] > 0 for d in ks.values())   # the sampled per-phase events
    one = line["c4_1gpu"]
    assert one["inner_steps_per_s"] == 123.0
    assert one["speedup_of_headline"] == round(line["value"] / 123.0, 3)
    assert line["speedup_over_1gpu"] == one["speedup_of_headline"]
    sch = line["config"]["exchange_schedules"]
    assert set(sch) == {"plain", "overlap", "headline"} and sch["headline"] in ("plain", "overlap")
    assert sch[sch["headline"]]["inner_steps_per_s"] == round(line["value"], 2)
    weak = line["weak"]
    assert weak["inner_steps_per_s"] > 0 and weak["elbo_finite"]
    assert "S=%d" % (4 * world) in weak["config"] and "M=5" in weak["config"]
    c5 = line["lenet_c5"]
    assert c5 is not None and c5["gpu_inner_steps_per_s"] > 0 and c5["elbo_finite"]
    assert "gpu_hvp_ms" not in c5      # second order: the GPU rehearsal covers it
    # the sharded steps: every rank ends with the world-1 oracle loop's state
    _, _, p0, params, m, v, negelbo, u, z, w, neps = res[0]
    S = 4 * world
    stride = (neps + 3) // 4 * 4
    draws = []
    for k in range(3):
        t = torch.empty(neps)
        _fake_draw(t, 77, k * stride)
        draws.append(t.numpy().astype(np.float64))
    o_elbo, _, o_traj, o_m, o_v = O.run_inner_loop("mvn", FN2, p0, u, z, w, draws, S, 1e-3,
                                                   "higher")
    for k in range(3):
        assert rel(negelbo[k], o_elbo[k]) < 1e-6, (k, negelbo[k], o_elbo[k])
    assert l2rel(params, o_traj[-1]) < 1e-6
    assert l2rel(m, o_m) < 1e-5 and l2rel(v, o_v) < 1e-5
    for r in res[1:]:
        assert np.array_equal(r[3], params), "replicas differ after gather_params"


def test_pmc_traffic_matches_template_keys(tmp_path):
    """bench.pmc_traffic sums the committed PMC summary's per-launch HBM bytes;
    the summary's keys carry template arguments, a listed name matches the key
    equal to it or starting with it and '<' (not a longer kernel name)."""
    import importlib.util
    import json

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    f = tmp_path / "t.json"
    f.write_text(json.dumps({"kernels": {
        "mvn_stream_kernel<4, 0, false, true>": {"hbm_bytes_per_launch": 100},
        "mvn_fwd_reduce_kernel": {"hbm_bytes_per_launch": 7},
        "mvn_fwd_reduce_kernel_x": {"hbm_bytes_per_launch": 1000}}}))
    assert b.pmc_traffic(["mvn_stream_kernel", "mvn_fwd_reduce_kernel"], str(f)) == 107
    assert b.pmc_traffic(["mvn_update_kernel"], str(f)) is None
    # the committed summary the bench line reads (the eight-wave bf16-piece
    # kernel, its band combine in the launch): at least the algorithmic bytes
    assert b.pmc_traffic(["mvn_stream_bf2_kernel"]) > 122379280
