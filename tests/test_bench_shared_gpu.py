"""bench.py at N > 1 with the real HIP kernels, rehearsed on one GPU.

The driver's scaling run (N = 2, 4, 8 under torchrun, one rank per GPU over
RCCL) is the first time the N > 1 bench meets hardware.  This test launches
the same command under torchrun with every rank on device 0 and the
collectives over gloo (``--comm gloo --share-gpu``, host-staged: RCCL takes one
rank per GPU), so every HIP path the scaling run takes -- the C4 headline
(strong scaling: rows of L x samples, two all_to_alls per step), the one-GPU
C4 reference of rank 0, the weak-scaled C3 shards, the data-parallel
alternative, the C5 leg (LeNet samples split over ranks, psvi_hvp_partial + all-reduce, a sharded
hyper_step) -- executes here at full size and must produce a finite rank-0 JSON
line with every key.  Timings from such a run mean nothing."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_bench_multi_rank_on_one_gpu(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"), "--gpus", str(world),
           "--steps", "5", "--warmup", "2", "--comm", "gloo", "--share-gpu",
           "--no-cpu-baseline"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    print(json.dumps(out)[:3000])
    assert out["n_gpus"] == world and out["config"]["S_total"] == 1024 and out["config"]["M"] == 200
    assert out["scaling"] == "strong" and out["config"]["workload"].startswith("C4")
    assert out["config"]["elbo_finite"] and out["value"] > 0
    assert abs(out["value"] - 1e3 / out["ms_per_step"]) <= 1e-3 * out["value"] + 0.01
    assert out["config"]["comm"].startswith("gloo")
    one = out["c4_1gpu"]
    assert one["inner_steps_per_s"] > 0
    assert out["speedup_over_1gpu"] == round(out["value"] / one["inner_steps_per_s"], 3)
    assert out["weak"]["elbo_finite"] and out["weak"]["inner_steps_per_s"] > 0
    c5 = out["lenet_c5"]
    assert c5["elbo_finite"] and c5["gpu_inner_steps_per_s"] > 0
    assert c5["gpu_hvp_ms"] > 0 and c5["hyper_step_loss_finite"]
    dp = out["dp_alternative"]   # the data-parallel alternative to the row-sharded step
    assert dp is not None and dp["inner_steps_per_s"] > 0 and "C4" in dp["config"]
