"""experiment_driver with world / rank: the flow_psvi driver's PSVI run with
its MC samples split over two ranks (torchrun, every rank on device 0, gloo
collectives host-staged -- the rehearsal of a multi-GPU run on one GPU) gives
the same results as the world-1 run: both ranks identical (every step's
outer gradient and evaluation all-reduced), and equal to world 1 up to the
samples' fp32 summation order."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tools", "driver_rank.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lines(r):
    assert r.returncode == 0, r.stderr[-4000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("trainer", ["nested", "hyper"])
def test_driver_two_ranks_match_one(trainer):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    one = _lines(subprocess.run([sys.executable, SCRIPT, "--trainer", trainer], cwd=ROOT, env=env,
                                capture_output=True, text=True, timeout=300))
    assert len(one) == 1 and one[0]["world"] == 1
    two = _lines(subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
         "--master-addr=127.0.0.1", f"--master-port={_free_port()}", SCRIPT, "--share-gpu",
         "--trainer", trainer], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300))
    assert sorted(o["rank"] for o in two) == [0, 1] and all(o["world"] == 2 for o in two)
    a, b = two
    for k in ("accs", "nlls", "vs"):
        assert np.allclose(a[k], b[k], rtol=1e-6, atol=1e-7), k
    ref = one[0]
    print({k: (ref[k][-1] if k != "vs" else None, a[k][-1] if k != "vs" else None)
           for k in ("accs", "nlls")})
    assert np.allclose(a["nlls"], ref["nlls"], rtol=1e-3), (a["nlls"], ref["nlls"])
    assert np.abs(np.asarray(a["accs"]) - ref["accs"]).max() <= 0.01
    assert np.linalg.norm(np.subtract(a["vs"], ref["vs"])) <= 1e-3 * np.linalg.norm(ref["vs"])
