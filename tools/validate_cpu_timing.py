#!/usr/bin/env python3
"""Timing check of the CPU baseline: the op-faithful CPU port
(oracle/cpu_reference.py, bench.py's ``cpu_baseline`` leg) against the
reference's own inner loop, both on this container's host cores with the same
thread count, at C3 (fn2 64-40-40-2, S = 128, M = 100, the reference init).

The reference side runs ONLY here (it is not on the GPU box).  Each side
runs in a fresh child interpreter, the two alternating twice: the reference's
child has /root/reference on sys.path and not this repo (both packages are
called ``psvi``), as tools/gen_golden.py.  The reference child times the
nested-trainer inner loop -- ``innerloop_ctx`` + ``DifferentiableAdam.step``
on ``PSVI.inner_elbo`` (psvi_classes.py:549-555, robust_higher/optim.py);
the port's child ``cpu_reference.RefInnerStep.run`` on the same inputs --
as loops of ``--steps`` steps (each a fresh unroll: the per-step cost grows
with the unroll, autograd walking the whole retained graph), ``--reps``
loops per child after a warm-up loop; the medians are compared.

  python tools/validate_cpu_timing.py [--steps 10] [--threads 8] [--reps 3] [--tol 0.15]

Prints both rates and their ratio; exit status 1 when the port is more than
--tol (default 15 %) off the reference.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAYERS = [(64, 40), (40, 40), (40, 2)]
S, M, N, LR = 128, 100, 800, 1e-3


def _inputs():
    import torch

    g = torch.Generator().manual_seed(0)
    u = torch.randn(M, 64, generator=g)
    p = torch.sigmoid(5.0 * u.sum(1))
    z = (torch.rand(M, generator=g) < p).float()
    return u, z


def _child_ref(steps, threads, reps):
    sys.path = [p for p in sys.path if os.path.abspath(p) != ROOT]
    import types

    for name in ["arff", "faiss", "torchvision", "torchvision.transforms",
                 "torchvision.datasets"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torchvision"].datasets = sys.modules["torchvision.datasets"]
    import torch

    from psvi.inference.psvi_classes import PSVILearnV
    from psvi.models.neural_net import categorical_fn, make_fc2net
    from psvi.robust_higher import innerloop_ctx

    torch.set_num_threads(threads)
    torch.manual_seed(0)
    model = make_fc2net(64, 40, 2, mc_samples=S, init_sd=1e-6)
    u, z = _inputs()
    obj = PSVILearnV.__new__(PSVILearnV)  # inner_elbo reads u, z, v, N, f, distr_fn, learn_z
    obj.u, obj.z, obj.N = u, z, N
    obj.v = torch.zeros(M)
    obj.f, obj.distr_fn, obj.learn_z = torch.softmax, categorical_fn, False
    optim_net = torch.optim.Adam(list(model.parameters()), LR)

    def run(n):
        with innerloop_ctx(model, optim_net) as (fmodel, diffopt):
            for _ in range(n):
                diffopt.step(obj.inner_elbo(model=fmodel))

    return _time(run, steps, reps)


def _child_port(steps, threads, reps):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    from cpu_reference import RefInnerStep, reference_init

    torch.set_num_threads(threads)
    torch.manual_seed(0)
    step = RefInnerStep("mvn", LAYERS, S)
    p0 = reference_init("mvn", LAYERS)
    u, z = _inputs()
    w = torch.full((M,), N / M)  # N softmax(v = 0)
    return _time(lambda n: step.run(p0, u, z, w, n, LR), steps, reps)


def _time(run, steps, reps):
    """steps-step loops (each a fresh unroll, as a nested_step's inner loop),
    after one warm-up loop: the loops' rates in order"""
    run(steps)
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run(steps)
        out.append(steps / (time.perf_counter() - t0))
    return out


def _spawn(kind, a):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    if kind == "ref":
        env["PYTHONPATH"] = REF
    r = subprocess.run([sys.executable, "-B", os.path.abspath(__file__), "--child", kind,
                        "--steps", str(a.steps), "--threads", str(a.threads), "--reps",
                        str(a.reps)], env=env, cwd="/tmp", capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-2000:])
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("[")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--tol", type=float, default=0.15)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", choices=("ref", "port"))
    a = ap.parse_args()
    if a.child:
        fn = _child_ref if a.child == "ref" else _child_port
        print(json.dumps(fn(a.steps, a.threads, a.reps)), flush=True)
        return 0
    if not os.path.isdir(REF):
        print("the reference tree is not here: the timing check runs in the development "
              "container only", file=sys.stderr)
        return 2
    # each side in a fresh interpreter, alternating, medians of the loops' rates
    ref, port = [], []
    for _ in range(2):
        ref += _spawn("ref", a)
        port += _spawn("port", a)
    med = lambda x: sorted(x)[len(x) // 2]
    r, p = med(ref), med(port)
    ratio = p / r
    ok = abs(ratio - 1.0) <= a.tol
    print(json.dumps({"config": "C3 fn2 64-40-40-2 S=128 M=100", "threads": a.threads,
                      "steps_per_loop": a.steps, "loops": len(ref),
                      "reference_steps_per_s": round(r, 3), "port_steps_per_s": round(p, 3),
                      "reference_loops": [round(x, 3) for x in ref],
                      "port_loops": [round(x, 3) for x in port],
                      "port_over_reference": round(ratio, 3), "tolerance": a.tol,
                      "within_tolerance": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
