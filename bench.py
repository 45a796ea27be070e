#!/usr/bin/env python3
"""Benchmark: ELBO inner-steps/sec of the coreset-weighted inner loop on MI355X.

Workload (BASELINE.json north star / SURVEY.md §8(d)): fn2 = make_fc2net
(VILinearMultivariateNormal 64 -> 40 -> 40 -> 2, full-covariance Gaussian
posterior, P = 4,730,326 parameters), M = 100 pseudopoints, S = 128 MC
samples PER GPU (C3 on one GPU; weak scaling: S = 128 N on N GPUs, the
N = 8 point being the C4 sample count).  One step = fresh eps draw (Philox),
reparameterised sampling x_s = mean + L eps_s, batched forward over S x M,
coreset-weighted NLL + KL, hand-derived backward, higher-Adam update of all
parameters.  One GPU: the K timed steps are ONE psvi_inner_loop call (the
product path: T chained steps, fresh Adam state, tiled corr/m/v, every
conversion and the first sample inside the timed region); the W warm-up
steps are a separate call.  Inputs are synthetic (make_synthetic-shaped: X ~ N(0, I_64),
labels ~ Bernoulli(sigmoid(5 sum x))), parameters at the reference init
(mean = 0, sd = softplus^-1(1e-6), corr = 0), N_data = 800, v = 0.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
         (a bare `bench.py --gpus N` starts that itself, as a child process)
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))

import torch  # noqa: E402

LAYERS = [(64, 40), (40, 40), (40, 2)]
S_PER_GPU = 128
M = 100
N_DATA = 800
LR = 1e-3
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
FP32_MFMA_PEAK_TFLOPS = 157.3  # v_mfma_f32_32x32x2_f32 dense peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (MI355X_MICROARCH.md, no sparsity)
BF_PIECES = 6  # bf16 piece products per fp32-faithful product (mvn_stream_bf_kernel)


def synthetic_inputs(device, seed=0):
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(M, LAYERS[0][0], generator=g)
    p = torch.sigmoid(5.0 * u.sum(1))
    z = (torch.rand(M, generator=g) < p).to(torch.int32)
    w = torch.full((M,), N_DATA / M)  # N * softmax(v = 0)
    return u.to(device), z.to(device), w.to(device)


def reference_init_params(n_layers_sizes, device):
    parts = []
    isp = math.log(math.expm1(1e-6))
    for din, dout in n_layers_sizes:
        n = din * dout + dout
        parts += [torch.zeros(n), torch.full((n,), isp), torch.zeros((n - 1) * (n - 2) // 2)]
    return torch.cat(parts).to(device)


def algorithmic_work_fused(S):
    """update kernel with the fused next-step sample (world == 1): the update's
    traffic plus eps_next read and x_next written, and a second triangular GEMM
    (x_next = L' eps_next)."""
    w = algorithmic_work(S)
    n_tot = sum(i * o + o for i, o in LAYERS)
    return dict(bytes=w["update"]["bytes"] + 8 * S * n_tot,
                flops=w["update"]["flops"] + w["sample"]["flops"])


def algorithmic_work(S, rows_frac=1.0, layers=LAYERS):
    """Per-launch algorithmic bytes / flops of the two dominant kernels
    (SURVEY.md §8(d)); rows_frac = this rank's share of the rows (nnz).
    update: p, m, v of the owned parameters read + written once (24 B each),
    G of the owned rows and eps (all columns) read once (4 B each), dL = G^T eps
    over the strict lower triangle (2 flops per MAC)."""
    n = [i * o + o for i, o in layers]
    n_tot = sum(n)
    nc = sum((k - 1) * (k - 2) // 2 for k in n)
    upd_bytes = 24 * (nc + 2 * n_tot) * rows_frac + 4 * S * n_tot * rows_frac + 4 * S * n_tot
    upd_flops = 2.0 * S * nc * rows_frac
    fwd_flops = 2.0 * S * nc * rows_frac
    fwd_bytes = 4 * (nc + 2 * n_tot) * rows_frac + 4 * S * n_tot + 4 * S * n_tot * rows_frac
    return dict(update=dict(bytes=upd_bytes, flops=upd_flops),
                sample=dict(bytes=fwd_bytes, flops=fwd_flops))


# The PMC summary the roofline's `traffic` is read from, and the commit whose
# bench it profiled (tools/round_session.sh pmc step: separate FETCH_SIZE /
# WRITE_SIZE rocprofv3 passes of this bench); reported as `traffic_source`
PMC_TRAFFIC = dict(file="profiles/r06_pmc_traffic.json", head="72299d8")


def pmc_traffic(kernels, path=os.path.join(ROOT, PMC_TRAFFIC["file"])):
    """HBM bytes per launch of the listed kernels (summed: the phase the
    roofline times) from the committed rocprofv3 PMC summary
    (tools/pmc_session.sh -> tools/pmc_report.py --json: separate FETCH_SIZE /
    WRITE_SIZE passes, gfx950 FETCH_SIZE x2 correction), or None.  Summary
    keys carry template arguments ("mvn_stream_kernel<4, 0, false, true>"):
    a listed name matches the key equal to it or starting with it and "<"."""
    try:
        d = json.load(open(path))["kernels"]
        tot = 0
        for k in kernels:
            key = next(x for x in d if x == k or x.startswith(k + "<"))
            tot += d[key]["hbm_bytes_per_launch"]
        return int(tot)
    except Exception:
        return None


def _cpu_model():
    try:
        return open("/proc/cpuinfo").read().split("model name")[1].split(":")[1].split("\n")[0].strip()
    except Exception:
        return "unknown"


def pin_cpu_threads():
    """the reference on all the cores this process may
    use -- the CPU affinity, capped by OMP_NUM_THREADS where the host sets it
    (the GPU box's CPU share; its affinity and os.cpu_count() report the whole
    machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    torch.set_num_threads(max(1, n))
    return torch.get_num_threads()


def log(msg):
    """Progress on stderr (the JSON line stays alone on stdout)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


class Runtime:
    """The process's place in the job and the device / collective plumbing the
    legs share: `dev`, `world`, `rank`, `comm` (psvi.runtime.sharded comm:
    RCCL through torch.distributed, or gloo with host staging for rehearsals
    on one GPU or on the CPU), `sync()`, `barrier()`, `max_over_ranks(x)`,
    `event()` (HIP events on the launch stream; wall-clock stand-ins on the
    CPU)."""

    def __init__(self, dev, world, rank, comm=None):
        self.dev, self.world, self.rank, self.comm = dev, int(world), int(rank), comm

    @property
    def cuda(self):
        return self.dev.type == "cuda"

    def sync(self):
        if self.cuda:
            torch.cuda.synchronize(self.dev)

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def max_over_ranks(self, x):
        if self.world == 1:
            return float(x)
        import torch.distributed as dist
        t = torch.tensor([float(x)], dtype=torch.float64,
                         device=self.dev if self.comm_on_device else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    @property
    def comm_on_device(self):
        return self.cuda and not getattr(self.comm, "host_staged", False)

    def timed(self, fn):
        """Wall seconds of fn() between synchronised barriers, the max over ranks."""
        self.sync()
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        fn()
        self.sync()
        self.barrier()
        self.sync()
        return self.max_over_ranks(time.perf_counter() - t0)

    def event(self):
        if self.cuda:
            return torch.cuda.Event(enable_timing=True)
        return _WallEvent()


class _WallEvent:
    """torch.cuda.Event's record / elapsed_time on the host clock (CPU rehearsal)."""

    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def cpu_baseline(budget_s=12.0):
    """Op-faithful torch CPU restatement of the reference inner step
    (oracle/cpu_reference.py) on a bounded number of C3 steps, with the
    anomaly-detection setting of the reference's driver
    (psvi/experiments/flow_psvi.py:50 turns it on) timed beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from cpu_reference import RefInnerStep, reference_init

    threads = pin_cpu_threads()
    torch.manual_seed(0)
    r = RefInnerStep("mvn", LAYERS, S_PER_GPU)
    p0 = reference_init("mvn", LAYERS)
    u, z, w = synthetic_inputs("cpu")
    z = z.float()
    r.run(p0, u, z, w, 2, LR)  # warm-up
    t0 = time.perf_counter()
    r.run(p0, u, z, w, 3, LR)
    per = (time.perf_counter() - t0) / 3
    n = max(3, min(60, int(budget_s / max(per, 1e-3))))
    t0 = time.perf_counter()
    r.run(p0, u, z, w, n, LR)
    dt = time.perf_counter() - t0
    # anomaly detection on (the reference driver's setting), a short sample
    na = max(2, min(10, n // 4))
    with torch.autograd.set_detect_anomaly(True, check_nan=True):
        t0 = time.perf_counter()
        r.run(p0, u, z, w, na, LR)
        dta = time.perf_counter() - t0
    model = _cpu_model()
    return dict(value=n / dt, unit="inner-steps/s", cores=threads, kind="port",
                anomaly_on_value=round(na / dta, 3),
                sample=(f"C3 fn2 S=128 M=100: one nested inner loop of {n} steps "
                        f"(autograd.grad create_graph=True + higher-Adam, anomaly off) "
                        f"in {dt:.1f} s on {threads} threads (torch.set_num_threads: the "
                        f"process's CPU affinity capped by OMP_NUM_THREADS) of {model}; "
                        f"anomaly_on_value: {na} steps "
                        f"with torch.autograd.set_detect_anomaly(True) as flow_psvi.py:50"))


def c2_timings(dev, steps=1000, cpu=True, reps=3):
    """Auxiliary line for BASELINE.json configs[1] (C2): fn = make_fcnet 2 -> 100
    -> 4 (one hidden layer, diagonal covariance) on a four_blobs-shaped
    problem, M = 50 pseudopoints, S = 32, psvi_inner_loop with in-library draws;
    and the op-faithful CPU step of the same model."""
    from psvi.runtime import InnerLoopPlan

    layers, S, M = [(2, 100), (100, 4)], 32, 50
    plan = InnerLoopPlan("meanfield", layers, S, M)
    g = torch.Generator().manual_seed(3)
    u = torch.randn(M, 2, generator=g)
    z = torch.randint(0, 4, (M,), generator=g)
    w = torch.full((M,), 1000.0 / M)
    params = _mf_init(layers).to(dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    ud, zd, wd = u.to(dev), z.to(dev, torch.int32), w.to(dev)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
    plan.inner_loop(ud, zd, wd, params, m, v, 20, LR, seed=1, ws=ws)
    torch.cuda.synchronize()
    rates = []
    for rep in range(reps):  # ~50 us steps: the median of a few 1000-step runs
        t0 = time.perf_counter()
        plan.inner_loop(ud, zd, wd, params, m, v, steps, LR, seed=2 + rep, ws=ws)
        torch.cuda.synchronize()
        rates.append(steps / (time.perf_counter() - t0))
    out = {"config": "C2 fn 2-100-4 meanfield, S=32, M=50 (four_blobs-shaped)",
           "gpu_inner_steps_per_s": round(sorted(rates)[len(rates) // 2], 1)}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from cpu_reference import RefInnerStep, reference_init

        r = RefInnerStep("mf", layers, S)
        p0 = reference_init("mf", layers)
        r.run(p0, u, z.float(), w, 3, LR)
        t0 = time.perf_counter()
        r.run(p0, u, z.float(), w, 30, LR)
        out["cpu_inner_steps_per_s"] = round(30 / (time.perf_counter() - t0), 2)
        out["cpu_threads"] = torch.get_num_threads()
    return out


def _mf_init(layers, init_sd=1e-3):
    parts = []
    isp = math.log(math.expm1(init_sd))
    g = torch.Generator().manual_seed(4)
    for din, dout in layers:
        bound = 1.0 / math.sqrt(din)
        parts += [(torch.rand(din * dout + dout, generator=g) * 2 - 1) * bound,
                  torch.full((din * dout + dout,), isp)]
    return torch.cat(parts)


C4 = dict(S=1024, M=200)


def make_sharded_loop(family, layers, S, M, rt):
    """This rank's ShardedInnerLoop (rows of L x samples for full-cov, samples
    for LeNet), collectives on rt.comm."""
    from psvi.runtime.sharded import ShardedInnerLoop
    return ShardedInnerLoop(family, layers, S, M, rt.world, rt.rank, device=rt.dev, comm=rt.comm)


def fn2_inputs(layers, M, dev, seed):
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(M, layers[0][0], generator=g)
    z = (torch.rand(M, generator=g) < torch.sigmoid(5.0 * u.sum(1))).to(torch.int32)
    return u.to(dev), z.to(dev), torch.full((M,), N_DATA / M, device=dev)


def sharded_steps(rt, loop, u, z, w, params, m, v, seed, k0, n, parts=None, ev=None, overlap=False):
    """n sharded inner steps (Adam steps k0 + 1 ..) -- ShardedInnerLoop.run:
    full-cov x all_to_all, network, G all_to_all, the update fused with the
    next step's sample, the next eps drawn by the network launch
    (LeNet: the samples' accumulator all-reduced per step).  The
    draws are the psvi_inner_loop stream at offset k0 * eps_stride.  ev: {step:
    4 events} around the exchanges + network and the update + sample."""
    stride = (loop.plan.eps_count + 3) // 4 * 4
    loop.run(u, z, w, params, m, v, n, LR, step0=k0 + 1, seed=seed, offset=k0 * stride,
             elbo_parts=None if parts is None else parts[k0:k0 + n], phase_events=ev,
             overlap=overlap)


def sharded_timed(rt, steps, warmup, layers, S, M, ev_every=5, seed=20251015, overlap=False):
    """K timed sharded inner steps of fn2 at (S, M) after W warm-up steps
    (ShardedInnerLoop.run: rows of L (whole 64-row bands) x samples sharded,
    two all_to_alls per step), the timed call continuing the warm-up's Philox
    stream and Adam steps.  Returns (elapsed s, the (warmup + steps) x 2 [NLL,
    KL] parts of this rank, per-phase ms from a separate 50-step call after the
    timed one, loop)."""
    loop = make_sharded_loop("fullcov", layers, S, M, rt)
    u, z, w = fn2_inputs(layers, M, rt.dev, 0)
    params = reference_init_params(layers, rt.dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    total = warmup + steps
    parts = torch.zeros(total, 2, dtype=torch.float64, device=rt.dev)
    sharded_steps(rt, loop, u, z, w, params, m, v, seed, 0, warmup, parts, overlap=overlap)
    elapsed = rt.timed(lambda: sharded_steps(rt, loop, u, z, w, params, m, v, seed,
                                             warmup, steps, parts, overlap=overlap))
    # the per-phase split: HIP events between the launches of a separate call
    # (outside the timed region), every ev_every-th of 50 steps
    nph = 50
    ev = {k: [rt.event() for _ in range(4)] for k in range(nph) if k % ev_every == 0}
    pp, mm, vv = params.clone(), m.clone(), v.clone()
    loop.run(u, z, w, pp, mm, vv, nph, LR, step0=total + 1, seed=seed + 1, phase_events=ev,
             overlap=overlap)
    rt.sync()
    ph = {"exchange+net": [], "update+sample": []}
    for e in ev.values():
        ph["exchange+net"].append(e[0].elapsed_time(e[1]))
        ph["update+sample"].append(e[1].elapsed_time(e[2]))
    avg_ms = {k: sum(x) / max(len(x), 1) for k, x in ph.items()}
    avg_ms["samples"] = len(ev)
    return elapsed, parts, avg_ms, loop


def weak_line(rt, steps, warmup, layers=LAYERS, s_per_gpu=S_PER_GPU, M=M):
    """Side line at N > 1: C3 shards weak-scaled (S = 128 N, M = 100), the same
    sharded step.  inner-steps/s of the whole job (one step = all S samples;
    not multiplied by N)."""
    S = s_per_gpu * rt.world
    elapsed, parts, _, loop = sharded_timed(rt, steps, warmup, layers, S, M)
    negelbo = loop.reduce_elbo(parts)
    return {"config": f"C3 shards x {rt.world}: fn2 full-cov S={S} ({s_per_gpu} per GPU), "
                      f"M={M} (weak scaling)",
            "inner_steps_per_s": round(steps / elapsed, 2),
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "elbo_finite": bool(torch.isfinite(negelbo).all().item())}


def c4_single_gpu(rt, steps=100, warmup=10, layers=LAYERS, S=None, M=None):
    """At N > 1, on rank 0 alone (the other ranks wait at the next barrier):
    C4 on ONE GPU of the same node in the same run (psvi_inner_loop, the
    c4_1gpu line of an N = 1 run), the denominator of the strong-scaling
    speed-up the N > 1 headline reports."""
    from psvi.runtime import InnerLoopPlan

    S, M = S or C4["S"], M or C4["M"]
    dev = rt.dev
    u, z, w = fn2_inputs(layers, M, dev, 5)
    params = reference_init_params(layers, dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    plan = InnerLoopPlan("fullcov", layers, S, M)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
    plan.inner_loop(u, z, w, params, m, v, warmup, LR, seed=11, ws=ws)
    rt.sync()
    t0 = time.perf_counter()
    plan.inner_loop(u, z, w, params, m, v, steps, LR, seed=12, ws=ws)
    rt.sync()
    dt = time.perf_counter() - t0
    return {"config": f"C4 fn2 full-cov S={S} M={M} on 1 GPU (rank 0's device, same run)",
            "inner_steps_per_s": round(steps / dt, 2), "ms_per_step": round(dt / steps * 1e3, 4)}


def step_flops(layers, S, M):
    """SURVEY.md section 8(d)'s algorithmic flops of one full-cov inner step:
    the two triangular GEMMs (x = L eps and dL = G^T eps, each sum n(n+1) S)
    and the network (forward, weight gradients, propagation below the head's
    input except into the first layer's input)."""
    n = [i * o + o for i, o in layers]
    io = [i * o for i, o in layers]
    return 2.0 * S * sum(k * (k + 1) for k in n) + 2.0 * S * M * (2 * sum(io) + sum(io[1:]))


def c4_timings(rt, steps=100, warmup=10, layers=LAYERS, S=C4["S"], M=C4["M"]):
    """Auxiliary line of an N = 1 run for BASELINE.json configs[3] (C4): fn2
    64-40-40-2 full-cov, S = 1024, M = 200 on one GPU (psvi_inner_loop) -- the
    denominator of the N > 1 headline, which is C4 itself (strong scaling)."""
    from psvi.runtime import InnerLoopPlan

    dev = rt.dev
    u, z, w = fn2_inputs(layers, M, dev, 5)
    params = reference_init_params(layers, dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    plan = InnerLoopPlan("fullcov", layers, S, M)
    ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
    elbo = torch.empty(steps, dtype=torch.float64, device=dev)
    plan.inner_loop(u, z, w, params, m, v, warmup, LR, seed=11, ws=ws)
    dt = rt.timed(lambda: plan.inner_loop(u, z, w, params, m, v, steps, LR, seed=12, ws=ws,
                                          elbo_out=elbo))
    return {"config": f"C4 fn2 full-cov S={S} M={M}, 1 GPU",
            "inner_steps_per_s": round(steps / dt, 2), "ms_per_step": round(dt / steps * 1e3, 4),
            "elbo_finite": bool(torch.isfinite(elbo[-1:]).all().item())}


def dp_timings(rt, steps=20, warmup=3, layers=LAYERS, S=C4["S"], M=C4["M"]):
    """The data-parallel alternative to the headline's row-sharded step
    (N > 1 only; SURVEY.md §8(e) frames the choice): every rank holds all of
    L, runs its S/N samples' inner objective and gradient on a world-1 plan
    (psvi_elbo_grad), ONE all-reduce of the 4.73 M-float gradient (18.9 MB)
    and the ELBO, then the same Adam step on every replica
    (SampleShardedPlan.inner_loop).  Same workload as the headline (C4)."""
    from psvi.runtime.sharded import SampleShardedPlan

    plan = SampleShardedPlan("fullcov", layers, S, M, rt.world, rt.rank, rt.comm)
    u, z, w = fn2_inputs(layers, M, rt.dev, 0)
    params = reference_init_params(layers, rt.dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    ws = plan.workspace(rt.dev)
    plan.inner_loop(u, z, w, params, m, v, warmup, LR, seed=3, ws=ws)
    dt = rt.timed(lambda: plan.inner_loop(u, z, w, params, m, v, steps, LR, step0=warmup + 1,
                                          seed=3, offset=warmup * plan.eps_stride, ws=ws))
    return {"config": f"C4 fn2 S={S} M={M} over {rt.world} GPUs: data parallel, one all-reduce "
                      f"of the {plan.param_count}-float gradient per step",
            "inner_steps_per_s": round(steps / dt, 2), "ms_per_step": round(dt / steps * 1e3, 4)}


def lenet_timings(rt, cpu=True, T=10, S=256, M=500, second_order=True):
    """Auxiliary line for BASELINE.json configs[4] (C5, make_lenet, S = 256,
    M = 500 MNIST-shaped synthetic pseudopoints, N = 60000; strong scaling:
    the same S at every N).  One GPU: psvi_inner_loop with in-library draws;
    N GPUs: the samples split over ranks (ShardedInnerLoop: one all-reduce of
    the accumulator per step).  Then C5's bilevel outer: one psvi_hvp (N > 1:
    psvi_hvp_partial + all-reduce, SampleShardedPlan) and one hyper_step
    (inner_it = 10, K = 30, CG_normaleq: /root/reference/psvi/hypergrad/
    hypergradients.py:199-244) through the reference-shaped PSVILearnV, sample-
    sharded at N > 1.  At N = 1 also one op-faithful CPU step of the same
    model (oracle/cpu_reference.py RefLenetStep)."""
    from psvi.models import LENET_LAYERS, make_lenet
    from psvi.runtime import InnerLoopPlan

    dev, world = rt.dev, rt.world
    torch.manual_seed(0)
    net = make_lenet(mc_samples=S, init_sd=0.05)
    p0 = torch.nn.utils.parameters_to_vector(net.parameters()).detach()
    g = torch.Generator().manual_seed(2)
    u = torch.randn(M, 1, 28, 28, generator=g)
    z = torch.randint(0, 10, (M,), generator=g)
    w = torch.full((M,), 60000.0 / M)
    params = p0.to(dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    ud, zd, wd = u.to(dev), z.to(dev, torch.int32), w.to(dev)
    if world == 1:
        plan = InnerLoopPlan("lenet", LENET_LAYERS, S, M)
        ws = torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev)
        elbo = torch.empty(T, dtype=torch.float64, device=dev)
        plan.inner_loop(ud, zd, wd, params, m, v, 2, LR, seed=1, ws=ws)
        dt = rt.timed(lambda: plan.inner_loop(ud, zd, wd, params, m, v, T, LR, seed=2, ws=ws,
                                              elbo_out=elbo))
        finite = bool(torch.isfinite(elbo).all().item())
    else:
        loop = make_sharded_loop("lenet", LENET_LAYERS, S, M, rt)
        parts = torch.zeros(2 + T, 2, dtype=torch.float64, device=dev)
        sharded_steps(rt, loop, ud, zd, wd, params, m, v, 1, 0, 2, parts)
        dt = rt.timed(lambda: sharded_steps(rt, loop, ud, zd, wd, params, m, v, 2, 2, T,
                                            parts))
        finite = bool(torch.isfinite(loop.reduce_elbo(parts[2:])).all().item())
    ms = dt / T * 1e3
    # 289.8 GFLOP of algorithmic work per C5 inner step
    # (106.6 forward + 183.2 backward); fp32 peak 157.3 TFLOP/s per GPU (VALU and MFMA alike)
    tfl = 289.8e9 / (ms * 1e-3) / 1e12
    out = {"config": f"C5 lenet S={S} M={M}, {world} GPU(s) (strong scaling: S/{world} per GPU)",
           "gpu_ms_per_inner_step": round(ms, 3), "gpu_inner_steps_per_s": round(1e3 / ms, 2),
           "elbo_finite": finite,
           "roofline": {"bound": "fp32 (VALU = MFMA peak)", "achieved": round(tfl, 2),
                        "peak": round(157.3 * world, 1), "unit": "TFLOP/s",
                        "frac": round(tfl / (157.3 * world), 4),
                        "algorithmic_gflop_per_step": 289.8}}
    if not second_order:
        return out
    from psvi.inference import PSVILearnV
    from psvi.runtime import randn_

    if world == 1:
        hplan = plan
    else:
        from psvi.runtime.sharded import SampleShardedPlan
        hplan = SampleShardedPlan("lenet", LENET_LAYERS, S, M, world, rt.rank, rt.comm)
    e = torch.empty(hplan.eps_count, device=dev)
    randn_(e, 5)
    vec = torch.randn(hplan.param_count, generator=g).to(dev)
    hplan.hvp(ud, zd, wd, e, params, vec)

    def hvps():
        for _ in range(3):
            hplan.hvp(ud, zd, wd, e, params, vec)
    out["gpu_hvp_ms"] = round(rt.timed(hvps) / 3 * 1e3, 3)
    net_d = make_lenet(mc_samples=S, init_sd=0.05).to(dev)
    ps = PSVILearnV(u=ud.clone().requires_grad_(True), z=zd.float(), N=60000, model=net_d,
                    mc_samples=S, device_id=dev.index, inner_it=10, seed=7, world=world,
                    rank=rt.rank, comm=rt.comm)
    ps.device = dev
    ps.register_elbos = False
    ps.setup_optimizers()
    xb = torch.randn(128, 1, 28, 28, generator=g).to(dev)
    yb = torch.randint(0, 10, (128,), generator=g).float().to(dev)
    ps.hyper_step(xb, yb, K=30)
    res = {}
    dt = rt.timed(lambda: res.setdefault("ll", ps.hyper_step(xb, yb, K=30)))
    out["gpu_hyper_step_T10_K30_ms"] = round(dt * 1e3, 1)
    out["hyper_step_loss_finite"] = bool(math.isfinite(res["ll"]))
    if cpu and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from cpu_reference import RefLenetStep

        t0 = time.perf_counter()
        RefLenetStep(S).run(p0, u, z.float(), w, 1, LR)
        out["cpu_ms_per_inner_step"] = round((time.perf_counter() - t0) * 1e3, 1)
        out["cpu_threads"] = torch.get_num_threads()
    return out


def trainer_timings(dev, cpu=True, cpu_T=2):
    """Auxiliary evidence, not the metric: the outer step of the trainers at C3
    (fn2 64-40-40-2, S = 128, M = 100 pseudopoints, a 128-row data batch, the
    reference init): wall ms per call of psvi_elbo forward + backward,
    psvi_hvp, one nested_step (inner_it = cpu_T and 100) and one hyper_step
    (inner_it = 100, K = 30), and the op-faithful CPU nested_step
    (oracle/cpu_reference.py, the reference's op sequence) at inner_it = cpu_T."""
    from psvi.inference import PSVILearnV
    from psvi.models import make_fc2net
    from psvi.runtime import randn_

    torch.manual_seed(0)
    model = make_fc2net(64, 40, 2, mc_samples=S_PER_GPU, init_sd=1e-6).to(dev)
    u, z, w = synthetic_inputs(dev)
    g = torch.Generator().manual_seed(1)
    xb = torch.randn(128, LAYERS[0][0], generator=g)
    yb = (torch.rand(128, generator=g) < torch.sigmoid(5.0 * xb.sum(1))).float()
    xb, yb = xb.to(dev), yb.to(dev)
    ps = PSVILearnV(u=u.clone().requires_grad_(True), z=z.float(), N=N_DATA, model=model,
                    mc_samples=S_PER_GPU, device_id=dev.index, inner_it=100, seed=7)
    ps.device = dev
    ps.register_elbos = False
    ps.setup_optimizers()

    def wall_ms(fn, n, warm=1):
        for _ in range(warm):  # plan creation, workspace and allocator growth
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / n * 1e3, 3)

    out = {}
    out["psvi_elbo_fwd_bwd_ms"] = wall_ms(lambda: ps.psvi_elbo(xb, yb).backward(), 20, warm=3)
    plan = ps._plan(model)
    pv = torch.nn.utils.parameters_to_vector(model.parameters()).detach().clone()
    vec = torch.randn(pv.numel(), device=dev)
    e = torch.empty(plan.eps_count, device=dev)
    randn_(e, 3)
    zi = z.to(torch.int32)
    out["psvi_hvp_ms"] = wall_ms(lambda: plan.hvp(u, zi, w, e, pv, vec), 20, warm=3)
    ps.inner_it = cpu_T
    out[f"nested_step_T{cpu_T}_ms"] = wall_ms(lambda: ps.nested_step(xb, yb), 3)
    ps.inner_it = 100
    out["nested_step_T100_ms"] = wall_ms(lambda: ps.nested_step(xb, yb), 1)
    out["hyper_step_T100_K30_ms"] = wall_ms(lambda: ps.hyper_step(xb, yb, K=30), 1)
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from cpu_reference import RefInnerStep, reference_init

        r = RefInnerStep("mvn", LAYERS, S_PER_GPU)
        p0 = reference_init("mvn", LAYERS)
        t0 = time.perf_counter()
        r.nested_step(p0, u.cpu(), z.float().cpu(), torch.zeros(M), N_DATA, xb.cpu(), yb.cpu(),
                      cpu_T, LR)
        out[f"cpu_nested_step_T{cpu_T}_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        out["cpu_threads"] = torch.get_num_threads()
    return out


def headline_prep(rt, args):
    """The headline's host-side set-up (plan, inputs, the reference init on the
    device, buffers), done before the C4 line so that no host stall (idle GPU)
    separates that line from the headline's warm-up and timed call."""
    from psvi.runtime import InnerLoopPlan

    dev = rt.dev
    plan = InnerLoopPlan("fullcov", LAYERS, S_PER_GPU, M)
    u, z, w = synthetic_inputs(dev)
    p_init = reference_init_params(LAYERS, dev)
    return dict(plan=plan, u=u, z=z, w=w, p_init=p_init,
                ws=torch.empty(plan.loop_ws_bytes, dtype=torch.uint8, device=dev),
                elbo_w=torch.empty(max(args.warmup, 1), dtype=torch.float64, device=dev),
                elbo_t=torch.empty(args.steps, dtype=torch.float64, device=dev))


def headline_world1(rt, args, prep=None):
    """The headline on one GPU: the K timed steps are ONE psvi_inner_loop call
    (T chained steps on tiled corr/m/v) that continues the W warm-up steps'
    call: same Philox stream (offset W * stride), Adam steps W + 1 .. W + K,
    and the loop's state left resident by the warm-up (psvi_inner_loop_ex
    KEEP / RESUME: the tiled state, step W's draw and sample).  The timed call
    does the full work of K steps -- each a network step with the next draw
    and an update with the next sample, the last one writing the packed
    arrays -- and its numbers are those of one call of W + K steps, bit for
    bit (tests/test_hip_loop_resident.py).  Per-phase HIP
    events (PSVI_DBG_LOOP_TIMING) on every 10th step of one more call after
    the timed one."""
    dev = rt.dev
    prep = prep or headline_prep(rt, args)
    plan, u, z, w, p_init = prep["plan"], prep["u"], prep["z"], prep["w"], prep["p_init"]
    ws, elbo_w, elbo_t = prep["ws"], prep["elbo_w"], prep["elbo_t"]
    params = p_init.clone()
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    eps_stride = (plan.eps_count + 3) // 4 * 4
    lib = plan.lib
    if args.warmup:
        # ~15 ms of the loop on scratch copies first: every kernel of the
        # timed call launched once (HIP loads a kernel's code at its first
        # launch; the warm-up call below ends in the fused update, the timed
        # one in the packed-out update) and the device at its working clock
        # (a fresh process's steps run 4 % slower at first and settle after
        # ~10 ms of work: profiles/r05_driver_cfg_probe.txt)
        scratch = [t.clone() for t in (params, m, v)]
        plan.inner_loop(u, z, w, *scratch, 200, LR, seed=1, ws=ws)
        del scratch
        plan.inner_loop(u, z, w, params, m, v, args.warmup, LR, seed=20251015,
                        elbo_out=elbo_w, ws=ws, keep=True)
    rt.sync()
    elapsed = rt.timed(lambda: plan.inner_loop(u, z, w, params, m, v, args.steps, LR,
                                               step0=args.warmup + 1, seed=20251015,
                                               offset=args.warmup * eps_stride,
                                               elbo_out=elbo_t, ws=ws))
    # the same K steps as a cold call (fresh Adam state and packed arrays: the
    # packed -> tiled conversion, the first draw and sample inside), as every
    # hyper_step / nested_step inner loop runs: the per-call fixed cost the
    # resumed headline leaves out
    pc, mc_, vc = p_init.clone(), torch.zeros_like(m), torch.zeros_like(v)
    cold_s = rt.timed(lambda: plan.inner_loop(u, z, w, pc, mc_, vc, args.steps, LR,
                                              seed=20251017, ws=ws))
    # the fixed cost itself from short cold calls (10 steps; the median of 5)
    # less 10 resumed steps: the K-step difference is within the run-to-run
    # noise of K steps
    short = []
    for rep in range(5):
        pc.copy_(p_init)
        mc_.zero_()
        vc.zero_()
        short.append(rt.timed(lambda: plan.inner_loop(u, z, w, pc, mc_, vc, 10, LR,
                                                      seed=20251018 + rep, ws=ws)))
    short.sort()
    cold = {"inner_steps_per_s": round(args.steps / cold_s, 2),
            "ms_per_step": round(cold_s / args.steps * 1e3, 5),
            "fixed_cost_us_per_call": round((short[2] - 10 * elapsed / args.steps) * 1e6, 1),
            "fixed_cost_method": "median wall time of 5 cold 10-step calls (host call included) "
                                 "less 10 resumed steps"}
    del pc, mc_, vc
    # the per-phase split from a separate call (its HIP event records on the
    # stream would otherwise sit inside the timed region): 100 steps, events
    # around the network and the update of every 10th -- 10 samples whatever
    # the timed call's K
    if lib.psvi_debug_set(8, 10):  # PSVI_DBG_LOOP_TIMING: every 10th step
        raise RuntimeError("psvi_debug_set(PSVI_DBG_LOOP_TIMING) failed")
    pp, mm, vv = params.clone(), torch.zeros_like(m), torch.zeros_like(v)
    plan.inner_loop(u, z, w, pp, mm, vv, 100, LR, seed=20251016, ws=ws)
    rt.sync()
    tm = (ctypes.c_double * 3)()
    if lib.psvi_debug_loop_timing(tm):
        raise RuntimeError("psvi_debug_loop_timing failed")
    lib.psvi_debug_set(8, 0)
    avg_ms = {"exchange+net": tm[0] * 1e-3, "update": tm[1] * 1e-3, "samples": int(tm[2])}
    return elapsed, elbo_t, avg_ms, plan.param_count, cold


def rows_fraction(loop, layers):
    """This rank's share of the strict-lower-triangle entries (nnz) of L."""
    n = [i * o + o for i, o in layers]
    info = loop.info[loop.rank]
    nnz_own = 0
    for (l, lo, cnt, _) in info["runs"]:
        nnz_own += sum(min(r, n[l] - 1) for r in range(lo, lo + cnt))
    return nnz_own / sum((k - 1) * (k - 2) // 2 for k in n)


def run(rt, args, shapes=None):
    """Everything after the process set-up; returns the JSON line's dict on
    rank 0 (None on the other ranks).  shapes: smaller stand-ins for the
    configs (CPU rehearsals of the N > 1 control flow under gloo,
    tests/test_bench_gloo.py); None = the BASELINE configs.

    N = 1: the headline is C3 (BASELINE configs[2]: fn2 S = 128, M = 100 on one
    GPU), with C4 on one GPU as the side line `c4_1gpu`.  N > 1: the headline
    is C4 (configs[3]: S = 1024, M = 200 over the N GPUs, strong scaling; one
    step is one step of all 1024 samples), with C4 on one GPU of the same run
    as `c4_1gpu` and the speed-up over it, and the weak-scaled C3 shards as
    the side line `weak`."""
    sh = dict(layers=LAYERS, s_per_gpu=S_PER_GPU, M=M, c4={}, c5={})
    sh.update(shapes or {})
    world, rank = rt.world, rt.rank
    c4sh = dict(layers=LAYERS, S=C4["S"], M=C4["M"])
    c4sh.update({k: sh["c4"][k] for k in ("layers", "S", "M") if k in sh["c4"]})
    # N = 1: the C4 line first, so that the headline's one short timed call
    # (K = 20 steps, ~1.4 ms, in the driver's run) starts on a GPU at its
    # working clocks rather than straight after process start-up
    c4 = None
    schedules = None
    if world == 1:
        prep = headline_prep(rt, args) if shapes is None else None
        if not args.no_c4:
            log("C4 line")
            c4 = c4_timings(rt, **sh["c4"])
        elapsed, parts, avg_ms, pcount, cold = headline_world1(rt, args, prep)
        elbo = parts
        S, Mh, layers = sh["s_per_gpu"], sh["M"], sh["layers"]
    else:
        S, Mh, layers = c4sh["S"], c4sh["M"], c4sh["layers"]
        # two complete schedules of the same step (ShardedInnerLoop.run): the
        # exchanges in series with the network, and overlapped with it (two
        # sample halves, each its own x -> network -> G chain, the second on a
        # side stream); the headline is the faster (the same pick on every
        # rank: the times are maxima over ranks), both are reported
        sched = {}
        for ov in (False, True):
            log(f"C4 headline over {world} ranks ({'overlapped' if ov else 'plain'} exchanges)")
            r_ = sharded_timed(rt, args.steps, args.warmup, layers, S, Mh, overlap=ov)
            sched["overlap" if ov else "plain"] = r_
        pick = min(sched, key=lambda k: sched[k][0])
        elapsed, parts, avg_ms, loop = sched[pick]
        schedules = {k: {"inner_steps_per_s": round(args.steps / v_[0], 2),
                         "ms_per_step": round(v_[0] / args.steps * 1e3, 4)} for k, v_ in sched.items()}
        schedules["headline"] = pick
        elbo = loop.reduce_elbo(parts)
        pcount = loop.plan.param_count
        cold = None
    finite = bool(torch.isfinite(elbo).all().item())
    steps_per_s = args.steps / elapsed
    value = steps_per_s  # one step = one inner step of ALL S samples, on every N
    if world == 1:
        upd_s = max(avg_ms["update"], 1e-9) * 1e-3
        # dominant kernel: the update with the fused next-step sample (its
        # band combine in the same launch since round 6)
        wk = algorithmic_work_fused(S)
        kname = ("mvn_stream_bf2_kernel (fused update + next-step sample with the band "
                 "combine, tiled state; fp32-faithful bf16-piece MFMA, eight waves)")
        kernels = {kname: dict(avg_us=avg_ms["update"] * 1e3, gbs=wk["bytes"] / upd_s / 1e9,
                               tflops=wk["flops"] / upd_s / 1e12),
                   "net_kernel (+ next-step Philox draw)": dict(avg_us=avg_ms["exchange+net"] * 1e3)}
    else:
        # dominant phase: the update (K-split streaming kernel at K = S) and
        # the next step's sample on this rank's rows (the segmented sample
        # kernel + its (row block, pass) reduce)
        work = algorithmic_work(S, rows_fraction(loop, layers), layers)
        wk = dict(bytes=work["update"]["bytes"] + work["sample"]["bytes"],
                  flops=work["update"]["flops"] + work["sample"]["flops"])
        upd_s = max(avg_ms["update+sample"], 1e-9) * 1e-3
        kname = "mvn_kstream_kernel + mvn_fwd_seg_kernel + reduce (update + next-step sample)"
        kernels = {kname: dict(avg_us=avg_ms["update+sample"] * 1e3,
                               gbs=wk["bytes"] / upd_s / 1e9, tflops=wk["flops"] / upd_s / 1e12),
                   "net_kernel(+exchange)": dict(avg_us=avg_ms["exchange+net"] * 1e3)}
    hbm_s, mfma_s = wk["bytes"] / (HBM_PEAK_GBS * 1e9), wk["flops"] / (FP32_MFMA_PEAK_TFLOPS * 1e12)
    if hbm_s >= mfma_s:
        roofline = dict(bound="hbm", achieved=round(wk["bytes"] / upd_s / 1e9, 1),
                        peak=HBM_PEAK_GBS, unit="GB/s")
    else:
        roofline = dict(bound="mfma", achieved=round(wk["flops"] / upd_s / 1e12, 2),
                        peak=FP32_MFMA_PEAK_TFLOPS, unit="TFLOP/s")
    roofline.update(frac=round(roofline["achieved"] / roofline["peak"], 4),
                    traffic=pmc_traffic(["mvn_stream_bf2_kernel"])
                    if world == 1 else None,
                    traffic_source=dict(PMC_TRAFFIC, measured_in_this_run=False,
                                        method="rocprofv3 --pmc FETCH_SIZE, then --pmc "
                                               "WRITE_SIZE (separate passes) over this bench; "
                                               "FETCH_SIZE x2 (gfx950 correction)")
                    if world == 1 else None,
                    timing_samples=avg_ms.get("samples"),
                    kernel=kname, algorithmic_bytes_per_launch=int(wk["bytes"]),
                    algorithmic_flops_per_launch=int(wk["flops"]),
                    floors_us=dict(hbm=round(hbm_s * 1e6, 2), mfma=round(mfma_s * 1e6, 2)),
                    # the instructions the dominant kernel issues: each fp32
                    # product as six bf16 piece products on v_mfma_f32_32x32x16_bf16
                    executed=dict(unit="TFLOP/s (bf16 MFMA, 6 piece products per fp32 product)",
                                  achieved=round(BF_PIECES * wk["flops"] / upd_s / 1e12, 1),
                                  peak=BF16_MFMA_PEAK_TFLOPS,
                                  frac=round(BF_PIECES * wk["flops"] / upd_s / 1e12
                                             / BF16_MFMA_PEAK_TFLOPS, 4)) if world == 1 else None,
                    kernels={k: {kk: round(vv, 2) for kk, vv in d.items()}
                             for k, d in kernels.items()})
    # the whole inner step's algorithmic work (C3: 2.682
    # GFLOP per step; C4: 23.54 GFLOP, split over the N GPUs) against the fp32
    # MFMA peak of the N GPUs -- the step's roofline fraction, beside the
    # dominant kernel's own above
    gflop = step_flops(layers, S, Mh) / 1e9
    step_floor_us = gflop * 1e9 / (FP32_MFMA_PEAK_TFLOPS * 1e12 * world) * 1e6
    step_roofline = dict(bound="mfma (fp32)", algorithmic_gflop_per_step=round(gflop, 3),
                         gpus=world, floor_us=round(step_floor_us, 2),
                         frac=round(step_floor_us / (elapsed / args.steps * 1e6), 4))
    log(f"headline: {steps_per_s:.1f} steps/s")
    weak = one = None
    if world > 1:
        log("weak-scaled C3 shards")
        weak = weak_line(rt, args.steps, args.warmup, layers=sh["layers"],
                         s_per_gpu=sh["s_per_gpu"], M=sh["M"])
        if rank == 0 and not args.no_c4:
            log("C4 on one GPU (rank 0)")
            one = c4_single_gpu(rt, **c4sh)
            one["speedup_of_headline"] = round(value / one["inner_steps_per_s"], 3)
        rt.barrier()
    dp = None
    if world > 1 and not args.no_dp:
        log("data-parallel alternative")
        dp = dp_timings(rt, **dict(c4sh, **sh.get("dp", {})))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("CPU baseline")
        cpu = cpu_baseline(args.cpu_budget)
    c2 = None
    if rank == 0 and world == 1 and not args.no_c2:
        log("C2 line")
        c2 = c2_timings(rt.dev, cpu=not args.no_cpu_baseline)
    trainers = None
    if rank == 0 and world == 1 and not args.no_trainers:
        log("trainers")
        trainers = trainer_timings(rt.dev, cpu=not args.no_cpu_baseline)
    lenet = None
    if not args.no_lenet:
        # every rank takes part at N > 1 (C5 is an 8-GPU config: samples sharded)
        log("C5 lenet")
        lenet = lenet_timings(rt, cpu=not args.no_cpu_baseline, **sh["c5"])
    rt.barrier()
    if rank != 0:
        return None
    if world == 1:
        workload = "C3 fn2 full-cov MLP 64-40-40-2, S=128, M=100, one GPU (BASELINE configs[2])"
        unit = "inner-steps/s (one step: all S=128 samples x M=100 pseudopoints)"
        par = "one GPU"
    else:
        workload = (f"C4 fn2 full-cov MLP 64-40-40-2, S={S}, M={Mh}, over {world} GPUs "
                    f"(BASELINE configs[3], strong scaling)")
        unit = f"inner-steps/s (one step: all S={S} samples x M={Mh} pseudopoints)"
        par = f"rows-of-L x samples sharded over {world}"
    return {
        "metric": "ELBO inner-steps/sec (S MC samples x M pseudopoints) at 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak" if world == 1 else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (make_synthetic-shaped X~N(0,I64), Bernoulli labels; reference init)",
        "config": {"workload": workload, "S_total": S, "M": Mh, "D": 64, "H": 40,
                   "C": 2, "params": pcount, "parallelism": par,
                   "comm": getattr(rt.comm, "name", None) if world > 1 else None,
                   "adam": "robust_higher DifferentiableAdam", "elbo_finite": finite,
                   "timed_call": ("continues the warm-up call (resident loop state)"
                                  if world == 1 and args.warmup else "continues the warm-up's "
                                  "Philox stream and Adam steps"),
                   "exchange_schedules": schedules},
        "cold_call": cold,
        "speedup_over_1gpu": None if world == 1 or one is None else one["speedup_of_headline"],
        "roofline": roofline,
        "step_roofline": step_roofline,
        "cpu_baseline": cpu,
        "c4_1gpu": c4 if world == 1 else one,
        "weak": weak,
        "dp_alternative": dp,
        "c2": c2,
        "trainers": trainers,
        "lenet_c5": lenet,
    }


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(n, argv, script=None):
    """Run `script argv` (default: this file) as n ranks of one node under
    torch.distributed.run in a CHILD process and return its exit status.
    The child's stdout is relayed line by line: a JSON object line (rank 0's
    result) to stdout, anything else (collective-library chatter) to stderr,
    so the JSON line stays alone on stdout.  Called before any GPU call: the
    parent only relays and waits."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={int(n)}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", script or os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
    log("launching: " + " ".join(cmd[1:]))
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        try:
            is_line = isinstance(json.loads(line), dict)
        except ValueError:
            is_line = False
        (sys.stdout if is_line else sys.stderr).write(line)
        (sys.stdout if is_line else sys.stderr).flush()
    return proc.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-lenet", action="store_true",
                    help="skip the auxiliary C5 (lenet) inner-step / HVP / hyper_step timing")
    ap.add_argument("--no-trainers", action="store_true",
                    help="skip the auxiliary outer-step (trainer) timings")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the auxiliary C4 (S=1024, M=200) strong-scaling line")
    ap.add_argument("--no-dp", action="store_true",
                    help="skip the N > 1 data-parallel alternative line (one all-reduce of "
                         "the full gradient per step)")
    ap.add_argument("--no-c2", action="store_true",
                    help="skip the auxiliary C2 (fn, S=32, M=50) line")
    ap.add_argument("--comm", choices=("rccl", "gloo"), default="rccl",
                    help="N > 1 collectives: RCCL (torch.distributed 'nccl'), or gloo with "
                         "host staging (a rehearsal of the N > 1 control flow, not a measurement)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on device 0 (rehearsing N ranks on a one-GPU box; "
                         "needs --comm gloo)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # a bare `bench.py --gpus N`: start the N ranks under torchrun as a
        # child process (this process never touches the GPU) and exit with
        # its status; rank 0's JSON line reaches stdout through the child
        raise SystemExit(relaunch(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.share_gpu and args.comm != "gloo":
        raise SystemExit("--share-gpu needs --comm gloo (RCCL takes one rank per GPU)")
    dev = torch.device("cuda", 0 if args.share_gpu else local)
    torch.cuda.set_device(dev)
    comm = None
    if world > 1:
        import torch.distributed as dist
        from psvi.runtime.sharded import HostStagedComm, TorchDistComm

        if args.comm == "rccl":
            dist.init_process_group("nccl", device_id=dev)
            comm = TorchDistComm()
        else:
            dist.init_process_group("gloo")
            comm = HostStagedComm()
    rt = Runtime(dev, world, rank, comm)
    out = run(rt, args)
    if out is not None:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
