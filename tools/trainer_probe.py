#!/usr/bin/env python3
"""Where the wall time of the C3 outer objective (psvi_elbo forward +
backward, bench.py's trainer line) goes: wall ms per call, device ms per call
(HIP events), and the host-side op table of one call (torch profiler, CPU
only).

  python tools/trainer_probe.py [calls]
  python tools/trainer_probe.py --trainers   (one nested_step and one hyper_step at
                                              inner_it 100, K 30: for a rocprofv3 trace)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from bench import LAYERS, N_DATA, S_PER_GPU, synthetic_inputs  # noqa: E402


def main():
    trainers = "--trainers" in sys.argv
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 20
    from psvi.inference import PSVILearnV
    from psvi.models import make_fc2net

    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = make_fc2net(64, 40, 2, mc_samples=S_PER_GPU, init_sd=1e-6).to(dev)
    u, z, w = synthetic_inputs(dev)
    g = torch.Generator().manual_seed(1)
    xb = torch.randn(128, LAYERS[0][0], generator=g)
    yb = (torch.rand(128, generator=g) < torch.sigmoid(5.0 * xb.sum(1))).float()
    xb, yb = xb.to(dev), yb.to(dev)
    ps = PSVILearnV(u=u.clone().requires_grad_(True), z=z.float(), N=N_DATA, model=model,
                    mc_samples=S_PER_GPU, device_id=0, inner_it=100, seed=7)
    ps.device = dev
    ps.register_elbos = False
    ps.setup_optimizers()
    if trainers:
        for name, f in (("nested_step", lambda: ps.nested_step(xb, yb)),
                        ("hyper_step", lambda: ps.hyper_step(xb, yb, K=30))):
            f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            print(f"{name} (inner_it 100): {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
        return
    fn = lambda: ps.psvi_elbo(xb, yb).backward()  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"psvi_elbo fwd+bwd: wall {t_wall / n * 1e3:.3f} ms/call, host issue "
          f"{t_host / n * 1e3:.3f} ms/call, stream span {e0.elapsed_time(e1) / n:.3f} ms/call")
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
