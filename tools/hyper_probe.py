#!/usr/bin/env python3
"""C3 hyper_step (inner_it = 100, K = 30) and nested_step wall time, as
bench.py's trainer timings (the reference init, a 128-row data batch):
  python tools/hyper_probe.py [n] [hyper|nested]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    from psvi.inference import PSVILearnV
    from psvi.models import make_fc2net

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = make_fc2net(64, 40, 2, mc_samples=bench.S_PER_GPU, init_sd=1e-6).to(dev)
    u, z, w = bench.synthetic_inputs(dev)
    g = torch.Generator().manual_seed(1)
    xb = torch.randn(128, bench.LAYERS[0][0], generator=g)
    yb = (torch.rand(128, generator=g) < torch.sigmoid(5.0 * xb.sum(1))).float()
    xb, yb = xb.to(dev), yb.to(dev)
    ps = PSVILearnV(u=u.clone().requires_grad_(True), z=z.float(), N=bench.N_DATA, model=model,
                    mc_samples=bench.S_PER_GPU, device_id=0, inner_it=100, seed=7)
    ps.device = dev
    ps.register_elbos = False
    ps.setup_optimizers()
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, fn in (("hyper_step_T100_K30", lambda: ps.hyper_step(xb, yb, K=30)),
                     ("nested_step_T100", lambda: ps.nested_step(xb, yb))):
        if only and not name.startswith(only):
            continue
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"{name}: " + " ".join(f"{t:.2f}" for t in ts) + " ms", flush=True)


if __name__ == "__main__":
    main()
