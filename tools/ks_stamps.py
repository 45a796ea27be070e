#!/usr/bin/env python3
"""One rank of the row-sharded full-cov step (world W, S samples): the
K-split update (mvn_kstream_kernel) and the sample kernel (mvn_fwd_kernel)
under the diagnostics API -- event timing and per-workgroup shader-clock
phase sums / 100 MHz timeline.

  python tools/ks_stamps.py [W] [rank] [S] [kstream workgroups, 0 = default] [grad]

"grad": the gradient mode (grad_out, no KL: the HVP's J^T G_dot) instead of Adam.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

LAYERS = [(64, 40), (40, 40), (40, 2)]


def timed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def q(x):
    v = torch.quantile(x.float(), torch.tensor([0.1, 0.5, 0.9, 1.0]))
    return f"p10 {v[0]:8.0f}  p50 {v[1]:8.0f}  p90 {v[2]:8.0f}  max {v[3]:8.0f}"


def timeline(rt0, rt1):
    t0 = rt0.min()
    s, e = (rt0 - t0) / 100, (rt1 - t0) / 100
    qq = lambda x: "/".join(f"{float(v):.1f}" for v in torch.quantile(x.float(), torch.tensor([0.1, 0.5, 0.9, 1.0])))
    print(f"  timeline (us): span {float(e.max()):.1f}; starts p10/50/90/max {qq(s)}; ends {qq(e)}; life {qq(e - s)}")


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    r = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    wgs = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    from psvi.runtime import _lib
    _lib.load().psvi_debug_set(21, wgs)
    plan = InnerLoopPlan("fullcov", LAYERS, S, 200, world=W, rank=r)
    g = torch.Generator().manual_seed(0)
    dev = "cuda"
    eps = torch.randn(plan.eps_count, generator=g).to(dev)
    params = (torch.randn(plan.param_count, generator=g) * 0.01).to(dev)
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    gs = (torch.randn(plan.xshard_count, generator=g) * 0.05).to(dev)
    xs = torch.empty(plan.xshard_count, device=dev)
    kl = torch.zeros(1, dtype=torch.float64, device=dev)
    lib = plan.lib
    maxblk = 1 << 14
    st = torch.zeros(maxblk * 16, dtype=torch.int64, device=dev)

    grad = len(sys.argv) > 5 and sys.argv[5] == "grad"
    gout = torch.zeros_like(params)
    if grad:
        upd = lambda: plan.mvn_update(eps, gs, params, grad_out=gout, include_kl=False)
    else:
        upd = lambda: plan.mvn_update(eps, gs, params, m, v, step=3, lr=1e-3, kind="higher", kl_out=kl)
    us = timed(upd)
    st.zero_()
    lib.psvi_debug_set_ptr(4, ctypes.c_void_p(st.data_ptr()))
    upd()
    torch.cuda.synchronize()
    lib.psvi_debug_set_ptr(4, None)
    t = st.view(maxblk, 16).cpu()
    nblk = int((t[:, 12] != 0).nonzero().max()) + 1
    t = t[:nblk].double()
    print(f"W{W} r{r} S{S}: K-split update {us:.1f} us/launch, {nblk} workgroups; "
          f"segments/wg mean {float(t[:, 6].mean()):.2f}, combines/wg mean {float(t[:, 7].mean()):.2f}")
    timeline(t[:, 13], t[:, 14])
    for k, nm in ((1, "first load"), (2, "passes"), (3, "hand-off"), (4, "partials"), (5, "epilogue")):
        print(f"  {nm:11s} {q(t[:, k])}")
    print(f"  {'total':11s} {q(t[:, 12] - t[:, 0])}")

    smp = lambda: plan.mvn_sample(eps, params, xs)
    us = timed(smp)
    st.zero_()
    lib.psvi_debug_set_ptr(7, ctypes.c_void_p(st.data_ptr()))
    smp()
    torch.cuda.synchronize()
    lib.psvi_debug_set_ptr(7, None)
    t = st.view(maxblk, 16).cpu()
    print(f"sample {us:.1f} us/launch (kernel + reduce)")
    if bool((t[:, 12] != 0).any()):  # the segmented kernel
        nblk = int((t[:, 12] != 0).nonzero().max()) + 1
        t = t[:nblk].double()
        print(f"  segmented: {nblk} workgroups, stages/wg mean {float(t[:, 6].mean()):.2f} max {float(t[:, 6].max()):.0f}")
        timeline(t[:, 13], t[:, 14])
        for k, nm in ((1, "first stage"), (2, "stages+mfma"), (3, "slot write")):
            print(f"  {nm:11s} {q(t[:, k])}")
        print(f"  {'total':11s} {q(t[:, 12] - t[:, 0])}")
        return
    nblk = int((t[:, 3] != 0).nonzero().max()) + 1
    t = t[:nblk].double()
    timeline(t[:, 6], t[:, 7])
    for nm, x in (("first stage", t[:, 1] - t[:, 0]), ("stages+mfma", t[:, 2] - t[:, 1]),
                  ("slot write", t[:, 3] - t[:, 2]), ("total", t[:, 3] - t[:, 0])):
        print(f"  {nm:11s} {q(x)}")


if __name__ == "__main__":
    main()
