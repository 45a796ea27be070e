#!/usr/bin/env python3
"""Full-cov update kernel under the diagnostics API: per-workgroup shader-clock
stamps (start / first staging / step loop done / end, HW_ID, XCC_ID, summed
loop phases) and event timing under ablation masks (psvi_hip.h
PSVI_DBG_UPD_ABLATION: 1 G/eps loads, 2 MFMAs, 4 corr/m/v loads, 8 stores,
16 fused-sample MFMAs, 32 eps_next loads, 64 Adam math).

  python tools/upd_stamps.py [c3|c4] [abl,abl,...] [grad|adam|fused]

fused = the bench's kernel: tiled state + next-step sample.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

CFG = {"c3": ([(64, 40), (40, 40), (40, 2)], 128, 100),
       "c4": ([(64, 40), (40, 40), (40, 2)], 1024, 200)}


def timed(fn, iters=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def report(t, nblk):
    t = t.view(nblk, 16)
    start, staged, loop, end = (t[:, k].double() for k in range(4))
    hwid, xcc = t[:, 4], t[:, 5]
    cu = (xcc & 0xF) * 1000 + ((hwid >> 13) & 7) * 100 + ((hwid >> 12) & 1) * 20 + ((hwid >> 8) & 15)
    ucu, inv = torch.unique(cu, return_inverse=True)
    print(f"  distinct CUs: {len(ucu)}; chunks/CU max {int(torch.bincount(inv).max())}")
    parts = (("first stage", staged - start), ("step loop", loop - staged),
             ("tail", end - loop), ("chunk total", end - start))
    for nm, x in parts:
        q = torch.quantile(x.float(), torch.tensor([0.1, 0.5, 0.9]))
        print(f"  {nm:12s} p10 {q[0]:8.0f}  p50 {q[1]:8.0f}  p90 {q[2]:8.0f}")
    # per-XCD wall (s_memtime is per-XCD): first start -> last end
    xid = xcc & 0xF
    walls = [float(end[xid == x].max() - start[xid == x].min()) for x in torch.unique(xid)]
    print(f"  per-XCD wall ticks: min {min(walls):.0f} max {max(walls):.0f}")
    timeline(t, 12, 13)
    names = ("eps stage 1", "MFMA half 1", "eps stage 2", "MFMA half 2", "epilogue",
             "sample GEMM")
    ph = t[:, 6:12].double()
    if float(ph.sum()) > 0:
        print("  loop phases (median per workgroup, summed over its c-blocks):")
        for k, nm in enumerate(names):
            print(f"    {nm:12s} {float(ph[:, k].median()):8.0f}")


def timeline(t, c0, c1):
    """Chip timeline from the 100 MHz s_memrealtime stamps in slots c0 (start), c1 (end)."""
    st, en = t[:, c0].double(), t[:, c1].double()
    ok = (st > 0) & (en > 0)
    st, en = st[ok], en[ok]
    if st.numel() == 0:
        return
    t0 = float(st.min())
    q = lambda x: [float(v) for v in torch.quantile((x - 0).float(), torch.tensor([0.1, 0.5, 0.9, 1.0]))]
    s_ = q((st - t0) * 0.01)
    e_ = q((en - t0) * 0.01)
    d_ = q((en - st) * 0.01)
    print(f"  realtime (us from first start): start p10/50/90/max {s_[0]:.1f}/{s_[1]:.1f}/{s_[2]:.1f}/{s_[3]:.1f}"
          f"  end {e_[0]:.1f}/{e_[1]:.1f}/{e_[2]:.1f}/{e_[3]:.1f}  life {d_[0]:.1f}/{d_[1]:.1f}/{d_[2]:.1f}/{d_[3]:.1f}")


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    abls = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    mode = sys.argv[3] if len(sys.argv) > 3 else "grad"
    layers, S, M = CFG[name]
    plan = InnerLoopPlan("fullcov", layers, S, M)
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    eps = torch.randn(plan.eps_count, generator=g).to(dev)
    gs = torch.randn(plan.xshard_count, generator=g).to(dev) * 0.01
    params = (torch.randn(plan.param_count, generator=g) * 0.01).to(dev)
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    grad = torch.empty_like(params)
    kl = torch.zeros(1, dtype=torch.float64, device=dev)
    lib = plan.lib

    if mode == "fused":
        tstate = plan.tiled_state()
        plan.tiled_convert(params, m, v, tstate, True)
        eps_n = torch.randn(plan.eps_count, generator=g).to(dev)
        x_n = torch.empty(plan.xshard_count, device=dev)

    def run():
        if mode == "grad":
            plan.mvn_update(eps, gs, params, kl_out=kl, grad_out=grad)
        elif mode == "fused":
            plan.mvn_update_tiled(eps, gs, params, m, v, tstate, step=1, lr=0.0, kl_out=kl,
                                  eps_next=eps_n, x_next=x_n)
        else:
            plan.mvn_update(eps, gs, params, m, v, step=1, lr=0.0, kl_out=kl)

    # block count: stamp buffer sized generously, rows with start == 0 unused
    maxblk = 1 << 16
    st = torch.zeros(maxblk * 16, dtype=torch.int64, device=dev)
    for abl in abls:
        lib.psvi_debug_set(3, abl)
        us = timed(run)
        st.zero_()
        lib.psvi_debug_set_ptr(4, ctypes.c_void_p(st.data_ptr()))
        run()
        torch.cuda.synchronize()
        lib.psvi_debug_set_ptr(4, None)
        lib.psvi_debug_set(3, 0)
        t = st.view(maxblk, 16).cpu()
        nblk = int((t[:, 3] != 0).nonzero().max()) + 1
        print(f"{name} {mode} abl={abl}: {us:.1f} us/launch, {nblk} workgroups")
        report(t[:nblk].clone(), nblk)


if __name__ == "__main__":
    main()
