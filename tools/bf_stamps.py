#!/usr/bin/env python3
"""Per-phase shader clocks of the bf16-piece streaming update
(mvn_stream_bf2_kernel, DIAG build through PSVI_DBG_BF_STAMPS): one C3
inner loop in Philox mode (its first step runs the kernel), clocks summed over
each workgroup's tiles, median over workgroups, per tile.

  python3 tools/bf_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

PH = ["pmv+prefetch", "dL (+diag sums)", "barrier 1", "stage eps+G ld+diag adam", "x' st0",
      "x' st1", "flush", "barrier 2", "store eps'+split G"]


def main():
    layers, S, M = [(64, 40), (40, 40), (40, 2)], 128, 100
    plan = InnerLoopPlan("fullcov", layers, S, M)
    g = torch.Generator().manual_seed(0)
    u = torch.randn(M, 64, generator=g).cuda()
    z = (torch.rand(M, generator=g) < 0.5).to(torch.int32).cuda()
    w = torch.full((M,), 8.0, device="cuda")
    p = (torch.randn(plan.param_count, generator=g) * 0.01).cuda()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    lib = plan.lib
    nwg = 256
    st = torch.zeros(nwg * 16, dtype=torch.int64, device="cuda")
    plan.inner_loop(u, z, w, p.clone(), m.clone(), v.clone(), 3, 1e-3, seed=1)
    lib.psvi_debug_set_ptr(25, ctypes.c_void_p(st.data_ptr()))
    plan.inner_loop(u, z, w, p.clone(), m.clone(), v.clone(), 2, 1e-3, seed=1)
    torch.cuda.synchronize()
    lib.psvi_debug_set_ptr(25, None)
    a = st.cpu().numpy().reshape(nwg, 16).astype(np.float64)
    a = a[a[:, 9] > 0]
    tiles = a[:, 9]
    print(f"{len(a)} workgroups, tiles per workgroup median {np.median(tiles):.1f}")
    tot = 0.0
    for q, name in enumerate(PH):
        per = np.median(a[:, q] / tiles)
        tot += per
        print(f"  {name:28s} {per:8.0f} clocks / tile")
    print(f"  {'sum':28s} {tot:8.0f}")
    life = np.median(a[:, 10] - a[:, 13])
    print(f"  workgroup life {life:.0f} clocks ({life / np.median(tiles):.0f} / tile)")
    comb = a[:, 12]
    print(f"  band combines after the walk: {int((comb > 0).sum())} workgroups, clocks median "
          f"{np.median(comb[comb > 0]) if (comb > 0).any() else 0:.0f}, max {comb.max():.0f}")
    end = a[:, 10] - a[:, 13]
    k = np.argsort(end)[-8:]
    print("  the 8 longest-lived workgroups: life / combine clocks / tiles: " +
          ", ".join(f"{end[i]:.0f}/{comb[i]:.0f}/{tiles[i]:.0f}" for i in k))
    # by XCD (workgroup w on XCD w % 8) and by place in the run list (the
    # host deals XCD x the contiguous eighth x of the runs: w // 8 is the
    # run's place within its XCD's eighth)
    full = st.cpu().numpy().reshape(nwg, 16).astype(np.float64)
    life_all = full[:, 10] - full[:, 13]
    xcd = np.arange(nwg) % 8
    print("  life by XCD (median / max): " + ", ".join(
        f"{x}: {np.median(life_all[xcd == x]):.0f}/{life_all[xcd == x].max():.0f}" for x in range(8)))
    pos = np.arange(nwg) // 8
    q = np.array_split(np.arange(nwg // 8), 4)
    print("  life by place in the XCD's eighth (quarters, median / max): " + ", ".join(
        f"{i}: {np.median(life_all[np.isin(pos, qq)]):.0f}/{life_all[np.isin(pos, qq)].max():.0f}"
        for i, qq in enumerate(q)))
    # the phases of the slowest and the fastest workgroups (clocks summed over their tiles)
    order = np.argsort(life_all)
    hdr = "  " + " ".join(f"{n[:9]:>9s}" for n in PH) + "   combine      life tiles"
    for tag, idx in (("fastest", order[:6]), ("slowest", order[-10:])):
        print(f"  {tag}:")
        print(hdr)
        for i in idx:
            print("  " + " ".join(f"{full[i, qq]:9.0f}" for qq in range(len(PH))) +
                  f" {full[i, 12]:9.0f} {life_all[i]:9.0f} {full[i, 9]:5.0f}  wg {i}")
    rt = full[:, 11] - full[:, 11].min()
    print(f"  end (realtime, 100 MHz ticks from the first end): p50 {np.median(rt):.0f} max {rt.max():.0f}")


if __name__ == "__main__":
    main()
