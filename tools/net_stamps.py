#!/usr/bin/env python3
"""Per-phase shader-clock breakdown of the network kernel (s_memtime stamps,
diagnostics API), optionally under ablation masks.

  python tools/net_stamps.py [c3|c4] [abl,abl,...] [world rank]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
import torch  # noqa: E402

from psvi.runtime import InnerLoopPlan  # noqa: E402

CFG = {"c3": ([(64, 40), (40, 40), (40, 2)], 128, 100),
       "s512": ([(64, 40), (40, 40), (40, 2)], 512, 100),
       "c4": ([(64, 40), (40, 40), (40, 2)], 1024, 200),
       "w8": ([(64, 40), (40, 40), (40, 2)], 1024, 100)}


def report(name, t, abl, S):
    """Per role (workgroup rows s + S*role): median shader-clock ticks per phase."""
    t = t[: 2 * S]
    for role in (0, 1):
        r = t[role * S:(role + 1) * S]
        r = r[r[:, 0] != 0]
        if r.shape[0] == 0:
            continue
        d = (r.double() - r[:, 0:1].double())
        print(f"{name} abl={abl} role {role}: {r.shape[0]} workgroups; s_memtime ticks, median per phase:")
        prev = torch.zeros(r.shape[0], dtype=torch.float64)
        # phases (kernels_net.hip): 1 loads done, 2 row chain (forward, loss
        # head, gradient propagation) done, 3 weight gradients done, 12 end
        for k, nm in ((1, "loads"), (2, "row chain"), (3, "weight grads"), (12, "tail")):
            cur = d[:, k]
            print(f"  {nm:12s} {float((cur - prev).median()):10.0f}")
            prev = cur
        print(f"  total        {float(d[:, 12].median()):10.0f}  (max {float(d[:, 12].max()):.0f})")
        # wave 0's finer marks: 4 setup done, 5 load loop done (its own loads
        # landed and stored), 1 barrier; 6/7/8 forward layers of tile 0, 9 loss
        # head, 10 backward propagation, 2 barrier
        for k, nm in ((4, "setup"), (11, "loads issued"), (5, "load loop"), (1, "load barrier"), (6, "fwd l0"), (7, "fwd l1"),
                      (8, "fwd l2"), (9, "head"), (10, "bwd"), (2, "chain barrier")):
            print(f"    wave0 @ {nm:13s} {float(d[:, k].median()):8.0f}")
        sk = (r[:, 15].double() - r[:, 0].double())
        print(f"  wave launch skew (last wave start - workgroup start) median {float(sk.median()):.0f} max {float(sk.max()):.0f}")
        timeline(r, 13, 14)
        # workgroups that started late (a second round on their CU): warm caches
        st = r[:, 13].double()
        late = st > st.min() + 0.5 * (st.max() - st.min())
        if 0 < int(late.sum()) < r.shape[0]:
            for nm, msk in (("early", ~late), ("late", late)):
                dd = d[msk]
                print(f"  {nm:5s} starters ({int(msk.sum())}): loads {float(dd[:, 1].median()):.0f}"
                      f" fwd l0 {float((dd[:, 6] - dd[:, 1]).median()):.0f} fwd l1 {float((dd[:, 7] - dd[:, 6]).median()):.0f}"
                      f" fwd l2 {float((dd[:, 8] - dd[:, 7]).median()):.0f} total {float(dd[:, 12].median()):.0f}")


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
    abls = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 and sys.argv[2] else [0]
    # optional: world rank -- the network phase of one rank of a row-sharded
    # plan (x_recv from every source rank, gradients through the band table)
    world = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rank = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    layers, S, M = CFG[name]
    if world > 1 and name == "c3":
        S = 128 * world
    plan = InnerLoopPlan("fullcov", layers, S, M, world=world, rank=rank)
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    u = torch.randn(M, 64, generator=g).to(dev)
    z = torch.randint(0, 2, (M,), generator=g).to(torch.int32).to(dev)
    w = torch.full((M,), 8.0, device=dev)
    xs = torch.randn(plan.xrecv_count, generator=g).to(dev) * 0.1
    gs = torch.zeros(plan.xrecv_count, device=dev)
    nll = torch.zeros(1, dtype=torch.float64, device=dev)
    S = plan.s_local
    nblk = S * 8
    st = torch.zeros(nblk * 16, dtype=torch.int64, device=dev)
    for abl in abls:
        plan.lib.psvi_debug_set(1, abl)
        plan.mvn_net(u, z, w, xs, gs, nll)
        st.zero_()
        plan.lib.psvi_debug_set_ptr(2, ctypes.c_void_p(st.data_ptr()))
        plan.mvn_net(u, z, w, xs, gs, nll)
        torch.cuda.synchronize()
        plan.lib.psvi_debug_set_ptr(2, None)
        plan.lib.psvi_debug_set(1, 0)
        report(name, st.view(nblk, 16).cpu().clone(), abl, S)


if __name__ == "__main__":
    main()
