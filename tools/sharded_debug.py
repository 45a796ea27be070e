#!/usr/bin/env python3
"""Debug the row-sharded full-cov step in one process: W ranks' phases with
the two all_to_alls as device copies, finiteness after every phase, and the
fused update + next-step sample against update-then-sample.

  python tools/sharded_debug.py [W] [S] [M] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = int(sys.argv[2]) if len(sys.argv) > 2 else 256
M = int(sys.argv[3]) if len(sys.argv) > 3 else 100
T = int(sys.argv[4]) if len(sys.argv) > 4 else 3
# optional debug switches "key=val,key=val" (include/psvi_hip.h PSVI_DBG_*)
DBG = [tuple(int(v) for v in kv.split("=")) for kv in sys.argv[5].split(",")] if len(sys.argv) > 5 else []
from bench import LAYERS, fn2_inputs, reference_init_params  # noqa: E402
from psvi.runtime import randn_  # noqa: E402
from psvi.runtime.sharded import ShardedInnerLoop  # noqa: E402


def offs(splits):
    o = [0]
    for x in splits:
        o.append(o[-1] + x)
    return o


dev = torch.device("cuda", 0)
loops = [ShardedInnerLoop("fullcov", LAYERS, S, M, W, r, device=dev) for r in range(W)]
for k, v in DBG:
    loops[0].plan.lib.psvi_debug_set(k, v)
    print(f"debug {k} = {v}", flush=True)
u, z, w = fn2_inputs(LAYERS, M, dev, 0)
p0 = reference_init_params(LAYERS, dev)
P = [p0.clone() for _ in range(W)]
Mm = [torch.zeros_like(p0) for _ in range(W)]
V = [torch.zeros_like(p0) for _ in range(W)]
e = [torch.empty(loops[0].plan.eps_count, device=dev) for _ in range(2)]
stride = loops[0].plan.eps_stride


def fin(name, t):
    ok = bool(torch.isfinite(t).all())
    if not ok:
        bad = (~torch.isfinite(t)).nonzero()
        print(f"  NONFINITE {name}: {bad.numel()} entries, first {bad[:5].flatten().tolist()}", flush=True)
    return ok


randn_(e[0], 5, 0)
for r in range(W):
    loops[r].phase_sample(e[0], P[r])
    fin(f"x_shard r{r} step0", loops[r].x_shard)
for t in range(T):
    ec, en = e[t & 1], e[(t + 1) & 1]
    randn_(en, 5, (t + 1) * stride)
    for r in range(W):
        parts = [loops[p].x_shard[offs(loops[p].x_in)[r]:offs(loops[p].x_in)[r + 1]] for p in range(W)]
        torch.cat(parts, out=loops[r].x_recv)
    for r in range(W):
        loops[r].phase_net(u, z, w)
        fin(f"g_send r{r} t{t}", loops[r].g_send)
        fin(f"nll r{r} t{t}", loops[r].parts)
    for r in range(W):
        parts = [loops[q].g_send[offs(loops[q].g_in)[r]:offs(loops[q].g_in)[r + 1]] for q in range(W)]
        torch.cat(parts, out=loops[r].g_shard)
    for r in range(W):
        # fused vs separate on copies
        pc, mc, vc = P[r].clone(), Mm[r].clone(), V[r].clone()
        loops[r].phase_update(ec, pc, mc, vc, t + 1, 1e-3, "higher")
        xs = loops[r].x_shard.clone()
        loops[r].phase_sample(en, pc)
        x_sep = loops[r].x_shard.clone()
        loops[r].x_shard.copy_(xs)
        loops[r].phase_update_sample(ec, P[r], Mm[r], V[r], t + 1, 1e-3, "higher", en)
        fin(f"params r{r} t{t}", P[r])
        fin(f"x_next r{r} t{t}", loops[r].x_shard)
        dp = (P[r] - pc).abs().max().item()
        dx = (loops[r].x_shard - x_sep).abs().max().item()
        print(f"t{t} r{r}: nll {loops[r].parts[0].item():.6g} kl {loops[r].parts[1].item():.6g} "
              f"fused-vs-separate params {dp:.3g} x {dx:.3g}", flush=True)
