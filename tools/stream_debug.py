"""Where does the streaming update's next-step sample differ from the chunked
packed kernel's?  Prints the worst entries by (layer, row, sample) and per-slot
error summary.  Diagnostic only."""
import sys

import numpy as np
import torch

sys.path.insert(0, "blackbox-coresets-vi_amd")
sys.path.insert(0, "tests")
from psvi.runtime import InnerLoopPlan, _lib  # noqa: E402

layers = [(64, 40), (40, 40), (40, 2)] if len(sys.argv) < 2 else eval(sys.argv[1])
S = 128 if len(sys.argv) < 3 else int(sys.argv[2])
plan = InnerLoopPlan("fullcov", layers, S, 10)
rng = np.random.default_rng(11)
parts = []
for din, dout in layers:
    n = din * dout + dout
    parts += [0.1 * rng.standard_normal(n), rng.uniform(-5, -3, n),
              (0.15 / np.sqrt(n)) * rng.standard_normal((n - 1) * (n - 2) // 2)]
p0 = np.concatenate(parts).astype(np.float32)
t = lambda a: torch.tensor(a, device="cuda")
eps0 = t(rng.standard_normal(plan.eps_count).astype(np.float32))
eps1 = t(rng.standard_normal(plan.eps_count).astype(np.float32))
gs = t((0.05 * rng.standard_normal(plan.xshard_count)).astype(np.float32))
res = {}
for mode in ("packed", "stream", "chunked"):
    p = t(p0)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    x = torch.full((plan.xshard_count,), float("nan"), device="cuda")
    if mode == "packed":
        plan.mvn_update(eps0, gs, p, m, v, step=1, lr=1e-3, eps_next=eps1, x_next=x)
    else:
        _lib.load().psvi_debug_set(10, 1 if mode == "chunked" else 0)
        ts = plan.tiled_state()
        plan.tiled_convert(p, m, v, ts, True)
        plan.mvn_update_tiled(eps0, gs, p, m, v, ts, step=1, lr=1e-3, eps_next=eps1, x_next=x)
        plan.tiled_convert(p, m, v, ts, False)
        _lib.load().psvi_debug_set(10, 0)
    torch.cuda.synchronize()
    res[mode] = (p.cpu().numpy(), x.cpu().numpy())
n_tot = sum(i * o + o for i, o in layers)
for mode in ("stream", "chunked"):
    dp = np.abs(res[mode][0] - res["packed"][0]).max()
    X = res[mode][1].reshape(S, n_tot)
    R = res["packed"][1].reshape(S, n_tot)
    d = np.abs(X - R)
    print(f"{mode}: max|dp| {dp:.3e}  max|dx| {d.max():.3e}")
    col0 = 0
    for l, (i, o) in enumerate(layers):
        n = i * o + o
        dl = d[:, col0:col0 + n]
        rows = np.where(dl.max(0) > 1e-5)[0]
        samp = np.where(dl.max(1) > 1e-5)[0]
        print(f"  layer {l} n={n}: bad rows {len(rows)} (bands {sorted(set((rows // 64).tolist()))[:20]}), "
              f"bad samples {len(samp)} {samp[:10].tolist()}")
        col0 += n
