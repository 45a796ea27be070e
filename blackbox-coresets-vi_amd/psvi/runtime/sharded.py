"""Multi-GPU inner loop: one process per GPU, collectives over RCCL (xGMI).

The reference has no collectives (its only multi-GPU mode is a process pool of
independent jobs, psvi/experiments/flow-psvi-parallel.py:457-463).  Here one
inner step is split across ranks where the math allows it:

  full-cov (fn2):  rows of every layer's L (and the matching mean/sd/corr
      slices + Adam state) are sharded as whole 64-row bands balanced by their
      64 x 64 tile counts; MC samples are sharded in contiguous blocks.  Per
      step (ShardedInnerLoop.run fuses the update with the next step's sample
      and the network with the next step's eps draw):
        sample  x_shard[S][rows_r] = mean + L eps     (own rows, ALL samples)
        all_to_all  -> x_recv: own samples, all rows   (blocked by source rank)
        net     g_send = per-sample gradients          (own samples)
        all_to_all  -> g_shard: all samples, own rows
        update  dL = G^T eps + Adam for own rows (fused epilogue)
      Traffic per rank and step ~ 2 * S * n_tot * 4 B * (W-1)/W^2, independent
      of the 4.7 M-parameter gradient (never communicated).
  mean-field (fn, logreg): samples sharded, parameters replicated; one
      all-reduce of [NLL | sum_s dW | sum_s dW*eps] per step, then the KL +
      Adam update runs identically on every rank.

Every rank must pass the same eps (all S samples) -- in throughput mode each
rank draws it from the same Philox stream, so it never crosses the wire.
"""
import torch

from .engine import InnerLoopPlan, adam_update_, randn_


def check_exchange(out, inp, out_splits, in_splits, world):
    """The all_to_all contract, asserted before every exchange so that a
    mismatch fails loudly on the first scaling run instead of moving the
    wrong bytes: one split per rank, non-negative, summing to each buffer's
    numel; both buffers contiguous float32 on one device."""
    for name, t, sp in (("out", out, out_splits), ("inp", inp, in_splits)):
        if len(sp) != world:
            raise ValueError(f"all_to_all {name}: {len(sp)} splits for world {world}")
        if any(int(x) < 0 for x in sp):
            raise ValueError(f"all_to_all {name}: negative split in {list(sp)}")
        if sum(int(x) for x in sp) != t.numel():
            raise ValueError(f"all_to_all {name}: splits sum to {sum(sp)}, buffer has "
                             f"{t.numel()} elements")
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"all_to_all {name}: contiguous float32 expected (got {t.dtype}, "
                             f"contiguous={t.is_contiguous()})")
    if out.device != inp.device:
        raise ValueError(f"all_to_all: buffers on {out.device} and {inp.device}")


def check_exchange_list(outs, ins, world):
    """all_to_all_list's contract: one block per rank on each side, contiguous
    float32, one device."""
    for name, ts in (("outs", outs), ("ins", ins)):
        if len(ts) != world:
            raise ValueError(f"all_to_all {name}: {len(ts)} blocks for world {world}")
        for t in ts:
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"all_to_all {name}: contiguous float32 blocks expected")
    devs = {t.device for t in list(outs) + list(ins)}
    if len(devs) > 1:
        raise ValueError(f"all_to_all: blocks on {devs}")


class TorchDistComm:
    """Collectives on torch.distributed (backend 'nccl' == RCCL on ROCm)."""

    name = "rccl"
    host_staged = False

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._checked = set()

    def all_to_all(self, out, inp, out_splits, in_splits):
        # the contract is checked once per (buffers, splits): the sharded loop
        # exchanges the same buffers every step (host time per step matters at
        # N = 8, where a step is ~0.1 ms of device work)
        key = (out.data_ptr(), inp.data_ptr(), out.numel(), inp.numel(), tuple(out_splits),
               tuple(in_splits))
        if key not in self._checked:
            check_exchange(out, inp, out_splits, in_splits, self.world)
            self._checked.add(key)
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def all_to_all_list(self, outs, ins):
        """One block per peer as lists of contiguous tensors (views into the
        exchange buffers; grouped point-to-point sends and receives on RCCL).
        Backends without a list all_to_all (gloo) go through one staged
        all_to_all_single."""
        key = tuple((t.data_ptr(), t.numel()) for t in list(outs) + list(ins))
        if key not in self._checked:
            check_exchange_list(outs, ins, self.world)
            self._checked.add(key)
        if self.dist.get_backend(self.group) == "nccl":
            self.dist.all_to_all(list(outs), list(ins), group=self.group)
            return
        src = torch.cat([t.reshape(-1) for t in ins])
        dst = torch.empty(sum(t.numel() for t in outs), dtype=torch.float32, device=src.device)
        self.dist.all_to_all_single(dst, src, [t.numel() for t in outs], [t.numel() for t in ins],
                                    group=self.group)
        o = 0
        for t in outs:
            t.copy_(dst[o:o + t.numel()].view(t.shape))
            o += t.numel()

    def all_reduce(self, t):
        # a strided view (e.g. one output of a plan's fused result) is reduced
        # through a contiguous copy and written back in place
        if not t.is_contiguous():
            c = t.contiguous()
            self.dist.all_reduce(c, group=self.group)
            t.copy_(c)
            return
        self.dist.all_reduce(t, group=self.group)


class HostStagedComm(TorchDistComm):
    """The same collectives over a gloo process group with device tensors
    staged through host memory (gloo has no device all_to_all).  For
    rehearsing the N > 1 control flow -- several ranks sharing one GPU, or
    CPU tensors -- not for measurements: RCCL (TorchDistComm) is the product
    transport."""

    name = "gloo (host-staged)"
    host_staged = True

    def all_to_all(self, out, inp, out_splits, in_splits):
        check_exchange(out, inp, out_splits, in_splits, self.world)
        o = torch.empty(out.shape, dtype=out.dtype)
        self.dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
        out.copy_(o)

    def all_to_all_list(self, outs, ins):
        check_exchange_list(outs, ins, self.world)
        src = torch.cat([t.reshape(-1).cpu() for t in ins])
        dst = torch.empty(sum(t.numel() for t in outs), dtype=torch.float32)
        self.dist.all_to_all_single(dst, src, [t.numel() for t in outs], [t.numel() for t in ins],
                                    group=self.group)
        o = 0
        for t in outs:
            t.copy_(dst[o:o + t.numel()].view(t.shape))
            o += t.numel()

    def all_reduce(self, t):
        h = t.cpu()
        self.dist.all_reduce(h, group=self.group)
        t.copy_(h)


def layer_rows(info, l):
    """(rows, cols): the rows of layer l a rank owns (ascending) and their
    columns in its x / g shard, from shard_info's runs (numpy int arrays)."""
    import numpy as np

    rows, cols = [], []
    for (ll, lo, cnt, col) in info["runs"]:
        if ll == l:
            rows.append(np.arange(lo, lo + cnt))
            cols.append(np.arange(col, col + cnt))
    if not rows:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    return np.concatenate(rows), np.concatenate(cols)


class ShardedInnerLoop:
    def __init__(self, family, layers, S, M, world, rank, prior_sd=1.0, device="cuda",
                 comm=None):
        self.plan = InnerLoopPlan(family, layers, S, M, prior_sd=prior_sd, world=world,
                                  rank=rank)
        self.family, self.world, self.rank = family, world, rank
        self.comm = comm
        self.device = device
        self.info = [self.plan.shard_info(r) for r in range(world)]
        f32 = dict(dtype=torch.float32, device=device)
        if family == "fullcov":
            self.x_shard = torch.empty(self.plan.xshard_count, **f32)
            self.x_recv = torch.empty(self.plan.xrecv_count, **f32)
            self.g_send = torch.empty(self.plan.xrecv_count, **f32)
            self.g_shard = torch.empty(self.plan.xshard_count, **f32)
            me = self.info[rank]
            # all_to_all split sizes (elements)
            self.x_in = [q["s_count"] * me["rows"] for q in self.info]
            self.x_out = [me["s_count"] * p["rows"] for p in self.info]
            self.g_in = list(self.x_out)
            self.g_out = list(self.x_in)
        else:
            self.acc = torch.empty(self.plan.acc_count, **f32)
        # [local NLL, local KL] of the last step (fp64 accumulators)
        self.parts = torch.zeros(2, dtype=torch.float64, device=device)

    # -------------------------------------------------------------- phases
    def phase_sample(self, eps, params):
        self.plan.mvn_sample(eps, params, self.x_shard)

    def phase_net(self, u, z, w, draw=None):
        """draw = (eps_out, seed, offset): the next step's global eps drawn by
        the same launch (psvi_mvn_phase_net_draw)."""
        self.parts.zero_()
        if draw is None:
            self.plan.mvn_net(u, z, w, self.x_recv, self.g_send, self.parts[0:1])
        else:
            self.plan.mvn_net(u, z, w, self.x_recv, self.g_send, self.parts[0:1], draw=draw)

    def phase_update(self, eps, params, m, v, step, lr, kind, grad_out=None):
        self.plan.mvn_update(eps, self.g_shard, params, m, v, step=step, lr=lr, kind=kind,
                             kl_out=self.parts[1:2], grad_out=grad_out)

    def phase_update_sample(self, eps, params, m, v, step, lr, kind, eps_next):
        """The update fused with the next step's sample into x_shard
        (psvi_mvn_phase_update_sample)."""
        self.plan.mvn_update(eps, self.g_shard, params, m, v, step=step, lr=lr, kind=kind,
                             kl_out=self.parts[1:2], eps_next=eps_next, x_next=self.x_shard)

    def draw(self, out, seed, offset):
        """eps of the global layout from the Philox stream (psvi_randn)."""
        randn_(out, seed, offset)

    # ---------------------------------------------------------------- step
    def step(self, u, z, w, eps, params, m, v, step, lr, kind="higher", elbo_parts=None):
        """One inner step on this rank.  elbo_parts (2 doubles, optional)
        receives this rank's [NLL, KL] contributions; their sum over ranks
        (see reduce_elbo) is the negative inner ELBO."""
        if self.family == "fullcov":
            self.phase_sample(eps, params)
            self.comm.all_to_all(self.x_recv, self.x_shard, self.x_out, self.x_in)
            self.phase_net(u, z, w)
            self.comm.all_to_all(self.g_shard, self.g_send, self.g_out, self.g_in)
            self.phase_update(eps, params, m, v, step, lr, kind)
            if elbo_parts is not None:
                elbo_parts.copy_(self.parts)
        else:
            self.parts.zero_()
            self.plan.mf_accumulate(u, z, w, eps, params, self.acc, self.parts[0:1])
            self.comm.all_reduce(self.acc)
            # replicated update; the KL value is counted on rank 0 only
            self.plan.mf_update(self.acc, params, m, v, step=step, lr=lr, kind=kind,
                                kl_out=self.parts[1:2] if self.rank == 0 else None)
            if elbo_parts is not None:
                elbo_parts.copy_(self.parts)

    # ------------------------------------------------- overlapped exchanges
    def _halves(self, q):
        """Rank q's local samples split in two: [(lo, count), (lo, count)]."""
        n = self.info[q]["s_count"]
        a = (n + 1) // 2
        return [(0, a), (a, n - a)]

    def _views(self):
        """Per half h, the exchange blocks as views: x send / receive, G send /
        receive (one per peer, in rank order; see run(overlap=True))."""
        if getattr(self, "_hv", None) is not None:
            return self._hv
        W, me = self.world, self.rank
        S = self.plan.S
        rows = [q["rows"] for q in self.info]
        s_off = [q["s_offset"] for q in self.info]
        S_loc = self.info[me]["s_count"]
        xs = self.x_shard.view(S, rows[me])
        gs = self.g_shard.view(S, rows[me])
        base = [0]
        for q in range(W):
            base.append(base[-1] + S_loc * rows[q])
        hv = []
        for h in range(2):
            lo_me, n_me = self._halves(me)[h]
            xo, xi, go, gi = [], [], [], []
            for q in range(W):
                lo_q, n_q = self._halves(q)[h]
                # x: my rows of q's half-h samples out; q's rows of my half-h samples in
                xi.append(xs[s_off[q] + lo_q:s_off[q] + lo_q + n_q].reshape(-1))
                blk = self.x_recv[base[q]:base[q + 1]].view(S_loc, rows[q])
                xo.append(blk[lo_me:lo_me + n_me].reshape(-1))
                # G: q's rows of my half-h samples out; my rows of q's half-h samples in
                gblk = self.g_send[base[q]:base[q + 1]].view(S_loc, rows[q])
                gi.append(gblk[lo_me:lo_me + n_me].reshape(-1))
                go.append(gs[s_off[q] + lo_q:s_off[q] + lo_q + n_q].reshape(-1))
            hv.append(dict(xo=xo, xi=xi, go=go, gi=gi, lo=lo_me, n=n_me))
        self._hv = hv
        return hv

    def phase_net_half(self, u, z, w, h, draw=None):
        """The network on half h of this rank's samples (psvi_mvn_phase_net_part),
        adding to parts[0]; draw: part h of 2 of the next step's eps."""
        hv = self._views()[h]
        self.plan.mvn_net(u, z, w, self.x_recv, self.g_send, self.parts[0:1], draw=draw,
                          samples=(hv["lo"], hv["n"]), draw_part=(h, 2))

    def _net_half(self, u, z, w, h, nxt):
        self.phase_net_half(u, z, w, h, draw=nxt if (nxt is not None and self.x_recv.is_cuda)
                            else None)

    def _net_half_launcher(self, u, z, w):
        """psvi_mvn_phase_net_part for the two halves with the argument checks
        done once: f(h, eps_out or None, seed, offset, stream handle) -- the
        overlap schedule's per-step host cost (two launches where the plain
        schedule has one)."""
        import ctypes

        from ._lib import check
        plan = self.plan
        hv = self._views()
        for t, d in ((u, None), (z, torch.int32), (w, None)):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("u / z / w must be contiguous device tensors")
        plan_checked = (u.numel() == plan.M * plan.in_features and z.numel() == plan.M
                        and z.dtype == torch.int32 and w.numel() == plan.M)
        if not plan_checked:
            raise ValueError("u / z / w do not match the plan")
        lib, fn = plan.lib, plan.lib.psvi_mvn_phase_net_part
        base = (plan.handle, u.data_ptr(), z.data_ptr(), w.data_ptr(), self.x_recv.data_ptr(),
                self.g_send.data_ptr(), self.parts.data_ptr())
        rng = [(hv[h]["lo"], hv[h]["n"]) for h in range(2)]
        n_eps = plan.eps_count

        def launch(h, out, seed, offset, stream):
            lo, n = rng[h]
            rc = fn(*base, lo, n, out.data_ptr() if out is not None else None,
                    n_eps if out is not None else 0, seed, offset, h, 2, ctypes.c_void_p(stream))
            if rc:
                check(rc, "psvi_mvn_phase_net_part")
        return launch

    def run(self, u, z, w, params, m, v, T, lr, kind="higher", step0=1, seed=0, offset=0,
            elbo_parts=None, phase_events=None, overlap=False):
        """T chained inner steps on this rank with in-library Philox draws
        (psvi_inner_loop's stream: step t at offset + t * eps_stride of the
        global layout, identical on every rank, so eps never crosses the wire).

        Full-cov schedule per step t (x_shard holds x_t on entry):
          x all_to_all -> network (which also draws eps_{t+1}: Philox, split
          over its workgroups after their gradients) -> G all_to_all
          update of t fused with the next step's sample: Adam on the rank's rows
            (K-split streaming kernel at K = S > 128), then x_{t+1} = mean' +
            L' eps_{t+1} on those rows (psvi_mvn_phase_update_sample)
        The first step's x_0 is sampled before the loop; the last step
        samples nothing.  elbo_parts (T, 2) float64 receives this rank's [NLL,
        KL] per step (reduce_elbo sums them).  phase_events: optional {t:
        [4 events]} recorded around the exchanges + network, the update and
        the sample (diagnostics; they sit between launches).

        overlap=True (full-cov): the rank's samples in two halves A, B, each
        with its own chain of exchange -> network -> exchange (list
        all_to_alls of per-peer views, no copies): A on the compute stream, B
        on a side stream, issued x(A), x(B), net(A), net(B), G(A), G(B) -- the
        order a serialising transport (one RCCL stream) runs them in -- so x(B)
        travels during net(A), G(A) during net(B), and the two network halves
        (half the workgroups each) run side by side; the update waits for both
        chains.  The per-sample work and the exchanged bytes are those of the
        plain schedule (the same parameters bit for bit; the NLL's atomic adds
        come in another order); the draw is split between the two network
        launches, which share no plan scratch (net_part_ok)."""
        T = int(T)
        if T <= 0:
            return
        dev = params.device
        stride = self.plan.eps_stride
        if self.family != "fullcov":
            e = torch.empty(self.plan.eps_count, device=dev)
            for t in range(T):
                self.draw(e, seed, offset + t * stride)
                self.step(u, z, w, e, params, m, v, step0 + t, lr, kind=kind,
                          elbo_parts=None if elbo_parts is None else elbo_parts[t])
            return
        if getattr(self, "_eps2", None) is None or self._eps2[0].device != dev:
            self._eps2 = [torch.empty(self.plan.eps_count, device=dev) for _ in range(2)]
        e_cur, e_nxt = self._eps2
        cuda = e_cur.is_cuda
        self.draw(e_cur, seed, offset)
        self.phase_sample(e_cur, params)
        if overlap and getattr(self.plan, "net_part_ok", True):
            # (plans whose pseudopoint chunks use per-chunk gradient slots take
            # whole network launches: the plain schedule)
            self._run_overlap(u, z, w, params, m, v, T, lr, kind, step0, seed, offset, elbo_parts,
                              phase_events, e_cur, e_nxt, stride, cuda)
            return
        for t in range(T):
            ev = phase_events.get(t) if phase_events else None
            last = t + 1 == T
            nxt = None if last else (e_nxt, seed, offset + (t + 1) * stride)
            if nxt is not None and not cuda:
                self.draw(*nxt)  # host tensors: the draw on its own
            if ev: ev[0].record()
            self.comm.all_to_all(self.x_recv, self.x_shard, self.x_out, self.x_in)
            # e_nxt was last read by the previous update, earlier on this stream
            if cuda and nxt is not None:
                self.phase_net(u, z, w, draw=nxt)
            else:
                self.phase_net(u, z, w)
            self.comm.all_to_all(self.g_shard, self.g_send, self.g_out, self.g_in)
            if ev: ev[1].record()
            if last:
                self.phase_update(e_cur, params, m, v, step0 + t, lr, kind)
            else:
                self.phase_update_sample(e_cur, params, m, v, step0 + t, lr, kind, e_nxt)
            if ev: ev[2].record()
            if elbo_parts is not None:
                elbo_parts[t].copy_(self.parts)
            e_cur, e_nxt = e_nxt, e_cur
            if ev: ev[3].record()
        self._eps2 = [e_cur, e_nxt]

    def _run_overlap(self, u, z, w, params, m, v, T, lr, kind, step0, seed, offset, elbo_parts,
                     phase_events, e_cur, e_nxt, stride, cuda):
        import contextlib

        hv = self._views()
        cs = None
        if cuda:
            if getattr(self, "_cs", None) is None:
                self._cs = torch.cuda.Stream(device=e_cur.device)
            cs = self._cs
            main = torch.cuda.current_stream(e_cur.device)
        side = (lambda: torch.cuda.stream(cs)) if cuda else contextlib.nullcontext
        a2a = self.comm.all_to_all_list
        net = self._net_half_launcher(u, z, w) if cuda else None
        if cuda:
            hm, hs = main.cuda_stream, cs.cuda_stream
        for t in range(T):
            ev = phase_events.get(t) if phase_events else None
            last = t + 1 == T
            nxt = None if last else (e_nxt, seed, offset + (t + 1) * stride)
            if nxt is not None and not cuda:
                self.draw(*nxt)
            if ev: ev[0].record()
            self.parts.zero_()
            if cuda:
                cs.wait_stream(main)        # x_shard from the last update, parts zeroed
            a2a(hv[0]["xo"], hv[0]["xi"])                                # x(A)
            with side():
                a2a(hv[1]["xo"], hv[1]["xi"])                            # x(B)
            if cuda:
                d = (None, 0, 0) if nxt is None else nxt
                net(0, d[0], d[1], d[2], hm)                             # net(A)
                net(1, d[0], d[1], d[2], hs)                             # net(B), side stream
            else:
                self._net_half(u, z, w, 0, nxt)
                self._net_half(u, z, w, 1, nxt)
            a2a(hv[0]["go"], hv[0]["gi"])                                # G(A)
            with side():
                a2a(hv[1]["go"], hv[1]["gi"])                            # G(B)
            if cuda:
                main.wait_stream(cs)        # chain B done
            if ev: ev[1].record()
            if last:
                self.phase_update(e_cur, params, m, v, step0 + t, lr, kind)
            else:
                self.phase_update_sample(e_cur, params, m, v, step0 + t, lr, kind, e_nxt)
            if ev: ev[2].record()
            if elbo_parts is not None:
                elbo_parts[t].copy_(self.parts)
            e_cur, e_nxt = e_nxt, e_cur
            if ev: ev[3].record()
        self._eps2 = [e_cur, e_nxt]

    def reduce_elbo(self, elbo_parts):
        """elbo_parts (T, 2) stacked per step -> negative ELBO per step (all ranks)."""
        t = elbo_parts.clone()
        self.comm.all_reduce(t)
        return t.sum(-1)

    def owned_mask(self, r=None):
        """Boolean mask of the parameter entries owned by rank r (full-cov)."""
        r = self.rank if r is None else r
        mask = torch.zeros(self.plan.param_count, dtype=torch.bool, device=self.device)
        if self.family != "fullcov":
            mask[:] = r == 0
            return mask
        info = self.info[r]
        po = [0]
        for din, dout in self.plan.layers:
            n = din * dout + dout
            po.append(po[-1] + 2 * n + (n - 1) * (n - 2) // 2)
        for (l, lo, cnt, _) in info["runs"]:
            din, dout = self.plan.layers[l]
            n = din * dout + dout
            hi = lo + cnt
            mask[po[l] + lo:po[l] + hi] = True
            mask[po[l] + n + lo:po[l] + n + hi] = True
            clo = min(lo, n - 1)
            chi = min(hi, n - 1)
            mask[po[l] + 2 * n + clo * (clo - 1) // 2:po[l] + 2 * n + chi * (chi - 1) // 2] = True
        return mask

    def gather_params(self, *tensors):
        """Make every rank's copy of params (and Adam state) identical by
        summing the owned slices (end of an inner loop, not per step)."""
        mask = self.owned_mask()
        for t in tensors:
            t.mul_(mask)
            self.comm.all_reduce(t)


# ---------------------------------------------------------------------------
# Sample-sharded outer objective (PSVI.psvi_elbo, psvi_classes.py:447-486)
# ---------------------------------------------------------------------------
def sample_split(S, world):
    """Contiguous sample blocks [(offset, count)] per rank (first S % world
    ranks one larger), the split of the inner-loop plans."""
    base, rem = divmod(S, world)
    out, o = [], 0
    for r in range(world):
        c = base + (r < rem)
        out.append((o, c))
        o += c
    return out


def local_eps(family, layers, S, s_off, s_cnt, eps):
    """The noise of samples [s_off, s_off + s_cnt) out of the global eps (the
    reference draw order, include/psvi_hip.h) laid out for a world-1 plan of
    s_cnt samples.  LeNet's last layer is one shared draw (unbatched VILinear)."""
    parts, o = [], 0
    for l, (din, dout) in enumerate(layers):
        nw = din * dout
        if family == "fullcov":
            n = nw + dout
            parts.append(eps[o:o + S * n].view(S, n)[s_off:s_off + s_cnt].reshape(-1))
            o += S * n
        elif family == "lenet" and l == len(layers) - 1:
            parts.append(eps[o:o + nw + dout])
            o += nw + dout
        else:
            parts.append(eps[o:o + S * nw].view(S, nw)[s_off:s_off + s_cnt].reshape(-1))
            o += S * nw
            parts.append(eps[o:o + S * dout].view(S, dout)[s_off:s_off + s_cnt].reshape(-1))
            o += S * dout
    assert o == eps.numel(), (o, eps.numel())
    return torch.cat(parts).contiguous()


def outer_coefficients(terms):
    """Per-sample terms (S, 3) float64 [pseudo NLL sum, data NLL sum, KL-ish
    nkl] of ALL samples -> (loss, cp, cd, ck): the psvi_elbo value and the
    derivatives of the loss w.r.t. each sample's pseudo, data and nkl terms.
    loss = sum_s W_s (data_s - pseudo_s) - mean_s lw_s with lw = nkl - pseudo,
    W = softmax(lw) over samples (psvi_classes.py:463-481)."""
    pseudo, data, nkl = terms[:, 0], terms[:, 1], terms[:, 2]
    S = terms.shape[0]
    lw = nkl - pseudo
    W = torch.softmax(lw, 0)
    a = data - pseudo
    abar = (W * a).sum()
    loss = abar - lw.mean()
    ck = W * (a - abar) - 1.0 / S
    cp = -W - ck
    return loss, cp, W, ck


def pack_coef(cp, cd, ck, s_off, s_cnt):
    """[rowcoef (s_cnt, 2) | ck (s_cnt) | sck] for psvi_outer_elbo_grad_coef."""
    sl = slice(s_off, s_off + s_cnt)
    rc = torch.stack([cp[sl], cd[sl]], 1).reshape(-1)
    return torch.cat([rc, ck[sl], ck[sl].sum().reshape(1)]).float().contiguous()


class ShardedOuter:
    """The outer objective with the S samples split over ranks.  Pass 1: each
    rank's world-1 plan of its own samples gives the per-sample terms
    (psvi_outer_elbo_grad, sample_out only); one all-reduce assembles all S;
    the softmax over samples is formed on every rank identically (float64);
    pass 2 (psvi_outer_elbo_grad_coef) gives this rank's partial gradients,
    summed by one all-reduce.  Parameters, pseudo/data rows and the global eps
    are replicated; the per-sample towers are not."""

    def __init__(self, family, layers, S, M, world, rank, prior_sd=1.0, device="cuda",
                 comm=None, plan=None):
        """plan: a world-1 plan of this rank's samples (built when None)."""
        self.family, self.layers, self.S, self.M = family, list(layers), S, M
        self.world, self.rank, self.comm, self.device = world, rank, comm, device
        self.split = sample_split(S, world)
        self.s_off, self.s_cnt = self.split[rank]
        if self.s_cnt < 1:
            raise ValueError(f"rank {rank} has no samples (S={S}, world={world})")
        self.plan = plan if plan is not None else InnerLoopPlan(family, layers, self.s_cnt, M,
                                                                prior_sd=prior_sd)
        self.prior_sd = prior_sd
        self._full = None

    def local_terms(self, n_pseudo, x_all, z_all, w_all, eps, params):
        """Pass 1 -> (eps_local, terms (s_cnt, 3) float64)."""
        e = local_eps(self.family, self.layers, self.S, self.s_off, self.s_cnt, eps)
        o = self.plan.outer_elbo_grad(n_pseudo, x_all, z_all, w_all, e, params, grad=False,
                                      grad_w=False, sample_stats=True)
        return e, o["samples"][:, :3].contiguous()

    def local_grads(self, n_pseudo, x_all, z_all, w_all, eps_local, params, cp, cd, ck,
                    grad_u=True, grad_w=True):
        """Pass 2: this rank's partial gradients for global coefficients."""
        coef = pack_coef(cp, cd, ck, self.s_off, self.s_cnt).to(params.device)
        return self.plan.outer_grad_coef(n_pseudo, x_all, z_all, w_all, eps_local, params, coef,
                                         grad_u=grad_u, grad_w=grad_w)

    def elbo_grad(self, n_pseudo, x_all, z_all, w_all, eps, params, grad_u=True, grad_w=True,
                  grads=True, sample_weights=False):
        """Loss (float64 tensor) and the full gradients on every rank
        (grads=False: the loss only, pass 1 and one all-reduce).
        sample_weights: also "W", the softmax weights W_s of all S samples
        (float64; sample_out's fourth column of a world-1 plan)."""
        e, t = self.local_terms(n_pseudo, x_all, z_all, w_all, eps, params)
        terms = torch.zeros(self.S, 3, dtype=torch.float64, device=t.device)
        terms[self.s_off:self.s_off + self.s_cnt] = t
        self.comm.all_reduce(terms)
        loss, cp, cd, ck = outer_coefficients(terms)
        if not grads:
            return {"loss": loss.reshape(1)} | ({"W": cd} if sample_weights else {})
        g = self.local_grads(n_pseudo, x_all, z_all, w_all, e, params, cp, cd, ck,
                             grad_u=grad_u, grad_w=grad_w)
        for k in ("grad", "grad_u", "grad_w"):
            if k in g:
                self.comm.all_reduce(g[k])
        g["loss"] = loss.reshape(1)
        if sample_weights:
            g["W"] = cd
        return g

    def coef_grads(self, n_pseudo, x_all, z_all, w_all, eps, params, cp, cd, ck, grad_u=True,
                   grad_w=True):
        """Pass 2 alone for given global coefficients (global eps), summed
        over ranks."""
        e = local_eps(self.family, self.layers, self.S, self.s_off, self.s_cnt, eps)
        g = self.local_grads(n_pseudo, x_all, z_all, w_all, e, params, cp, cd, ck,
                             grad_u=grad_u, grad_w=grad_w)
        for k in ("grad", "grad_u", "grad_w"):
            if k in g:
                self.comm.all_reduce(g[k])
        return g

    # ---- InnerLoopPlan's outer-objective methods (global eps), for PSVI ----
    @property
    def eps_count(self):
        return eps_count(self.family, self.layers, self.S)

    @property
    def eps_stride(self):
        return (self.eps_count + 3) // 4 * 4

    @property
    def param_count(self):
        return self.plan.param_count

    @property
    def in_features(self):
        return self.plan.in_features

    def outer_elbo_grad(self, n_pseudo, x_all, z_all, w_all, eps, params, grad=True,
                        grad_u=True, grad_w=True, sample_stats=False, ws=None):
        """psvi_outer_elbo_grad's contract over all S samples (loss, grad,
        grad_u, grad_w as requested; per-sample stats are not assembled)."""
        if sample_stats:
            raise NotImplementedError("per-sample stats of a sharded outer objective: use "
                                      "local_terms")
        g = self.elbo_grad(n_pseudo, x_all, z_all, w_all, eps, params, grad_u=grad and grad_u,
                           grad_w=grad_w, grads=grad or grad_w)
        if not grad:
            g.pop("grad", None)
            g.pop("grad_u", None)
        return g

    def outer_ablated_elbo_grad(self, x_all, z_all, w_all, eps, params, grad=True,
                                sample_stats=False, ws=None):
        """PSVI_Ablated's objective mean_s data_s - mean_s nkl_s over all S
        samples: each rank's mean over its own samples, weighted s_cnt / S, one
        all-reduce of the loss and the gradient."""
        if sample_stats:
            raise NotImplementedError("per-sample stats of a sharded outer objective")
        e = local_eps(self.family, self.layers, self.S, self.s_off, self.s_cnt, eps)
        o = self.plan.outer_ablated_elbo_grad(x_all, z_all, w_all, e, params, grad=grad)
        f = self.s_cnt / self.S
        for k in ("loss", "grad"):
            if k in o:
                o[k] = (o[k] * f).contiguous()
                self.comm.all_reduce(o[k])
        return o

    def evaluate(self, n_pseudo, x_all, z_all, w_all, eps, params, correction=True,
                 probs=False, ws=None):
        """The importance-weighted predictive (once per log_every outer steps):
        replicated on every rank on a world-1 plan of all S samples."""
        if self._full is None:
            self._full = InnerLoopPlan(self.family, self.layers, self.S, self.M,
                                       prior_sd=self.prior_sd)
        return self._full.evaluate(n_pseudo, x_all, z_all, w_all, eps, params,
                                   correction=correction, probs=probs)


# ---------------------------------------------------------------------------
# Sample-sharded inner objective and second order (PSVI.inner_elbo / inner
# loop, hyper_step's CG_normaleq products, nested_step's reverse pass)
# ---------------------------------------------------------------------------
def eps_count(family, layers, S):
    """Floats of one draw of all S samples (include/psvi_hip.h eps layout;
    LeNet's last layer is one shared draw)."""
    n = 0
    for l, (din, dout) in enumerate(layers):
        k = din * dout + dout
        n += k if (family == "lenet" and l == len(layers) - 1) else S * k
    return n


class SampleShardedPlan:
    """InnerLoopPlan's inner-objective methods for S samples split over ranks
    (sample_split): this rank runs a world-1 plan of its own s_cnt samples on
    its slice of the global eps (local_eps), the sample-independent KL terms on
    rank 0 only (psvi_elbo_grad include_kl, psvi_hvp_partial), and one
    all-reduce sums each result.  The contract is a world-1 plan of all S
    samples -- same eps layout, same Philox draw sequence -- with values equal
    up to fp32 summation order, so PSVI's trainers run unchanged on it
    (C4 / C5 at 8 GPUs; hypergradients.py:199-244 and
    psvi_classes.py:541-687 split over samples).  Parameters and Adam state
    stay replicated: every rank applies the same all-reduced gradient."""

    def __init__(self, family, layers, S, M, world, rank, comm, prior_sd=1.0, plan=None,
                 adam=None):
        self.family, self.layers = family, [tuple(l) for l in layers]
        self.S, self.M, self.world, self.rank, self.comm = int(S), int(M), world, rank, comm
        self.split = sample_split(self.S, world)
        self.s_off, self.s_cnt = self.split[rank]
        if self.s_cnt < 1:
            raise ValueError(f"rank {rank} has no samples (S={S}, world={world})")
        self.plan = plan if plan is not None else InnerLoopPlan(family, layers, self.s_cnt, M,
                                                                prior_sd=prior_sd)
        self._adam = adam if adam is not None else adam_update_
        self.param_count = self.plan.param_count
        self.in_features = self.plan.in_features
        self.eps_count = eps_count(family, self.layers, self.S)
        self.eps_stride = (self.eps_count + 3) // 4 * 4
        self.ws_bytes = self.plan.ws_bytes
        self.hvp_ws_bytes = self.plan.hvp_ws_bytes
        self.n_tot = sum(i * o + o for i, o in self.layers)

    def local(self, eps):
        return local_eps(self.family, self.layers, self.S, self.s_off, self.s_cnt, eps)

    def workspace(self, device="cuda"):
        return self.plan.workspace(device)

    def _reduce(self, *ts):
        for t in ts:
            if t is not None:
                self.comm.all_reduce(t)

    def elbo_grad(self, u, z, w, eps, params, include_kl=True, ws=None):
        e, g = self.plan.elbo_grad(u, z, w, self.local(eps), params,
                                   include_kl=include_kl and self.rank == 0, ws=ws)
        self._reduce(e, g)
        return e, g

    def hvp(self, u, z, w, eps, params, vec, mixed=True, out=None, ws=None, include_kl=True):
        hv, du, dw = self.plan.hvp(u, z, w, self.local(eps), params, vec, mixed=mixed, out=out,
                                   ws=ws, include_kl=include_kl and self.rank == 0)
        self._reduce(hv, du, dw)
        return hv, du, dw

    def inner_step(self, u, z, w, eps, params, adam_m, adam_v, step, lr, kind="higher",
                   elbo_out=None, ws=None):
        """psvi_inner_step's contract: the all-reduced gradient, then the same
        Adam step on every rank's replica."""
        e, g = self.elbo_grad(u, z, w, eps, params, ws=ws)
        self._adam(params, g, adam_m, adam_v, step, lr, kind=kind)
        if elbo_out is None:
            return e
        elbo_out.copy_(e.reshape(elbo_out.shape))
        return elbo_out

    def inner_loop(self, u, z, w, params, adam_m, adam_v, T, lr, kind="higher", step0=1,
                   eps=None, seed=0, offset=0, elbo_out=None, ws=None):
        """psvi_inner_loop's contract (the same Philox draws: step t at
        offset + t * eps_stride of the global layout)."""
        T = int(T)
        dev = params.device
        out = elbo_out if elbo_out is not None else torch.empty(max(T, 1), dtype=torch.float64,
                                                                 device=dev)
        ev = eps.reshape(T, -1) if eps is not None else None
        buf = torch.empty(self.eps_count, device=dev) if eps is None else None
        for t in range(T):
            if ev is None:
                randn_(buf, seed, offset + t * self.eps_stride)
            self.inner_step(u, z, w, ev[t] if ev is not None else buf, params, adam_m, adam_v,
                            step0 + t, lr, kind=kind, elbo_out=out[t:t + 1], ws=ws)
        return out[:T]
