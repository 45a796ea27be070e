"""Multi-GPU inner loop: one process per GPU, collectives over RCCL (xGMI).

The reference has no collectives (its only multi-GPU mode is a process pool of
independent jobs, psvi/experiments/flow-psvi-parallel.py:457-463).  Here one
inner step is split across ranks where the math allows it:

  full-cov (fn2):  rows of every layer's L (and the matching mean/sd/corr
      slices + Adam state) are sharded nnz-balanced; MC samples are sharded in
      contiguous blocks.  Per step:
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

from .engine import InnerLoopPlan


class TorchDistComm:
    """Collectives on torch.distributed (backend 'nccl' == RCCL on ROCm)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group

    def all_to_all(self, out, inp, out_splits, in_splits):
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def all_reduce(self, t):
        self.dist.all_reduce(t, group=self.group)


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

    def phase_net(self, u, z, w):
        self.parts.zero_()
        self.plan.mvn_net(u, z, w, self.x_recv, self.g_send, self.parts[0:1])

    def phase_update(self, eps, params, m, v, step, lr, kind, grad_out=None):
        self.plan.mvn_update(eps, self.g_shard, params, m, v, step=step, lr=lr, kind=kind,
                             kl_out=self.parts[1:2], grad_out=grad_out)

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
        po = 0
        for l, (din, dout) in enumerate(self.plan.layers):
            n = din * dout + dout
            nc = (n - 1) * (n - 2) // 2
            lo, hi = info["row_lo"][l], info["row_lo"][l] + info["row_cnt"][l]
            mask[po + lo:po + hi] = True
            mask[po + n + lo:po + n + hi] = True
            clo = min(lo, n - 1)
            chi = min(hi, n - 1)
            mask[po + 2 * n + clo * (clo - 1) // 2:po + 2 * n + chi * (chi - 1) // 2] = True
            po += 2 * n + nc
        return mask

    def gather_params(self, *tensors):
        """Make every rank's copy of params (and Adam state) identical by
        summing the owned slices (end of an inner loop, not per step)."""
        mask = self.owned_mask()
        for t in tensors:
            t.mul_(mask)
            self.comm.all_reduce(t)
