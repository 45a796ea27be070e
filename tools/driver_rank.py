#!/usr/bin/env python3
"""One rank of a multi-GPU experiment_driver run (torchrun: RANK / WORLD_SIZE /
LOCAL_RANK from the environment).  --share-gpu puts every rank on device 0
with gloo collectives (a rehearsal on a one-GPU box); otherwise RCCL, one GPU
per rank.  Prints rank 0's results for the halfmoon PSVI run as one JSON line.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      tools/driver_rank.py --share-gpu
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blackbox-coresets-vi_amd"))

METHOD_ARGS = dict(coreset_sizes=[10], num_trials=1, mc_samples=8, num_epochs=4,
                   data_minibatch=128, inner_it=3, trainer="nested", log_every=2, lr0u=1e-3,
                   lr0net=1e-3, lr0v=1e-3, init_sd=1e-6, architecture="fn2", n_hidden=8,
                   n_layers=1, test_ratio=0.2, register_elbos=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--share-gpu", action="store_true")
    ap.add_argument("--trainer", default="nested")
    ap.add_argument("--method", default="psvi_learn_v")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = 0 if a.share_gpu else local
    torch.cuda.set_device(dev)
    comm = None
    if world > 1:
        import torch.distributed as dist
        from psvi.runtime.sharded import HostStagedComm, TorchDistComm

        if a.share_gpu:
            dist.init_process_group("gloo")
            comm = HostStagedComm()
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            comm = TorchDistComm()
    from psvi.experiments.flow_psvi import experiment_driver

    args = dict(METHOD_ARGS, trainer=a.trainer)
    res = experiment_driver(["halfmoon"], [a.method], args, write=False, world=world, rank=rank,
                            comm=comm)
    r = res["halfmoon"][a.method][10][0]
    out = {k: [float(x) for x in r[k]] for k in ("accs", "nlls")}
    out["vs"] = [float(x) for x in r["vs"][-1]]
    out.update(world=world, rank=rank)
    if world == 1:
        print(json.dumps(out), flush=True)
        return
    import torch.distributed as dist

    # one rank at a time: the ranks share the launcher's stdout, and lines
    # written at once can interleave
    for r in range(world):
        if r == rank:
            print(json.dumps(out), flush=True)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
