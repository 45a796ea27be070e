"""flow_psvi.experiment_driver (psvi/experiments/flow_psvi.py:357-454) over the
methods the HIP path runs: the PSVI variants' run_psvi and the MFVI
baselines.  No CLI: method_args is the reference's dict of parsed arguments.

Multi-GPU (one process per GPU): every rank calls
experiment_driver with the same arguments and its ``world`` / ``rank`` (or
``method_args["world"]`` / ``["rank"]``) and, optionally, a collective
backend ``comm`` (psvi.runtime.sharded: TorchDistComm over RCCL by default,
HostStagedComm for gloo).  The PSVI methods then split their MC samples over
the ranks (the objectives, HVPs and trainers all-reduce the ranks' shares:
every rank holds the same u, v and network after every step); the MFVI
baselines have no sample-sharded form and run whole on every rank.  Rank 0
alone writes the results files."""
from ..inference import (PSVI, PSVIAV, PSVIAFixedU, PSVIFixedU, PSVIFreeV, PSVILearnV,
                         PSVI_Ablated, PSVI_No_IW, PSVI_No_Rescaling, run_mfvi, run_mfvi_subset)
from .experiments_utils import read_dataset, rec_dd, write_to_files


def _psvi(cls):
    return lambda *a, **kw: cls(*a, **kw).run_psvi(*a, **kw)


# flow_psvi.py:306-354 (the regression variants and the selection baselines --
# sparsevi, giga, opsvi, random, sparsebbvi -- are not on the HIP path)
inf_dict = {
    "psvi": _psvi(PSVI),
    "psvi_ablated": _psvi(PSVI_Ablated),
    "psvi_learn_v": _psvi(PSVILearnV),
    "psvi_alpha_v": _psvi(PSVIAV),
    "psvi_no_iw": _psvi(PSVI_No_IW),
    "psvi_free_v": _psvi(PSVIFreeV),
    "psvi_no_rescaling": _psvi(PSVI_No_Rescaling),
    "psvi_fixed_u": _psvi(PSVIFixedU),
    "psvi_alpha_fixed_u": _psvi(PSVIAFixedU),
    "mfvi": run_mfvi,
    "mfvi_subset": run_mfvi_subset,
}


def experiment_driver(datasets, methods, method_args, write=True, world=None, rank=None,
                      comm=None):
    """For each dataset, method, trial and coreset size: run the method with
    the reference's keyword set and store its results dict at
    results[dataset][method][size][trial]; coreset-free methods use size -1.
    world / rank / comm: this process's place in a multi-GPU run (above)."""
    world = int(method_args.get("world", 1) if world is None else world)
    rank = int(method_args.get("rank", 0) if rank is None else rank)
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    shard = dict(world=world, rank=rank, comm=comm) if world > 1 else {}
    results = rec_dd()
    for dnm in datasets:
        x, y, xt, yt, N, D, train_dataset, test_dataset, nc = read_dataset(dnm, method_args)
        for nm_alg in methods:
            if nm_alg not in inf_dict:
                raise NotImplementedError(f"method {nm_alg!r} is not on the HIP path")
            logistic_regression = method_args.get(
                "logistic_regression", method_args.get("architecture") == "logreg")
            compute_weights_entropy = (not nm_alg.startswith(("opsvi", "mfvi_subset"))
                                       and method_args.get("compute_weights_entropy", True))
            sizes = (method_args["coreset_sizes"]
                     if nm_alg.startswith(("psvi", "opsvi", "mfvi_subset")) else [-1])
            extra = shard if nm_alg.startswith("psvi") else {}
            for t in range(method_args["num_trials"]):
                for ps in sizes:
                    results[dnm][nm_alg][ps][t] = inf_dict[nm_alg](
                        **extra,
                        mc_samples=method_args["mc_samples"],
                        num_epochs=method_args["num_epochs"],
                        data_minibatch=method_args["data_minibatch"],
                        D=D, N=N, tr=t, x=x, y=y, xt=xt, yt=yt,
                        inner_it=method_args["inner_it"],
                        logistic_regression=logistic_regression,
                        trainer=method_args["trainer"],
                        log_every=method_args["log_every"],
                        register_elbos=method_args.get("register_elbos", False),
                        lr0u=method_args["lr0u"], lr0net=method_args["lr0net"],
                        lr0v=method_args["lr0v"], lr0z=method_args.get("lr0z", 1e-2),
                        lr0alpha=method_args.get("lr0alpha", 1e-3),
                        init_args=method_args.get("init_at", "subsample"),
                        init_sd=method_args["init_sd"], num_pseudo=ps, seed=t,
                        compute_weights_entropy=compute_weights_entropy,
                        architecture=method_args.get("architecture"),
                        log_pseudodata=method_args.get("log_pseudodata", False),
                        n_hidden=method_args.get("n_hidden", 40),
                        n_layers=method_args.get("n_layers", 1),
                        train_dataset=train_dataset, test_dataset=test_dataset, dnm=dnm, nc=nc,
                        learn_z=method_args.get("learn_z", False))
    if write and rank == 0:
        return write_to_files(results, method_args.get("fnm", "results"),
                              method_args.get("results_folder", "results"))
    return results
