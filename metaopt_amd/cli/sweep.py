"""``mopt sweep``: run an experiment's trials as device populations (one process per GPU).

    mopt sweep -n mlp-asha --algo asha --population 256 --max-trials 2000
    torchrun --nproc-per-node 8 -m metaopt_amd sweep -n mlp-asha ...

The experiment (space, algorithm, trials) lives in the configured database exactly like a
``hunt`` experiment -- ``status``/``info``/``list`` work on it -- but trials are trained in-process
on the GPU by :class:`~metaopt_amd.worker.population_sweep.PopulationSweep`.
"""
from __future__ import annotations

import json
import logging

from .base import get_basic_args_group

log = logging.getLogger(__name__)

ALGOS = {"asha": lambda seed: {"asha": {"seed": seed, "repetitions": float("inf")}},
         "random": lambda seed: {"random": {"seed": seed}},
         "tpe": lambda seed: {"tpe": {"seed": seed}}}


def add_subparser(parser):
    p = parser.add_parser("sweep", help="Device population sweep (trials trained on GPU).")
    g = get_basic_args_group(p)
    g.add_argument("--task", default="mlp", choices=["mlp", "logreg"])
    g.add_argument("--algo", default="asha", choices=sorted(ALGOS))
    g.add_argument("--population", type=int, default=256, help="trials per GPU")
    g.add_argument("--max-trials", type=int, default=None)
    g.add_argument("--steps", type=int, default=100000, help="max population steps")
    g.add_argument("--sync-every", type=int, default=32)
    g.add_argument("--seed", type=int, default=0)
    p.set_defaults(func=main)
    return p


def main(args):
    import torch
    from ..io.experiment_builder import build_experiment, ExperimentBuilder
    from ..models.data import TeacherClassification
    from ..models.mlp import LOGREG_PRIORS, MLP_PRIORS, MLPSweepTask
    from ..ops.population import PopulationMLP
    from ..parallel.comm import init_from_env, shutdown
    from ..worker.population_sweep import PopulationSweep

    comm = init_from_env()
    logreg = args["task"] == "logreg"
    priors = dict(LOGREG_PRIORS if logreg else MLP_PRIORS)
    task = MLPSweepTask(priors=priors, n_hidden=0 if logreg else 3,
                        in_features=2 if logreg else 784, num_classes=2 if logreg else 10)
    experiment = None
    if comm.is_root:
        builder = ExperimentBuilder()
        builder.setup_storage({"debug": args.get("debug"), "database": {}})
        experiment = build_experiment(args["name"] or f"sweep-{args['task']}", priors=priors,
                                      algorithms=ALGOS[args["algo"]](args["seed"]),
                                      max_trials=args["max_trials"] or float("inf"),
                                      pool_size=args["population"] * comm.world_size)
    data = TeacherClassification(n_train=60032 if not logreg else 8192, n_val=1024,
                                 in_features=task.in_features, num_classes=task.num_classes,
                                 teacher_hidden=128 if not logreg else 4, seed=args["seed"],
                                 device=comm.device)
    pop = PopulationMLP(args["population"], in_features=task.in_features,
                        num_classes=task.num_classes, n_hidden=task.n_hidden,
                        max_width=task.max_width if not logreg else 64, eval_batch=1024,
                        device=comm.device)
    sweep = PopulationSweep(pop, task, data, comm=comm, experiment=experiment,
                            sync_every=args["sync_every"])
    summary = sweep.run(args["steps"])
    if comm.is_root:
        print(json.dumps({k: v for k, v in summary.items()}, default=str))
    shutdown()
    return 0
