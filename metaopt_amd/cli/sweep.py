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

ALGOS = {"asha": lambda seed, n: {"asha": {"seed": seed, "repetitions": float("inf")}},
         "random": lambda seed, n: {"random": {"seed": seed}},
         "tpe": lambda seed, n: {"tpe": {"seed": seed, "n_initial_points": n}},
         "pbt": lambda seed, n: {"pbt": {"seed": seed, "population_size": n}},
         "hyperband": lambda seed, n: {"hyperband": {"seed": seed}},
         "gridsearch": lambda seed, n: {"gridsearch": {"n_values": 4}}}


def add_subparser(parser):
    from ..worker.tasks import TASKS
    p = parser.add_parser("sweep", help="Device population sweep (trials trained on GPU).")
    g = get_basic_args_group(p)
    g.add_argument("--task", default="mlp", choices=sorted(TASKS))
    g.add_argument("--algo", default=None, choices=sorted(ALGOS),
                   help="search algorithm (default: the task's)")
    g.add_argument("--population", type=int, default=None, help="trials per GPU")
    g.add_argument("--max-trials", type=int, default=None)
    g.add_argument("--steps", type=int, default=100000, help="max population steps")
    g.add_argument("--sync-every", type=int, default=32)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--event-log", default=None,
                   help="JSONL event log path (rank r writes <path>.rank<r> when world > 1)")
    g.add_argument("--trial-events", action="store_true",
                   help="one event per finished trial in the event log")
    g.add_argument("--resume", action="store_true",
                   help="continue the stored experiment: replay its finished trials, re-reserve "
                        "interrupted/lost ones, restore the saved algorithm state")
    g.add_argument("--ckpt-dir", default=None,
                   help="directory for per-trial device-state sidecars written at the end of "
                        "the sweep (promotions and interrupted trials resume from them)")
    g.add_argument("--watchdog", type=float, default=0.0,
                   help="seconds without a sync before the rank fails the job cleanly "
                        "(in-flight trials -> interrupted); 0 disables")
    p.set_defaults(func=main)
    return p


DEFAULT_POPULATION = {"logreg": 64, "mlp": 256, "resnet20": 32, "lm-125m": 8, "lm-tiny": 16}


def main(args):
    from ..io.experiment_builder import ExperimentBuilder, build_experiment
    from ..parallel.comm import init_from_env, shutdown
    from ..worker.population_sweep import PopulationSweep
    from ..worker.tasks import get

    comm = init_from_env()
    spec = get(args["task"])
    P = args["population"] or DEFAULT_POPULATION.get(args["task"], 64)
    algo = (ALGOS[args["algo"]](args["seed"], P * comm.world_size) if args["algo"]
            else spec.algorithm(args["seed"], P * comm.world_size))
    task, pop, data = spec.build(P, comm.device, args["seed"])
    experiment = None
    if comm.is_root:
        builder = ExperimentBuilder()
        builder.setup_storage({"debug": args.get("debug"), "database": {}})
        experiment = build_experiment(args["name"] or f"sweep-{args['task']}",
                                      priors=dict(task.priors), algorithms=algo,
                                      max_trials=args["max_trials"] or float("inf"),
                                      pool_size=P * comm.world_size)
    events = watchdog = None
    if args.get("event_log"):
        from ..utils.events import EventLog
        path = args["event_log"]
        if comm.world_size > 1:
            path = f"{path}.rank{comm.rank}"
        events = EventLog(path, rank=comm.rank)
    if args.get("watchdog"):
        from ..parallel.watchdog import Watchdog
        watchdog = Watchdog(args["watchdog"], events=events, rank=comm.rank)
    sweep = PopulationSweep(pop, task, data, comm=comm, experiment=experiment,
                            sync_every=args["sync_every"],
                            ckpt_capacity=max(4, int(spec.ckpt_factor * P)),
                            events=events, trial_events=args.get("trial_events", False),
                            watchdog=watchdog, resume=args.get("resume", False),
                            restore_algorithm=args.get("resume", False),
                            ckpt_dir=args.get("ckpt_dir"))
    try:
        summary = sweep.run(args["steps"])
    except BaseException:
        # rank-local teardown only: the peers may be inside another collective; the original
        # error propagates (in-flight trials -> interrupted, the watchdog stops)
        sweep.close(failed=True)
        if events is not None:
            events.close()
        raise
    sweep.close()
    if events is not None:
        events.close()
    if comm.is_root:
        print(json.dumps({k: v for k, v in summary.items()}, default=str))
    shutdown()
    return 0
