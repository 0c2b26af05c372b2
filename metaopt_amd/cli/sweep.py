"""``mopt sweep``: run an experiment's trials as device populations (one process per GPU).

    mopt sweep -n mlp-asha --task mlp --gpus 8 --max-trials 20000 \\
        --lr~'loguniform(1e-4, 1)' --width~'loguniform(64, 512, discrete=True)' \\
        --dropout~'uniform(0, 0.3)' --steps~'fidelity(32, 512, 4)'
    mopt sweep -n mlp-asha --task mlp -c sweep.yaml        # algorithms / max_trials from a file
    torchrun --nproc-per-node 8 -m metaopt_amd sweep -n mlp-asha ...

The search space is the user's, in the prior grammar of ``hunt`` (``--name~prior(...)`` after
the options, or the task's default space when none is given): it is parsed by the same
command-line parser, validated against the task's tunable hyper-parameters, stored with the
experiment (so ``status`` / ``info`` / ``list`` and EVC branching work on it) and sampled by
the algorithm.  The experiment configuration is resolved with the reference's precedence
(defaults < environment < stored experiment < ``--config`` file < command line,
``src/orion/core/io/experiment_builder.py:175-185``): a file's ``algorithms`` / ``max_trials``
/ ``pool_size`` apply unless the command line sets them (``--algo`` / ``--max-trials``).

``--gpus N`` (N > 1, outside torchrun) makes this process a launcher of N rank processes
(``parallel/launch.py``, the launcher ``bench.py`` uses); ``--dtype`` picks the storage
precision of the optimizer state (``bf16``: bf16 momentum / AdamW first moment; ``fp32``).
Compute is bf16 MFMA with fp32 accumulation and an exact fp32 master either way.
"""
from __future__ import annotations

import json
import logging
import os
import sys

from .base import get_basic_args_group, get_user_args_group
from .evc import get_branching_args_group

log = logging.getLogger(__name__)

ALGOS = {"asha": lambda seed, n: {"asha": {"seed": seed, "repetitions": float("inf")}},
         "random": lambda seed, n: {"random": {"seed": seed}},
         "tpe": lambda seed, n: {"tpe": {"seed": seed, "n_initial_points": n}},
         "pbt": lambda seed, n: {"pbt": {"seed": seed, "population_size": n}},
         "hyperband": lambda seed, n: {"hyperband": {"seed": seed}},
         "gridsearch": lambda seed, n: {"gridsearch": {"n_values": 4}}}

DEFAULT_POPULATION = {"logreg": 64, "mlp": 256, "resnet20": 32, "lm-125m": 8, "lm-tiny": 16}


def add_subparser(parser):
    from ..worker.tasks import TASKS
    p = parser.add_parser("sweep", help="Device population sweep (trials trained on GPU).")
    g = get_basic_args_group(p)
    g.add_argument("--task", default="mlp", choices=sorted(TASKS))
    g.add_argument("--algo", default=None, choices=sorted(ALGOS),
                   help="search algorithm (default: the --config file's, else the task's)")
    g.add_argument("--gpus", type=int, default=1,
                   help="ranks to launch, one per GPU (ignored under torchrun)")
    g.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                   help="optimizer-state storage precision (compute: bf16 MFMA, fp32 accum)")
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
    get_branching_args_group(p)
    get_user_args_group(p)
    p.set_defaults(func=main)
    return p


def _user_priors(user_args):
    """The space of ``--name~prior`` user arguments (sweeps have no script: a leading token
    that is not an option is refused)."""
    from ..io.space_parser import SpaceCmdlineParser
    args = list(user_args or [])
    if args and args[0] == "--":
        args = args[1:]
    if not args:
        return None, []
    if not args[0].startswith("-"):
        raise ValueError(f"mopt sweep trains in-process: no script expected, got '{args[0]}' "
                         "(give the search space as --name~prior(...))")
    parser = SpaceCmdlineParser()
    parser.parse(args)
    return dict(parser.priors), args


def resolve(args: dict, world_size: int, population: int):
    """(full experiment configuration, priors, builder): the reference's precedence (the
    stored experiment of that name included), the user's space -- else the stored one, else
    the task's -- validated against the task."""
    from ..io.experiment_builder import ExperimentBuilder
    from ..space.builder import SpaceBuilder
    from ..worker.tasks import get
    spec = get(args["task"])
    cmd = {k: args.get(k) for k in ("name", "user", "version", "config", "debug",
                                    "manual_resolution", "auto_resolution", "branch",
                                    "algorithm_change", "code_change_type", "cli_change_type",
                                    "config_change_type")}
    if args.get("max_trials") is not None:
        cmd["max_trials"] = args["max_trials"]
    if args.get("algo"):
        cmd["algorithms"] = ALGOS[args["algo"]](args.get("seed", 0), population * world_size)
    if cmd["name"] is None:
        cmd["name"] = f"sweep-{args['task']}"
    builder = ExperimentBuilder()
    if args.get("debug"):
        builder.setup_storage({"debug": True})
    full = builder.fetch_full_config(cmd)
    stored = builder.fetch_config_from_db(cmd) or {}
    priors, user_args = _user_priors(args.get("user_args"))
    if priors is None:
        md = stored.get("metadata", {}) or {}
        if md.get("user_args") is not None and md.get("priors"):
            priors, user_args = dict(md["priors"]), list(md["user_args"])
        else:
            priors = dict(spec.priors)
            user_args = [f"--{k.lstrip('/')}~{v}" for k, v in priors.items()]
    spec.check_space(SpaceBuilder().build(priors))
    file_algos = (builder.fetch_file_config(cmd) or {}).get("algorithms")
    if args.get("algo"):          # an algorithm replaces, never merges with, the file's
        full["algorithms"] = cmd["algorithms"]
    elif file_algos:
        full["algorithms"] = file_algos
    elif not stored.get("algorithms"):
        full["algorithms"] = spec.algorithm(args.get("seed", 0), population * world_size)
    full["pool_size"] = population * world_size
    full.setdefault("metadata", {})["user_args"] = user_args
    full["metadata"].pop("user_script", None)
    return full, priors, builder


def main(args):
    if int(args.get("gpus") or 1) > 1 and "WORLD_SIZE" not in os.environ:
        from ..parallel.launch import spawn
        return spawn(int(args["gpus"]), ["-m", "metaopt_amd", *_argv()])
    return run(args)


def _argv():
    """This invocation's command line (``mopt ...`` / ``python -m metaopt_amd ...``)."""
    from . import current_argv
    return current_argv()


def run(args):
    from ..parallel.comm import init_from_env, shutdown
    from ..worker.population_sweep import PopulationSweep
    from ..worker.tasks import get

    comm = init_from_env()
    spec = get(args["task"])
    P = args["population"] or DEFAULT_POPULATION.get(args["task"], 64)
    experiment = None
    priors = None
    if comm.is_root:
        full, priors, builder = resolve(args, comm.world_size, P)
        experiment = builder.build_from_config(full)
        priors = dict(experiment.configuration["metadata"]["priors"])
    # every rank builds its population for the same (stored) space
    priors = comm.broadcast_object(priors)
    task, pop, data = spec.build(P, comm.device, args["seed"], priors=priors,
                                 state_dtype=args.get("dtype", "bf16"))
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
        summary["experiment"] = {"name": experiment.name, "version": experiment.version,
                                 "space": priors, "algorithms": experiment.configuration[
                                     "algorithms"], "world_size": comm.world_size}
        print(json.dumps(summary, default=str), flush=True)
    shutdown()
    return 0
