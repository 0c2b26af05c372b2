"""``mopt hunt``: run (or resume) an experiment with this process as one worker
(reference: ``cli/hunt.py:25-75``)."""
from __future__ import annotations

import logging

from ..io.experiment_builder import ExperimentBuilder
from ..worker.workon import workon
from .base import get_basic_args_group, get_user_args_group
from .evc import get_branching_args_group

log = logging.getLogger(__name__)


def add_subparser(parser):
    p = parser.add_parser("hunt", help="Conduct hyperparameter optimization.")
    g = get_basic_args_group(p)
    g.add_argument("--max-trials", type=int, metavar="#",
                   help="number of trials to be completed for the experiment (default: inf)")
    g.add_argument("--worker-trials", type=int, metavar="#",
                   help="number of trials to be completed for this worker (default: inf)")
    g.add_argument("--working-dir", type=str,
                   help="persistent working directory of the trials (default: temporary)")
    g.add_argument("--pool-size", type=int, metavar="#",
                   help="number of simultaneous trials the algorithm suggests (default: 1)")
    get_branching_args_group(p)
    get_user_args_group(p)
    p.set_defaults(func=main)
    return p


def main(args):
    builder = ExperimentBuilder()
    worker_trials = builder.fetch_full_config(args, use_db=False)["worker_trials"]
    experiment = builder.build_from(args)
    workon(experiment, worker_trials)
    return 0
