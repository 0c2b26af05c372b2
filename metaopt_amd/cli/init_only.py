"""``mopt init_only``: register an experiment without running it (reference: ``cli/init_only.py``)."""
from __future__ import annotations

from ..io.experiment_builder import ExperimentBuilder
from .base import get_basic_args_group, get_user_args_group
from .evc import get_branching_args_group


def add_subparser(parser):
    p = parser.add_parser("init_only", help="Only initialize experiment.")
    g = get_basic_args_group(p)
    g.add_argument("--max-trials", type=int, metavar="#")
    g.add_argument("--pool-size", type=int, metavar="#")
    g.add_argument("--working-dir", type=str)
    get_branching_args_group(p)
    get_user_args_group(p)
    p.set_defaults(func=main)
    return p


def main(args):
    ExperimentBuilder().build_from(args)
    return 0
