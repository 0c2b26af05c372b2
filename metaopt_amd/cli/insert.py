"""``mopt insert -n exp script -x=1``: insert a user-specified trial
(reference: ``cli/insert.py:39-198``).

Values are parsed with ``ast.literal_eval`` (the reference ``eval``s them) and cast by the
dimension; dimensions not given take their ``default_value`` or fail.
"""
from __future__ import annotations

import ast
import datetime
import logging

from ..core.config import config as global_config
from ..io.experiment_builder import ExperimentBuilder
from ..io.space_parser import SpaceCmdlineParser
from ..utils import format_trials
from .base import get_basic_args_group, get_user_args_group

log = logging.getLogger(__name__)


def add_subparser(parser):
    p = parser.add_parser("insert", help="Insert a trial with specified parameter values.")
    get_basic_args_group(p)
    get_user_args_group(p)
    p.set_defaults(func=main)
    return p


def _literal(v):
    if isinstance(v, str):
        try:
            return ast.literal_eval(v)
        except (ValueError, SyntaxError):
            return v
    return v


def _build_from_args(cmd_args, space):
    """{'/x': value} from ``--x=1`` style arguments of the insert command line."""
    parser = SpaceCmdlineParser(global_config.user_script_config)
    parser.parser.parse(cmd_args)
    values = {}
    for key, value in parser.parser.arguments.items():
        if key.startswith("_"):
            continue
        values["/" + key] = _literal(value)
    return values


def validate_dimensions(values, space):
    point = []
    for name, dim in space.items():
        if name in values:
            v = values[name]
            v = dim.cast(v) if dim.type not in ("fidelity",) else int(v)
        elif dim.default_value is not None:
            v = dim.default_value
        else:
            raise ValueError(f"Dimension {name} is unspecified and has no default value")
        if v not in dim:
            raise ValueError(f"Value {v} is outside of dimension's prior interval {dim}")
        point.append(v)
    unknown = set(values) - set(space.keys())
    if unknown:
        raise ValueError(f"Unknown dimensions {sorted(unknown)}")
    return tuple(point)


def main(args):
    builder = ExperimentBuilder()
    view = builder.build_view_from(args)
    experiment = view._experiment
    user_args = list(args.get("user_args") or [])
    values = _build_from_args(user_args[1:] if user_args else [], experiment.space)
    point = validate_dimensions(values, experiment.space)
    trial = format_trials.tuple_to_trial(point, experiment.space)
    storage = experiment._storage
    storage = getattr(storage, "_storage", storage)
    trial.experiment = experiment.id
    trial.status = "new"
    trial.submit_time = datetime.datetime.utcnow()
    storage.register_trial(trial)
    return 0
