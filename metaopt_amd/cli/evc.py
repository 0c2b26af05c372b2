"""Branching arguments generated from the EVC resolutions (reference: ``cli/evc.py:15-104``)."""
from __future__ import annotations

from ..evc import adapters
from ..evc import conflicts as C

RESOLUTION_ARGS = [
    (C.FLAGS["branch"], "-b",
     dict(type=str, metavar="stringID",
          help="Unique name for the new branching experiment")),
    (C.FLAGS["algorithm"], None,
     dict(action="store_true", help="Set algorithm change as resolved if a branching event "
                                    "occur")),
    (C.FLAGS["code"], None,
     dict(type=str, choices=list(adapters.CHANGE_TYPES),
          help="Set code change type (default: break)")),
    (C.FLAGS["cli"], None,
     dict(type=str, choices=list(adapters.CHANGE_TYPES),
          help="Set command line change type (default: break)")),
    (C.FLAGS["config"], None,
     dict(type=str, choices=list(adapters.CHANGE_TYPES),
          help="Set script config change type (default: break)")),
]


def get_branching_args_group(parser):
    g = parser.add_argument_group("Branching arguments",
                                  description="Arguments to automatically resolve branching "
                                              "events.")
    g.add_argument("--manual-resolution", action="store_true",
                   help="Starts the interactive prompt to resolve conflicts manually.")
    g.add_argument("--auto-resolution", action="store_true",
                   help="(deprecated) conflicts are resolved automatically by default")
    for arg, short, kwargs in RESOLUTION_ARGS:
        names = [arg] + ([short] if short else [])
        g.add_argument(*names, **kwargs)
    return g


def fetch_branching_configuration(config):
    keys = ["manual_resolution", "auto_resolution", "branch", "algorithm_change",
            "code_change_type", "cli_change_type", "config_change_type"]
    return {k: config[k] for k in keys if k in config}
