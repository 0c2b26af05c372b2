"""The ``mopt`` command line (reference: ``src/orion/core/cli/__init__.py:20-41``).

Sub-commands: ``hunt``, ``init_only``, ``insert``, ``list``, ``status``, ``info``,
``db {setup,test,upgrade}``, ``setup``/``test-db`` (deprecated aliases), and ``sweep`` (device
population sweeps).  Modules defining ``add_subparser`` are discovered automatically.
"""
from __future__ import annotations

import importlib
import logging
import pkgutil
import sys

from .base import ArgsParser

log = logging.getLogger(__name__)

_SKIP = {"base", "evc", "db"}


def load_modules_parser(parser: ArgsParser):
    for info in sorted(pkgutil.iter_modules(__path__), key=lambda m: m.name):
        if info.name in _SKIP or info.name.startswith("_"):
            continue
        mod = importlib.import_module(f"{__name__}.{info.name}")
        if hasattr(mod, "add_subparser"):
            mod.add_subparser(parser.get_subparsers())


def main(argv=None):
    parser = ArgsParser()
    load_modules_parser(parser)
    rc = parser.execute(sys.argv[1:] if argv is None else argv)
    return rc or 0


if __name__ == "__main__":
    sys.exit(main())
