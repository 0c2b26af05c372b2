"""The ``mopt`` command line (reference: ``src/orion/core/cli/__init__.py:20-41``).

Sub-commands: ``hunt``, ``init_only``, ``insert``, ``list``, ``status``, ``info``,
``db {setup,test,upgrade}``, ``setup``/``test-db`` (deprecated aliases), and ``sweep`` (device
population sweeps).  Modules defining ``add_subparser`` are discovered automatically.
"""
from __future__ import annotations

import importlib
import logging
import pkgutil
import re
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


_ARGV: list = []
_PRIOR_ARG = re.compile(r"^--?[^=~\s]+~")


def current_argv() -> list:
    """The argument list of the running ``main`` call (launchers re-run it per rank)."""
    return [*_ARGV]     # (``list`` here is the cli.list sub-module once it is imported)


def _subcommand_index(argv) -> int:
    """Position of the sub-command: the first argument that is not a global option (the global
    flags -V/-v/-d take no value), or -1."""
    for i, a in enumerate(argv):
        if not a.startswith("-"):
            return i
    return -1


def _space_after_options(argv):
    """``mopt sweep ... --lr~'loguniform(..)'``: a sweep has no script, so its space starts at
    the first ``--name~prior`` argument; a ``--`` there hands the rest to the user arguments.
    Only the ``sweep`` sub-command is rewritten: a ``sweep`` token elsewhere (an experiment name,
    a user argument's value) leaves the command line as typed."""
    sub = _subcommand_index(argv)
    if sub < 0 or argv[sub] != "sweep":
        return argv
    start = sub + 1
    for i in range(start, len(argv)):
        if argv[i] == "--":
            return argv
        if _PRIOR_ARG.match(argv[i]):
            return argv[:i] + ["--"] + argv[i:]
    return argv


def main(argv=None):
    argv = [*(sys.argv[1:] if argv is None else argv)]
    _ARGV[:] = argv
    parser = ArgsParser()
    load_modules_parser(parser)
    rc = parser.execute(_space_after_options(argv))
    return rc or 0


if __name__ == "__main__":
    sys.exit(main())
