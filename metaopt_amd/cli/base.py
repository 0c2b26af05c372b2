"""Argument parsing shared by every sub-command (reference: ``src/orion/core/cli/base.py:27-126``).

Global flags: ``-V/--version``, ``-v`` (repeatable: INFO, DEBUG), ``-d/--debug`` (in-memory
EphemeralDB).  ``get_basic_args_group`` adds ``-n/--name``, ``-u/--user``, ``--exp-version``
(``-v`` inside a sub-command, as in the reference, quirk 9 kept for compatibility), and
``-c/--config``; ``get_user_args_group`` adds the user script command line (REMAINDER).
"""
from __future__ import annotations

import argparse
import logging
import textwrap

from .. import __version__
from ..storage.database import DatabaseError
from ..utils.exceptions import NoConfigurationError

CLI_DOC_HEADER = "mopt: MI355X-native asynchronous hyper-parameter optimisation"


class ArgsParser:
    def __init__(self, description=CLI_DOC_HEADER):
        self.parser = argparse.ArgumentParser(
            prog="mopt", formatter_class=argparse.RawDescriptionHelpFormatter,
            description=textwrap.dedent(description))
        self.parser.add_argument("-V", "--version", action="version",
                                 version="mopt " + __version__)
        self.parser.add_argument("-v", "--verbose", action="count", default=0,
                                 help="logging levels (-v: INFO, -vv: DEBUG)")
        self.parser.add_argument("-d", "--debug", action="store_true",
                                 help="Use debugging mode with EphemeralDB.")
        self.subparsers = self.parser.add_subparsers(help="sub-command help")

    def get_subparsers(self):
        return self.subparsers

    def parse(self, argv):
        args = vars(self.parser.parse_args(argv))
        verbose = args.pop("verbose", 0)
        levels = {0: logging.WARNING, 1: logging.INFO, 2: logging.DEBUG}
        logging.basicConfig(level=levels.get(verbose, logging.DEBUG))
        logging.getLogger().setLevel(levels.get(verbose, logging.DEBUG))
        func = args.pop("func", None)
        if func is None:
            self.parser.print_help()
            raise SystemExit(0)
        return args, func

    def execute(self, argv):
        try:
            args, func = self.parse(argv)
            return func(args)
        except NoConfigurationError:
            print("Error: No commandline configuration found for new experiment.")
            return 1
        except DatabaseError as exc:
            print(exc)
            return 1


OrionArgsParser = ArgsParser


def get_basic_args_group(parser):
    g = parser.add_argument_group("mopt arguments (optional)",
                                  description="These arguments determine mopt's behaviour")
    g.add_argument("-n", "--name", type=str, metavar="stringID",
                   help="experiment's unique name (default: from a config file)")
    g.add_argument("-u", "--user", type=str, help="user associated to the experiment's name")
    g.add_argument("-v", "--version", type=int,
                   help="specific version of experiment to fetch (default: latest)")
    g.add_argument("-c", "--config", type=argparse.FileType("r"), metavar="path-to-config",
                   help="user provided mopt configuration file")
    return g


def get_user_args_group(parser):
    g = parser.add_argument_group(
        "User script related arguments",
        description="These arguments determine user's script behaviour and they can serve as "
                    "mopt's parameter declaration.")
    g.add_argument("user_args", nargs=argparse.REMAINDER, metavar="...",
                   help="Command line of user script.")
    return g
