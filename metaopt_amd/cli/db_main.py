"""``mopt db <setup|test|upgrade>`` dispatcher (reference: ``cli/db_main.py:19-39``)."""
from __future__ import annotations

from .db import setup as db_setup
from .db import test as db_test
from .db import upgrade as db_upgrade


def add_subparser(parser):
    p = parser.add_parser("db", help="database helper commands")
    sub = p.add_subparsers(help="database sub-commands")
    for mod in (db_setup, db_test, db_upgrade):
        mod.add_subparser(sub)
    return p
