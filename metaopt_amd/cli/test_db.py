"""``mopt test-db``: deprecated alias of ``mopt db test``."""
from __future__ import annotations

from .db import test as db_test


def add_subparser(parser):
    p = parser.add_parser("test-db", help="(deprecated) use `db test`")
    p.add_argument("-c", "--config", help="mopt configuration file (YAML)")
    p.set_defaults(func=main)
    return p


def main(args):
    print("Warning: `test-db` is deprecated, use `db test`.")
    return db_test.main(args)
