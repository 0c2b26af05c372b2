"""``mopt setup``: deprecated alias of ``mopt db setup`` (reference ``cli/setup.py:20-35``; the
deprecation warning is actually shown here, quirk 8)."""
from __future__ import annotations

import logging

from .db import setup as db_setup

log = logging.getLogger(__name__)


def add_subparser(parser):
    p = db_setup.add_subparser(parser)
    p.set_defaults(func=main)
    return p


def main(args):
    log.warning("Command `mopt setup` is deprecated, use `mopt db setup` instead.")
    print("Warning: `setup` is deprecated, use `db setup`.")
    return db_setup.main(args)
