"""``mopt db upgrade``: migrate an old database in place (reference: ``cli/db/upgrade.py:56-183``).

Drops the deprecated ``(name, metadata.user)`` indexes, converts a PickledDB file written in an
older on-disk format to the current one, adds ``version`` (default 1) and derives
``metadata.parser``/``metadata.priors`` from ``user_args`` for old experiment documents.
"""
from __future__ import annotations

import sys

from ...core.experiment import populate_priors
from ...storage.protocol import DocumentStorage, setup_storage, get_storage, storage_is_set


def add_subparser(parser):
    p = parser.add_parser("upgrade", help="Upgrade the database scheme")
    p.add_argument("-c", "--config", help="mopt configuration file (YAML)")
    p.add_argument("-f", "--force", action="store_true", help="Don't prompt user")
    p.set_defaults(func=main)
    return p


DEPRECATED_INDEXES = ["name_1_metadata.user_1", "name_1_metadata.user_1_version_1"]


def update_indexes(database):
    info = database.index_information("experiments")
    for idx in DEPRECATED_INDEXES:
        if idx in info:
            database.drop_index("experiments", idx)


def upgrade_db_specifics(database):
    """Backend-specific steps: deprecated indexes everywhere, the on-disk format of a PickledDB
    file, MongoDB's index set (re-created by the storage setup that follows)."""
    from ...storage.database import MongoDB, PickledDB
    if isinstance(database, PickledDB):
        # the format conversion is counted on the file as found: any write (an index drop
        # included) rewrites it in the current format, so it runs before the index step
        print("Updating pickleddb scheme...")
        n = database.upgrade_format()
        print(f"  {n} collection(s) converted to format 2")
    print("Updating indexes...")
    update_indexes(database)
    if isinstance(database, MongoDB):
        print("Updating mongodb scheme...")
        for col in ("experiments", "trials"):
            for name in list(database.index_information(col)):
                if name in DEPRECATED_INDEXES:
                    database.drop_index(col, name)


def upgrade_documents(storage):
    for exp in storage.fetch_experiments({}):
        exp.setdefault("version", 1)
        populate_priors(exp.setdefault("metadata", {}))
        uid = exp.pop("_id")
        storage.update_experiment(uid=uid, **exp)


def main(args):
    print("Upgrading your database may damage your data. Make sure to make a backup before the "
          "upgrade and stop any other process that may read/write the database during the "
          "upgrade.")
    if not args.get("force"):
        action = ""
        while action not in ("y", "yes", "n", "no"):
            action = (input("Do you wish to proceed? (y/N) ").strip() or "n").lower()
        if action in ("n", "no"):
            sys.exit(0)
    if storage_is_set():
        storage = get_storage()
    else:
        import yaml
        cfg = {}
        if args.get("config"):
            with open(args["config"]) as f:
                cfg = yaml.safe_load(f) or {}
        from ...core.config import config as gc
        db = {k: gc.database[k] for k in ("type", "name", "host", "port")}
        db.update(cfg.get("database", {}))
        from ...storage.database import create_database
        of_type = db.pop("type")
        storage = DocumentStorage(create_database(of_type.lower(), **db), setup=False)
    upgrade_db_specifics(storage.database)
    print("Updating documents...")
    upgrade_documents(storage)
    storage._setup_db()
    print("Database upgrade completed successfully")
    return 0
