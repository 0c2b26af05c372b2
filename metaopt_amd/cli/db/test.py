"""``mopt db test``: check the database configuration in three stages
(reference: ``cli/db/test.py:24-57`` and ``cli/checks/{presence,creation,operations}.py``).

1. presence -- where the configuration comes from (defaults, environment, file);
2. creation -- the backend can be instantiated and connected;
3. operations -- write / read / count / remove round-trip on a scratch collection.
"""
from __future__ import annotations

import os

from ...core.config import config as global_config
from ...storage.database import create_database
from ...utils.exceptions import CheckError


def add_subparser(parser):
    p = parser.add_parser("test", help="Run a series of checks on the database")
    p.add_argument("-c", "--config", help="mopt configuration file (YAML)")
    p.set_defaults(func=main)
    return p


class PresenceStage:
    def __init__(self, cmdargs):
        self.cmdargs = cmdargs
        self.db_config = {}

    def checks(self):
        yield self.check_default_config
        yield self.check_environment_vars
        yield self.check_configuration_file

    def check_default_config(self):
        self.db_config = {k: global_config.database[k] for k in ("type", "name", "host", "port")}
        return "Success", ""

    def check_environment_vars(self):
        env = global_config.env_vars().get("database", {})
        self.db_config.update(env)
        return ("Success", "") if env else ("Skipping", "No environment variables found.")

    def check_configuration_file(self):
        path = self.cmdargs.get("config")
        if not path:
            return "Skipping", "No configuration file found."
        import yaml
        with open(path) as f:
            cfg = yaml.safe_load(f) or {}
        if "database" not in cfg:
            return "Skipping", "No database found in configuration file."
        section = cfg["database"] or {}
        if not any(k in section for k in ("type", "name", "host", "port")):
            return "Skipping", "No configuration value found inside `database`."
        self.db_config.update(section)
        return "Success", ""

    def post_stage(self):
        print(f"Using configuration: {self.db_config}")


class CreationStage:
    def __init__(self, presence):
        self.presence = presence
        self.instance = None

    def checks(self):
        yield self.check_database_creation

    def check_database_creation(self):
        cfg = dict(self.presence.db_config)
        of_type = cfg.pop("type", "pickleddb")
        try:
            self.instance = create_database(of_type.lower(), **cfg)
        except Exception as exc:
            raise CheckError(str(exc)) from exc
        return "Success", ""


class OperationsStage:
    def __init__(self, creation):
        self.creation = creation

    def checks(self):
        yield self.check_write
        yield self.check_read
        yield self.check_count
        yield self.check_remove

    @property
    def db(self):
        return self.creation.instance

    def check_write(self):
        self.db.write("test", {"index": "value"})
        return "Success", ""

    def check_read(self):
        if not self.db.read("test", {"index": "value"}):
            raise CheckError("Expected to read a document")
        return "Success", ""

    def check_count(self):
        n = self.db.count("test", {"index": "value"})
        if n != 1:
            raise CheckError(f"Expected 1 document, found {n}")
        return "Success", ""

    def check_remove(self):
        self.db.remove("test", {"index": "value"})
        if self.db.count("test", {"index": "value"}) != 0:
            raise CheckError("Expected 0 document after remove")
        return "Success", ""


def main(args):
    presence = PresenceStage(args)
    creation = CreationStage(presence)
    operations = OperationsStage(creation)
    for stage in (presence, creation, operations):
        for check in stage.checks():
            name = check.__name__.replace("check_", "").replace("_", " ")
            try:
                status, msg = check()
                print(f"{name}... {status}" + (f" ({msg})" if msg else ""))
            except CheckError as exc:
                print(f"{name}... Failure\n{exc}")
                return 1
        post = getattr(stage, "post_stage", None)
        if post is not None:
            post()
    return 0
