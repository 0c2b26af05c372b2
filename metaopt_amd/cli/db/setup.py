"""``mopt db setup``: write the database section of the user configuration file
(reference: ``cli/db/setup.py:22-85``)."""
from __future__ import annotations

import os

import yaml

from ...core.config import user_config_dir


def add_subparser(parser):
    p = parser.add_parser("setup", help="Create db configuration file")
    p.add_argument("--type", help="database type (pickleddb, ephemeraldb, mongodb)")
    p.add_argument("--name", help="database name")
    p.add_argument("--host", help="database host or file path")
    p.add_argument("--port", type=int, help="database port")
    p.add_argument("-f", "--force", action="store_true", help="overwrite without asking")
    p.add_argument("--config-file", help="where to write (default: the user config file)")
    p.set_defaults(func=main)
    return p


def ask_question(question, default=None):
    suffix = f" (default: {default})" if default is not None else ""
    answer = input(f"{question}{suffix} ")
    return answer.strip() or default


def main(args):
    path = args.get("config_file") or os.path.join(user_config_dir(), "mopt_config.yaml")
    if os.path.exists(path) and not args.get("force"):
        if ask_question(f"Config file {path} already exists. Overwrite? (y/N)", "n").lower() \
                not in ("y", "yes"):
            return 0
    cfg = {}
    if os.path.exists(path):
        with open(path) as f:
            cfg = yaml.safe_load(f) or {}
    db = {}
    db["type"] = args.get("type") or ask_question("Enter the database type:", "pickleddb")
    db["name"] = args.get("name") or ask_question("Enter the database name:", "mopt")
    db["host"] = args.get("host") or ask_question("Enter the database host:", "")
    if args.get("port"):
        db["port"] = args["port"]
    cfg["database"] = db
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f, default_flow_style=False)
    print(f"Database configuration written to {path}")
    return 0
