"""``mopt list``: print the EVC trees of the experiments (reference: ``cli/list.py:32-54``)."""
from __future__ import annotations

from ..io.experiment_builder import ExperimentBuilder
from ..storage.protocol import get_storage
from ..utils.pptree import print_tree
from .base import get_basic_args_group


def add_subparser(parser):
    p = parser.add_parser("list", help="Gives a list of experiments and their relationships.")
    get_basic_args_group(p)
    p.set_defaults(func=main)
    return p


def main(args):
    builder = ExperimentBuilder()
    local = builder.fetch_full_config(args, use_db=False)
    builder.setup_storage(local)
    query = {"name": args["name"]} if args.get("name") else {}
    experiments = get_storage().fetch_experiments(query, {"name": 1, "version": 1,
                                                          "refers": 1})
    if args.get("name"):
        roots = experiments
    else:
        roots = [e for e in experiments if (e.get("refers") or {}).get("parent_id") is None]
    if not roots:
        print("No experiment found")
        return 0
    for root in roots:
        view = builder.build_view_from({"name": root["name"], "version": root.get("version", 1),
                                        "debug": args.get("debug")})
        print_tree(view.node, name=lambda n: n.tree_name)
        print()
    return 0
