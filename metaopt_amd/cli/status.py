"""``mopt status [-a] [-C] [-e]``: per-status trial counts (reference: ``cli/status.py:25-233``)."""
from __future__ import annotations

import collections

import tabulate

from ..io.experiment_builder import ExperimentBuilder
from ..storage.protocol import get_storage
from .base import get_basic_args_group


def add_subparser(parser):
    p = parser.add_parser("status", help="Gives an overview of experiments' trials")
    get_basic_args_group(p)
    p.add_argument("-a", "--all", action="store_true",
                   help="Show all trials line by line. Otherwise, they are aggregated by status")
    p.add_argument("-C", "--collapse", action="store_true",
                   help="Aggregate together results of all child experiments.")
    p.add_argument("-e", "--expand-versions", action="store_true",
                   help="Show all the versions of every experiment instead of only the latest.")
    p.set_defaults(func=main)
    return p


def main(args):
    builder = ExperimentBuilder()
    local = builder.fetch_full_config(args, use_db=False)
    builder.setup_storage(local)
    args = dict(args)
    args["all_trials"] = args.pop("all", False)
    experiments = get_experiments(args, builder)
    if not experiments:
        print("No experiment found")
        return 0
    if args.get("name"):
        print_evc([experiments[0]], builder, **args)
        return 0
    if args.get("version") and (args.get("collapse") or args.get("expand_versions")):
        raise RuntimeError("Cannot fetch specific version of experiments with --collapse or "
                           "--expand-versions.")
    print_evc([e for e in experiments if e.refers.get("parent_id") is None], builder, **args)
    return 0


def get_experiments(args, builder):
    query = {"name": args["name"]} if args.get("name") else {}
    found = get_storage().fetch_experiments(query, {"name": 1, "version": 1})
    return [builder.build_view_from({"name": e["name"], "version": e.get("version", 1)})
            for e in found]


def _has_named_children(exp):
    return any(node.name != exp.name for node in exp.node)


def print_evc(experiments, builder, version=None, all_trials=False, collapse=False,
              expand_versions=False, **kwargs):
    for exp in experiments:
        experiment = builder.build_view_from({"name": exp.name, "version": version})
        expand_exp = exp if version is None else experiment
        expand = expand_versions or _has_named_children(expand_exp)
        if expand and not collapse:
            print_status_recursively(expand_exp, all_trials=all_trials)
        else:
            print_status(experiment, all_trials=all_trials, collapse=True)


def print_status_recursively(exp, depth=0, **kwargs):
    print_status(exp, offset=depth * 2, **kwargs)
    for child in exp.node.children:
        print_status_recursively(child.item, depth + 1, **kwargs)


def print_status(exp, offset=0, all_trials=False, collapse=False):
    trials = exp.fetch_trials(with_evc_tree=collapse)
    title = exp.node.tree_name
    print(" " * offset, title, sep="")
    print(" " * offset, "=" * len(title), sep="")
    if all_trials:
        print_all_trials(trials, offset=offset)
    else:
        print_summary(trials, offset=offset)


def print_summary(trials, offset=0):
    by_status = collections.defaultdict(list)
    for t in trials:
        by_status[t.status].append(t)
    headers = ["status", "quantity"]
    lines = []
    for status, ts in sorted(by_status.items()):
        line = [status, len(ts)]
        if ts[0].objective:
            headers.append(f"min {ts[0].objective.name}")
            line.append(min(t.objective.value for t in ts if t.objective))
        lines.append(line)
    if trials:
        grid = tabulate.tabulate(lines, headers=headers)
        tab = " " * offset
        print(tab + ("\n" + tab).join(grid.split("\n")))
    else:
        print(" " * offset, "empty", sep="")
    print("\n")


def print_all_trials(trials, offset=0):
    headers = ["id", "status", "best objective"]
    lines = []
    for t in sorted(trials, key=lambda t: t.status):
        line = [t.id, t.status]
        if t.objective:
            headers[-1] = f"min {t.objective.name}"
            line.append(t.objective.value)
        lines.append(line)
    if not trials:
        lines.append(["empty", "", ""])
    grid = tabulate.tabulate(lines, headers=headers)
    tab = " " * offset
    print(tab + ("\n" + tab).join(grid.split("\n")))
    print("\n")
