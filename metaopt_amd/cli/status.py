"""``mopt status [-a] [-C] [-e]``: an overview of the trials of every experiment.

Behaviour follows the reference's ``orion status`` (``src/orion/core/cli/status.py:25-233``):
one block per experiment -- the tree name underlined, then either a per-status table (count and
best objective) or, with ``--all``, one row per trial.  Experiments are shown as version trees:
an experiment whose tree holds other names (or ``--expand-versions``) lists each node indented
by depth; ``--collapse`` shows the latest version's view of the whole tree instead.

Built differently: a pass collects :class:`Block` records (title, depth, trials) from the EVC
tree, and one renderer turns any block into text, so the per-status and per-trial layouts share
the indentation and table code.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, List

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


@dataclass
class Block:
    """What one experiment node contributes to the report."""

    title: str
    depth: int
    trials: list


def main(args):
    builder = ExperimentBuilder()
    builder.setup_storage(builder.fetch_full_config(args, use_db=False))
    name, version = args.get("name"), args.get("version")
    per_trial = bool(args.get("all"))
    collapse, expand = bool(args.get("collapse")), bool(args.get("expand_versions"))
    if name is None and version and (collapse or expand):
        raise RuntimeError("Cannot fetch specific version of experiments with --collapse or "
                           "--expand-versions.")
    views = _experiment_views(builder, name)
    if not views:
        print("No experiment found")
        return 0
    roots = views[:1] if name else [v for v in views if v.refers.get("parent_id") is None]
    for root in roots:
        for block in _blocks(builder, root, version, collapse, expand):
            print(render(block, per_trial))
    return 0


def _experiment_views(builder, name):
    query = {"name": name} if name else {}
    docs = get_storage().fetch_experiments(query, {"name": 1, "version": 1})
    return [builder.build_view_from({"name": d["name"], "version": d.get("version", 1)})
            for d in docs]


def _blocks(builder, root, version, collapse, expand) -> Iterable[Block]:
    """Blocks of one root experiment: its tree node by node, or one collapsed block."""
    chosen = builder.build_view_from({"name": root.name, "version": version})
    anchor = root if version is None else chosen
    many_names = any(node.name != anchor.name for node in anchor.node)
    if (expand or many_names) and not collapse:
        yield from _walk(anchor, 0)
    else:
        yield Block(chosen.node.tree_name, 0, chosen.fetch_trials(with_evc_tree=True))


def _walk(exp, depth) -> Iterable[Block]:
    yield Block(exp.node.tree_name, depth, exp.fetch_trials(with_evc_tree=False))
    for child in exp.node.children:
        yield from _walk(child.item, depth + 1)


# ---------------------------------------------------------------------------------- rendering
def render(block: Block, per_trial: bool = False) -> str:
    pad = " " * (2 * block.depth)
    out: List[str] = [pad + block.title, pad + "=" * len(block.title)]
    if per_trial:
        headers, rows = _trial_rows(block.trials)
    elif block.trials:
        headers, rows = _status_rows(block.trials)
    else:
        headers, rows = None, None
    if headers is None:
        out.append(pad + "empty")
    else:
        out.extend(pad + line for line in tabulate.tabulate(rows, headers=headers).split("\n"))
    return "\n".join(out) + "\n\n"


def _status_rows(trials):
    """(status, count[, best objective]) per status, statuses in alphabetical order."""
    groups = {}
    for t in trials:
        groups.setdefault(t.status, []).append(t)
    headers, rows = ["status", "quantity"], []
    for status in sorted(groups):
        members = groups[status]
        row = [status, len(members)]
        scored = [t.objective for t in members if t.objective]
        if members[0].objective:   # the reference names the column after the first trial's
            headers.append(f"min {members[0].objective.name}")
            row.append(min(o.value for o in scored))
        rows.append(row)
    return headers, rows


def _trial_rows(trials):
    """(id, status[, objective]) per trial, grouped by status."""
    headers = ["id", "status", "best objective"]
    rows = []
    for t in sorted(trials, key=lambda t: t.status):
        obj = t.objective
        if obj:
            headers[2] = f"min {obj.name}"
        rows.append([t.id, t.status] + ([obj.value] if obj else []))
    return headers, rows or [["empty", "", ""]]
