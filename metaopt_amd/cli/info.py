"""``mopt info -n exp``: detailed description of an experiment (reference: ``cli/info.py:21-439``).

Sections: Identification, Commandline, Config, Algorithm, Space, Meta-data, Parent experiment,
Stats -- same templates as the reference so its output-format tests carry over.
"""
from __future__ import annotations

import sys

from ..io.experiment_builder import ExperimentBuilder
from .base import get_basic_args_group


def add_subparser(parser):
    p = parser.add_parser("info", help="Gives detailed information about an experiment")
    get_basic_args_group(p)
    p.set_defaults(func=main)
    return p


def main(args):
    try:
        experiment = ExperimentBuilder().build_view_from(args)
    except ValueError:
        print(f"Experiment {args.get('name', None)} not found in db.")
        sys.exit(1)
    print(format_info(experiment))
    return 0


INFO_TEMPLATE = """\
{identification}
{commandline}
{configuration}
{algorithm}
{space}
{metadata}
{refers}
{stats}
"""


def format_info(experiment):
    return INFO_TEMPLATE.format(
        identification=format_identification(experiment),
        commandline=format_commandline(experiment),
        configuration=format_config(experiment),
        algorithm=format_algorithm(experiment),
        space=format_space(experiment),
        metadata=format_metadata(experiment),
        refers=format_refers(experiment),
        stats=format_stats(experiment))


def format_title(title):
    return f"{title}\n{'=' * len(title)}"


def format_dict(dictionary, depth=0, width=4, templates=None):
    if isinstance(dictionary, (list, tuple)):
        return format_list(dictionary, depth, width=width, templates=templates)
    templates = templates or {}
    empty_leaf = templates.get("empty_leaf", "{tab}{key}\n")
    leaf = templates.get("leaf", "{tab}{key}: {value}\n")
    node = templates.get("dict_node", "{tab}{key}:\n{value}\n")
    out = ""
    for key in sorted(dictionary.keys(), key=str):
        tab = " " * (depth * width)
        value = dictionary[key]
        if isinstance(value, (dict, list, tuple)):
            if not value:
                out += empty_leaf.format(tab=tab, key=key)
            else:
                out += node.format(tab=tab, key=key,
                                   value=format_dict(value, depth + 1, width=width,
                                                     templates=templates))
        else:
            out += leaf.format(tab=tab, key=key, value=value)
    return out.replace(" \n", "\n").rstrip("\n")


def format_list(a_list, depth=0, width=4, templates=None):
    templates = templates or {}
    list_t = templates.get("list", "{tab}[\n{items}\n{tab}]")
    item_t = templates.get("item", "{tab}{item}\n")
    node_t = templates.get("list_node", "{item}\n")
    tab = " " * (depth * width)
    items = ""
    for i, item in enumerate(a_list, 1):
        subtab = " " * ((depth + 1) * width)
        if isinstance(item, (dict, list, tuple)):
            items += node_t.format(tab=subtab, id=i,
                                   item=format_dict(item, depth + 1, width=width,
                                                    templates=templates))
        else:
            items += item_t.format(tab=subtab, id=i, item=item)
    return list_t.format(tab=tab, items=items.rstrip("\n"))


def format_identification(experiment):
    return (f"{format_title('Identification')}\nname: {experiment.name}\n"
            f"version: {experiment.version}\nuser: {experiment.metadata['user']}\n")


def format_commandline(experiment):
    return (f"{format_title('Commandline')}\n"
            f"{' '.join(experiment.metadata.get('user_args', []))}\n")


def format_config(experiment):
    return (f"{format_title('Config')}\npool size: {experiment.pool_size}\n"
            f"max trials: {experiment.max_trials}\n")


def format_algorithm(experiment):
    return f"{format_title('Algorithm')}\n{format_dict(experiment.configuration['algorithms'])}\n"


def format_space(experiment):
    space = experiment.space
    params = "\n".join(f"{name}: {space[name].get_prior_string()}" for name in space.keys())
    return f"{format_title('Space')}\n{params}\n"


def format_metadata(experiment):
    md = experiment.metadata
    return (f"{format_title('Meta-data')}\nuser: {md['user']}\ndatetime: {md.get('datetime')}\n"
            f"orion version: {md.get('orion_version')}\nVCS:\n"
            f"{format_dict(md.get('VCS', {}) or {}, depth=1, width=2)}\n")


def format_refers(experiment):
    node = experiment.node
    if node is None or node.root is node:
        root = parent = adapter = ""
    else:
        root = node.root.name
        parent = node.parent.name
        adapter = "\n" + format_dict(experiment.refers["adapter"].configuration, depth=1, width=2)
    return (f"{format_title('Parent experiment')}\nroot: {root}\nparent: {parent}\n"
            f"adapter: {adapter}\n")


def format_stats(experiment):
    stats = experiment.stats
    if not stats:
        return f"{format_title('Stats')}\nNo trials executed...\n"
    best = experiment.get_trial(uid=stats["best_trials_id"])
    params = {p.name: p.value for p in best.params} if best else {}
    return (f"{format_title('Stats')}\ntrials completed: {stats['trials_completed']}\n"
            f"best trial:\n  id: {stats['best_trials_id']}\n"
            f"  evaluation: {stats['best_evaluation']}\n  params:\n"
            f"{format_dict(params, depth=2, width=2)}\n"
            f"start time: {stats['start_time']}\nfinish time: {stats['finish_time']}\n"
            f"duration: {stats['duration']}\n")
