"""``mopt info`` output contract (the format the reference pins in
tests/unittests/core/cli/test_info.py): titles, nested dict / list rendering with depth, width and
custom templates, and every section of a real experiment's report.  Expected strings are the
documented format; written against this package's API."""
import datetime

import pytest

from metaopt_amd.cli import info
from metaopt_amd.core.trial import Trial
from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage

NESTED = {"a": {"b": 1, "c": {"d": 2}}, "e": 3, "f": [], "g": {}}


def test_title():
    assert info.format_title("Stats") == "Stats\n====="
    assert info.format_title("Identification").splitlines()[1] == "=" * len("Identification")


@pytest.mark.parametrize("depth", [0, 1, 2, 3])
def test_dict_depth_indents_by_width(depth):
    out = info.format_dict({"k": 1}, depth=depth)
    assert out == " " * (4 * depth) + "k: 1"


@pytest.mark.parametrize("width", [0, 1, 2, 5])
def test_dict_width(width):
    out = info.format_dict({"k": {"j": 1}}, width=width)
    assert out == "k:\n" + " " * width + "j: 1"


def test_dict_full():
    assert info.format_dict(NESTED) == "a:\n    b: 1\n    c:\n        d: 2\ne: 3\nf\ng"


def test_dict_full_depth_one_width_two():
    assert info.format_dict(NESTED, depth=1, width=2) == \
        "  a:\n    b: 1\n    c:\n      d: 2\n  e: 3\n  f\n  g"


def test_dict_keys_sorted():
    assert info.format_dict({"b": 1, "a": 2}) == "a: 2\nb: 1"


def test_empty_leaf_templates():
    assert info.format_dict({"k": []}) == "k"
    assert info.format_dict({"k": []}, templates={"empty_leaf": "{tab}{key}=EMPTY\n"}) == \
        "k=EMPTY"


def test_leaf_template():
    assert info.format_dict({"k": 1}, templates={"leaf": "{tab}{key}={value}\n"}) == "k=1"


def test_node_template():
    assert info.format_dict({"k": {"j": 1}}, templates={"dict_node": "{tab}{key}->\n{value}\n"}) \
        == "k->\n    j: 1"


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_list_depth(depth):
    tab, sub = " " * (4 * depth), " " * (4 * (depth + 1))
    assert info.format_list([1, 2], depth=depth) == f"{tab}[\n{sub}1\n{sub}2\n{tab}]"


@pytest.mark.parametrize("width", [1, 3])
def test_list_width(width):
    assert info.format_list(["x"], width=width) == "[\n" + " " * width + "x\n]"


def test_list_of_lists_and_dicts():
    assert info.format_list([1, [2, 3], {"x": 1}]) == \
        "[\n    1\n    [\n        2\n        3\n    ]\n    x: 1\n]"


def test_list_templates():
    t = {"list": "{tab}<\n{items}\n{tab}>", "item": "{tab}{id}:{item}\n"}
    assert info.format_list([1, 2], templates=t) == "<\n    1:1\n    2:2\n>"


def test_list_node_template():
    t = {"list_node": "{tab}#{id}\n{item}\n"}
    assert info.format_list([{"a": 1}], templates=t) == "[\n    #1\n    a: 1\n]"


def test_dict_with_list():
    assert info.format_dict({"k": [1, {"a": 2}]}) == "k:\n    [\n        1\n        a: 2\n    ]"


def test_dict_given_a_list_formats_the_list():
    assert info.format_dict([1]) == info.format_list([1])


# ------------------------------------------------------------------ experiment sections
@pytest.fixture
def experiment():
    st = DocumentStorage(EphemeralDB())
    return build_experiment("info-exp", priors={"/x": "uniform(0, 1)", "/n": "uniform(1, 5, "
                                                "discrete=True)"},
                            algorithms={"random": {"seed": 3}}, max_trials=7, pool_size=2,
                            storage=st)


def _complete(exp, x, obj):
    t = Trial(experiment=exp.id, params=[dict(name="/n", type="integer", value=2),
                                         dict(name="/x", type="real", value=x)])
    exp.register_trial(t)
    t = exp.reserve_trial()
    t.results = [dict(name="o", type="objective", value=obj)]
    exp.update_completed_trial(t)
    return t


def test_identification(experiment):
    out = info.format_identification(experiment)
    assert out.startswith("Identification\n==============\nname: info-exp\nversion: 1\nuser: ")


def test_commandline(experiment):
    assert info.format_commandline(experiment).startswith("Commandline\n===========\n")


def test_config(experiment):
    assert info.format_config(experiment) == \
        "Config\n======\npool size: 2\nmax trials: 7\n"


def test_algorithm(experiment):
    assert info.format_algorithm(experiment) == "Algorithm\n=========\nrandom:\n    seed: 3\n"


def test_space(experiment):
    # the prior string shows the scipy (loc, scale) arguments, as in the reference
    assert info.format_space(experiment) == \
        "Space\n=====\n/n: uniform(1, 4)\n/x: uniform(0, 1)\n"


def test_metadata(experiment):
    out = info.format_metadata(experiment)
    assert out.startswith("Meta-data\n=========\nuser: ") and "orion version: " in out
    assert "datetime: " in out and "VCS:" in out


def test_refers_root(experiment):
    assert info.format_refers(experiment) == \
        "Parent experiment\n=================\nroot: \nparent: \nadapter: \n"


def test_stats_empty(experiment):
    assert info.format_stats(experiment) == "Stats\n=====\nNo trials executed...\n"


def test_stats_best_trial(experiment):
    _complete(experiment, 0.7, 3.0)
    best = _complete(experiment, 0.2, 1.0)
    out = info.format_stats(experiment)
    lines = out.splitlines()
    assert lines[:4] == ["Stats", "=====", "trials completed: 2", "best trial:"]
    assert f"  id: {best.id}" in lines and "  evaluation: 1.0" in lines
    assert "    /n: 2" in lines and "    /x: 0.2" in lines
    assert any(l.startswith("duration: ") for l in lines)


def test_full_report_has_every_section(experiment):
    _complete(experiment, 0.4, 2.0)
    out = info.format_info(experiment)
    titles = ["Identification", "Commandline", "Config", "Algorithm", "Space", "Meta-data",
              "Parent experiment", "Stats"]
    pos = [out.index(t + "\n" + "=" * len(t)) for t in titles]
    assert pos == sorted(pos)
