"""Small host utilities (reference tests: tests/unittests/core/test_utils.py, utils/test_flatten.py,
core/test_working_dir.py, core/utils/test_format_trials.py -- behaviour, not code)."""
import os

import numpy
import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.space.dims import Real, Space
from metaopt_amd.utils.diff import GREEN, RED, colored_diff
from metaopt_amd.utils.flatten import flatten, unflatten
from metaopt_amd.utils.format_trials import (dict_to_trial, get_trial_results,
                                             standard_param_name, trial_to_tuple, tuple_to_trial)
from metaopt_amd.utils.points import flatten_dims, flatten_points, regroup_dims
from metaopt_amd.utils.pptree import format_tree
from metaopt_amd.utils.working_dir import WorkingDir


def _space():
    s = Space()
    s.register(Real("/x", "uniform", 0, 1))
    s.register(Real("/w", "uniform", 0, 1, shape=(2, 2)))
    return s


def test_flatten_roundtrip_keeps_empty_dicts():
    nested = {"a": {"b": 1, "c": {"d": [1, 2]}}, "e": {}, "f": "x"}
    flat = flatten(nested)
    assert flat == {"a.b": 1, "a.c.d": [1, 2], "e": {}, "f": "x"}
    assert unflatten(flat) == nested


def test_points_flatten_and_regroup_shaped_dims():
    space = _space()
    point = (0.5, numpy.arange(4.0).reshape(2, 2)) if list(space.keys())[0] == "/x" else \
        (numpy.arange(4.0).reshape(2, 2), 0.5)
    flat = flatten_dims(point, space)
    assert len(flat) == 5
    back = regroup_dims(flat, space)
    for a, b in zip(back, point):
        numpy.testing.assert_array_equal(numpy.asarray(a), numpy.asarray(b))
    assert flatten_points([point, point], space) == [flat, flat]
    with pytest.raises(ValueError, match="does not match"):
        regroup_dims(flat + [1.0], space)


def test_working_dir_temp_and_persistent(tmp_path):
    with WorkingDir(tmp_path / "wd", temp=True, prefix="exp_", suffix="_t") as path:
        assert os.path.isdir(path) and os.path.basename(path).startswith("exp_")
        inside = path
    assert not os.path.exists(inside)
    with WorkingDir(tmp_path / "wd", temp=False, prefix="exp_", suffix="abc") as path:
        assert path == str(tmp_path / "wd" / "exp_abc")
    assert os.path.isdir(path)


def test_trial_tuple_roundtrip_and_results():
    space = Space()
    space.register(Real("/x", "uniform", 0, 1))
    space.register(Real("/y", "uniform", 0, 1))
    trial = tuple_to_trial((0.25, 0.75), space)
    assert trial_to_tuple(trial, space) == (0.25, 0.75)
    assert trial_to_tuple(dict_to_trial({"/y": 0.75, "/x": 0.25}, space), space) == (0.25, 0.75)
    with pytest.raises(ValueError):
        tuple_to_trial((0.1,), space)
    trial.results = [Trial.Result(name="loss", type="objective", value=1.5),
                     Trial.Result(name="c", type="constraint", value=0.1),
                     Trial.Result(name="g", type="gradient", value=[1.0, 2.0])]
    assert get_trial_results(trial) == {"objective": 1.5, "constraint": [0.1],
                                        "gradient": (1.0, 2.0)}
    trial.results.append(Trial.Result(name="lie", type="lie", value=9.0))
    assert get_trial_results(trial)["objective"] == 9.0      # the lie takes precedence
    assert standard_param_name("/learning-rate") == "learning_rate"


def test_colored_diff_and_tree():
    d = colored_diff("a\nb\n", "a\nc\n")
    assert RED + "-b" in d and GREEN + "+c" in d

    class N:
        def __init__(self, name, children=()):
            self.name, self.children = name, list(children)

    text = format_tree(N("root", [N("v1", [N("v1.1")]), N("v2")]), name=lambda n: n.name)
    assert text.splitlines() == ["root", "├──v1", "│  └──v1.1", "└──v2"]
