"""Branching prompt, command by command (the behaviour the reference pins in
tests/unittests/core/io/interactive_commands/test_branching_prompt.py): add / remove / rename
with and without default values (real and categorical), repeated and invalid commands, change
types of code / command line / script config, the algorithm conflict, the experiment name,
reset of single and multiple resolutions, status / diff / auto / commit / abort / shell / help.
Written against this package's prompt, driven with ``onecmd``."""
import io

import pytest

from metaopt_amd.evc import conflicts as C
from metaopt_amd.evc.branch_builder import ExperimentBranchBuilder
from metaopt_amd.evc.prompt import BranchingPrompt
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage

VCS_OLD = {"type": "git", "HEAD_sha": "a", "is_dirty": False, "active_branch": None,
           "diff_sha": "d"}


def _config(priors, algorithms=None, vcs=None, extra_args=(), name="exp"):
    return {"name": name, "version": 1, "_id": f"{name}-1",
            "algorithms": algorithms or {"random": {"seed": None}},
            "metadata": {"priors": dict(priors), "user": "tester",
                         "user_args": [f"--{k.lstrip('/')}~{v}" for k, v in priors.items()]
                         + list(extra_args),
                         **({"VCS": vcs} if vcs is not None else {})}}


OLD = {"/x": "uniform(0, 1)", "/y": "uniform(0, 1)", "/c": "choices(['a', 'b'])"}
NEW = {"/x": "uniform(0, 2)", "/z": "uniform(0, 1)", "/d": "choices(['a', 'b'])"}


@pytest.fixture
def prompt():
    st = DocumentStorage(EphemeralDB())
    with C.using_storage(st):
        old = _config(OLD, vcs=VCS_OLD, extra_args=["--epochs", "10"])
        new = _config(NEW, algorithms={"asha": {}}, vcs=dict(VCS_OLD, HEAD_sha="abc"),
                      extra_args=["--epochs", "20"])
        builder = ExperimentBranchBuilder(C.detect_conflicts(old, new),
                                          {"manual_resolution": True})
        out = io.StringIO()
        yield BranchingPrompt(builder, stdin=io.StringIO(), stdout=out), out


def run(prompt, line):
    p, out = prompt
    out.truncate(0)
    out.seek(0)
    stop = p.onecmd(line)
    return stop, out.getvalue()


def status(prompt):
    return run(prompt, "status")[1]


def resolutions(prompt):
    return status(prompt).split("Remaining conflicts")[0]


def remaining(prompt):
    text = status(prompt)
    return text.split("Remaining conflicts")[1] if "Remaining conflicts" in text else ""


# ------------------------------------------------------------------ dimensions
def test_add_new_dimension(prompt):
    run(prompt, "add z")
    assert "z~+uniform(0, 1)" in resolutions(prompt) and "New z" not in remaining(prompt)


def test_add_unknown_dimension(prompt):
    _, text = run(prompt, "add nope")
    assert "Invalid" in text and "'nope' not found" in text


def test_add_twice(prompt):
    run(prompt, "add z")
    _, text = run(prompt, "add z")
    assert "Invalid" in text


def test_add_with_default(prompt):
    run(prompt, "add z --default-value 0.5")
    assert "z~+uniform(0, 1, default_value=0.5)" in resolutions(prompt)


def test_add_with_bad_default(prompt, capsys):
    run(prompt, "add z --default-value 3")
    assert "New z" in remaining(prompt)
    assert "outside of dimension's prior interval" in capsys.readouterr().out


def test_add_categorical_with_default(prompt):
    run(prompt, "add d --default-value b")
    assert "d~+choices(['a', 'b'], default_value='b')" in resolutions(prompt)


def test_add_categorical_with_bad_default(prompt, capsys):
    run(prompt, "add d --default-value q")
    assert "New d" in remaining(prompt)
    assert "Invalid category" in capsys.readouterr().out


def test_change_dimension(prompt):
    run(prompt, "add x")
    assert "x~+uniform(0, 2)" in resolutions(prompt)
    assert "x~uniform(0, 1) != x~uniform(0, 2)" not in remaining(prompt)


def test_change_twice(prompt):
    run(prompt, "add x")
    _, text = run(prompt, "add x")
    assert "Invalid" in text


def test_remove_missing_dimension(prompt):
    run(prompt, "remove y")
    assert "y~-" in resolutions(prompt) and "Missing y" not in remaining(prompt)


def test_remove_unknown(prompt):
    assert "Invalid" in run(prompt, "remove nope")[1]


def test_remove_twice(prompt):
    run(prompt, "remove y")
    assert "Invalid" in run(prompt, "remove y")[1]


def test_remove_with_default(prompt):
    run(prompt, "remove y --default-value 0.3")
    assert "y~-0.3" in resolutions(prompt)


def test_remove_categorical_with_default(prompt):
    run(prompt, "remove c --default-value a")
    assert "c~-'a'" in resolutions(prompt)


def test_remove_categorical_bad_default(prompt, capsys):
    run(prompt, "remove c --default-value q")
    assert "Missing c" in remaining(prompt)
    assert "Invalid category" in capsys.readouterr().out


def test_rename(prompt):
    run(prompt, "rename y z")
    res = resolutions(prompt)
    assert "y~>z" in res
    rem = remaining(prompt)
    assert "Missing y" not in rem and "New z" not in rem


def test_rename_bad_arguments(prompt):
    assert "usage" in run(prompt, "rename y")[1]
    assert "Invalid" in run(prompt, "rename nope z")[1]


def test_rename_onto_an_existing_dimension_is_refused(prompt):
    # x exists in both configurations (its prior changed): it is no new dimension
    assert "Invalid" in run(prompt, "rename y x")[1]
    assert "Missing y" in remaining(prompt)


def test_reset_add(prompt):
    run(prompt, "add z")
    run(prompt, "reset 'z~+uniform(0, 1)'")
    assert "New z" in remaining(prompt)


def test_reset_remove(prompt):
    run(prompt, "remove y")
    run(prompt, "reset y~-")
    assert "Missing y" in remaining(prompt)


def test_reset_rename_restores_both_conflicts(prompt):
    run(prompt, "rename y z")
    run(prompt, "reset 'y~>z'")
    rem = remaining(prompt)
    assert "Missing y" in rem and "New z" in rem


def test_reset_unknown(prompt):
    assert "Invalid" in run(prompt, "reset 'q~-'")[1]


def test_reset_many(prompt):
    run(prompt, "add z")
    run(prompt, "remove y")
    run(prompt, "reset 'z~+uniform(0, 1)' y~-")
    rem = remaining(prompt)
    assert "New z" in rem and "Missing y" in rem


# ------------------------------------------------------------------ change types
@pytest.mark.parametrize("cmd", ["noeffect", "break", "unsure"])
def test_code_change_types(prompt, cmd):
    run(prompt, f"code {cmd}")
    assert f"--code-change-type {cmd}" in resolutions(prompt)


def test_code_change_bad_type(prompt):
    _, text = run(prompt, "code sideways")
    assert "Invalid change type" in text and "Old hash commit" in remaining(prompt)


def test_code_change_twice(prompt):
    run(prompt, "code break")
    assert "Invalid" in run(prompt, "code noeffect")[1]


def test_reset_code(prompt):
    run(prompt, "code break")
    run(prompt, "reset '--code-change-type break'")
    assert "Old hash commit" in remaining(prompt)


def test_commandline_change_without_parser_state(prompt):
    # the non-prior arguments are compared through the stored parser state (metadata.parser),
    # absent here: no command-line conflict
    assert "No CommandLineConflict" in run(prompt, "commandline noeffect")[1]


def test_commandline_bad_type(prompt):
    assert "Invalid change type" in run(prompt, "commandline oops")[1]


def test_config_change_without_conflict(prompt):
    assert "No ScriptConfigConflict" in run(prompt, "config break")[1]


def test_algo(prompt):
    run(prompt, "algo")
    assert "--algorithm-change" in resolutions(prompt)


def test_algo_twice(prompt):
    run(prompt, "algo")
    assert "No AlgorithmConflict" in run(prompt, "algo")[1]


def test_reset_algo(prompt):
    run(prompt, "algo")
    run(prompt, "reset --algorithm-change")
    assert "{'asha': {}}" in remaining(prompt)


# ------------------------------------------------------------------ session
def test_commit_refused_until_resolved(prompt):
    stop, text = run(prompt, "commit")
    assert not stop and "There are still conflicts to solve" in text


def test_commit_when_resolved(prompt):
    for line in ("add z", "add d", "add x", "remove y", "remove c --default-value a", "algo",
                 "code noeffect"):
        run(prompt, line)
    stop, _ = run(prompt, "commit")
    p, _ = prompt
    assert stop and not p.abort


def test_auto(prompt):
    _, text = run(prompt, "auto")
    assert "Resolutions:" in text


def test_diff(prompt):
    _, text = run(prompt, "diff")
    assert "-uniform(0, 1)" in text and "+uniform(0, 2)" in text


@pytest.mark.parametrize("cmd", ["abort", "quit", "q", "EOF"])
def test_exits(prompt, cmd):
    stop, _ = run(prompt, cmd)
    assert stop and prompt[0].abort


def test_shell(prompt):
    assert run(prompt, "shell echo hi")[1].strip() == "hi"


def test_help(prompt):
    assert "current status" in run(prompt, "h status")[1]
    assert "rename <old-name> <new-name>" in run(prompt, "help rename")[1]


def test_completion(prompt):
    p, _ = prompt
    assert sorted(p.complete_add("", "add ", 4, 4)) == ["d", "x", "z"]
    assert sorted(p.complete_remove("", "remove ", 7, 7)) == ["c", "y"]
    assert p.complete_rename("z", "rename z", 7, 8) == ["z"]


def test_intro_contains_status(prompt):
    p, _ = prompt
    assert "Remaining conflicts" in p.intro % p.get_status()
