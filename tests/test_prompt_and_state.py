"""The interactive branching prompt driven programmatically (reference:
tests/unittests/core/io/interactive_commands/test_branching_prompt.py -- behaviour, not code),
and the MoptState test harness (reference ``core/utils/tests.py`` ``OrionState``)."""
import io

import pytest

from metaopt_amd.evc import conflicts as C
from metaopt_amd.evc.branch_builder import ExperimentBranchBuilder
from metaopt_amd.evc.prompt import BranchingPrompt
from metaopt_amd.storage import protocol
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.utils.testing import MockDatetime, MoptState


def _config(priors, name="exp", version=1, algorithms=None, vcs=None):
    return {"name": name, "version": version, "_id": f"{name}-{version}",
            "algorithms": algorithms or {"random": {"seed": None}},
            "metadata": {"priors": dict(priors), "user": "tester",
                         "user_args": [f"--{k.lstrip('/')}~{v}" for k, v in priors.items()],
                         **({"VCS": vcs} if vcs is not None else {})}}


@pytest.fixture
def prompt():
    st = DocumentStorage(EphemeralDB())
    with C.using_storage(st):
        old = _config({"/x": "uniform(0, 1)", "/y": "uniform(0, 1)"})
        new = _config({"/x": "uniform(0, 2)", "/z": "uniform(0, 1)"},
                      algorithms={"asha": {}}, vcs={"type": "git", "HEAD_sha": "abc"})
        builder = ExperimentBranchBuilder(C.detect_conflicts(old, new),
                                          {"manual_resolution": True})
        out = io.StringIO()
        yield BranchingPrompt(builder, stdin=io.StringIO(), stdout=out), out


def _run(p, out, line):
    out.truncate(0)
    out.seek(0)
    stop = p.onecmd(line)
    return stop, out.getvalue()


def test_status_lists_remaining_conflicts(prompt):
    p, out = prompt
    _, text = _run(p, out, "status")
    assert "Remaining conflicts" in text
    for frag in ("New z", "Missing y", "x~uniform(0, 1) != x~uniform(0, 2)"):
        assert frag in text


def test_resolve_step_by_step_then_commit(prompt):
    p, out = prompt
    stop, text = _run(p, out, "commit")
    assert not stop and "still conflicts" in text
    _run(p, out, "add z --default-value 0.5")
    _run(p, out, "add x")
    _run(p, out, "remove y")
    _run(p, out, "algo")
    _, text = _run(p, out, "code sideways")
    assert "Invalid change type" in text
    _run(p, out, "code noeffect")
    _, text = _run(p, out, "status")
    assert "Resolutions:" in text and "z~+uniform(0, 1, default_value=0.5)" in text
    stop, _ = _run(p, out, "commit")
    assert stop and not p.abort


def test_rename_reset_and_abort(prompt):
    p, out = prompt
    _run(p, out, "rename y z")
    _, text = _run(p, out, "status")
    assert "y~>z" in text
    _run(p, out, "reset 'y~>z'")
    _, text = _run(p, out, "status")
    assert "y~>z" not in text.split("Remaining conflicts")[0]
    _, text = _run(p, out, "rename y")
    assert "usage" in text
    stop, _ = _run(p, out, "abort")
    assert stop and p.abort


def test_completion_and_help(prompt):
    p, out = prompt
    assert p.complete_add("", "add ", 4, 4) == ["x", "z"] or \
        sorted(p.complete_add("", "add ", 4, 4)) == ["x", "z"]
    assert p.complete_remove("y", "remove y", 7, 8) == ["y"]
    _, text = _run(p, out, "help add")
    assert "add <dimension>" in text


def test_auto_resolves_what_it_can(prompt):
    p, out = prompt
    _, text = _run(p, out, "auto")
    assert "Resolutions:" in text


def test_moptstate_installs_and_restores_storage():
    before = getattr(protocol, "_STORAGE", None)
    exp = {"_id": 1, "name": "seeded", "version": 1, "metadata": {"user": "u"}}
    trial = {"_id": "t1", "experiment": 1, "status": "new", "params": [], "results": [],
             "parents": []}
    with MoptState(experiments=[exp], trials=[trial], storage="pickleddb") as state:
        st = protocol.get_storage()
        assert st is state.storage
        assert st.fetch_experiments({"name": "seeded"})[0]["version"] == 1
        assert st.database.read("trials", {"_id": "t1"})[0]["status"] == "new"
    assert getattr(protocol, "_STORAGE", None) is before
    assert MockDatetime.utcnow() == MockDatetime.frozen
