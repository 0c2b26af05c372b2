"""`status` output, character for character, against the expected strings of the reference's
functional tests (tests/functional/commands/test_status_command.py: one experiment with a trial
in every status, unrelated experiments, a parent and its child), on experiments built here
through init_only and storage writes."""
import datetime

import pytest

from metaopt_amd import cli
from metaopt_amd.core.trial import Trial
from metaopt_amd.storage import protocol

STATUSES = ("broken", "completed", "interrupted", "new", "reserved", "suspended")


@pytest.fixture
def env(tmp_path, monkeypatch):
    script = tmp_path / "box.py"
    script.write_text("print('never run here')\n")
    monkeypatch.setenv("MOPT_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", str(tmp_path / "db.pkl"))
    monkeypatch.chdir(tmp_path)
    for attr in ("_STORAGE", "_storage", "_instance"):
        if hasattr(protocol, attr):
            monkeypatch.setattr(protocol, attr, None)
    return str(script)


def _one_of_each(name, with_objective):
    """A trial in every status; the completed one has objective 0 (named 'obj') or none."""
    st = protocol.get_storage()
    exp = sorted(st.fetch_experiments({"name": name}), key=lambda e: e["version"])[-1]
    for i, status in enumerate(STATUSES):
        t = Trial(experiment=exp["_id"], status=status,
                  params=[dict(name="/x", type="real", value=float(i))])
        t.submit_time = datetime.datetime.utcnow()
        if status == "completed" and with_objective:
            t.results = [Trial.Result(name="obj", type="objective", value=0)]
            t.end_time = t.submit_time
        st.register_trial(t)


BLOCK_OBJ = """\
{name}
{bar}
status         quantity    min obj
-----------  ----------  ---------
broken                1
completed             1          0
interrupted           1
new                   1
reserved              1
suspended             1

"""

BLOCK_NO_OBJ = """\
{name}
{bar}
status         quantity
-----------  ----------
broken                1
completed             1
interrupted           1
new                   1
reserved              1
suspended             1

"""


def _block(template, name, indent=""):
    text = template.format(name=name, bar="=" * len(name))
    return "".join(indent + line if line.strip() else line
                   for line in text.splitlines(True)) + "\n"


def test_single_experiment_every_status(env, capsys):
    cli.main(["init_only", "-n", "test_single_exp", env, "-x~uniform(0, 10)"])
    _one_of_each("test_single_exp", with_objective=True)
    capsys.readouterr()
    cli.main(["status"])
    assert capsys.readouterr().out == _block(BLOCK_OBJ, "test_single_exp-v1")


def test_two_unrelated_experiments(env, capsys):
    # (created in the reference fixture's order: experiments are listed in database order)
    cli.main(["init_only", "-n", "test_double_exp", env, "-x~uniform(0, 10)"])
    cli.main(["init_only", "-n", "test_single_exp", env, "-x~uniform(0, 10)"])
    _one_of_each("test_single_exp", with_objective=True)
    _one_of_each("test_double_exp", with_objective=False)
    capsys.readouterr()
    cli.main(["status"])
    assert capsys.readouterr().out == (_block(BLOCK_NO_OBJ, "test_double_exp-v1") +
                                       _block(BLOCK_OBJ, "test_single_exp-v1"))


def test_parent_and_child(env, capsys):
    cli.main(["init_only", "-n", "test_double_exp", env, "-x~uniform(0, 10)"])
    _one_of_each("test_double_exp", with_objective=False)
    cli.main(["init_only", "-n", "test_double_exp", "--branch", "test_double_exp_child", env,
              "-x~uniform(0, 10)", "-y~+uniform(0, 1, default_value=0)"])
    _one_of_each("test_double_exp_child", with_objective=False)
    capsys.readouterr()
    cli.main(["status"])
    assert capsys.readouterr().out == (_block(BLOCK_NO_OBJ, "test_double_exp-v1") +
                                       _block(BLOCK_NO_OBJ, "test_double_exp_child-v1", "  "))


def test_no_experiment(env, capsys):
    cli.main(["status"])
    assert capsys.readouterr().out == "No experiment found\n"


def _ids_by_status(name):
    st = protocol.get_storage()
    exp = st.fetch_experiments({"name": name})[0]
    return {t.status: t.id for t in st.fetch_trials(uid=exp["_id"])}


def test_all_without_trials(env, capsys):
    cli.main(["init_only", "-n", "test_single_exp", env, "-x~uniform(0, 10)"])
    capsys.readouterr()
    cli.main(["status", "--all"])
    assert capsys.readouterr().out == """\
test_single_exp-v1
==================
id     status    best objective
-----  --------  ----------------
empty


"""


@pytest.mark.parametrize("with_objective", [True, False])
def test_all_trials(env, capsys, with_objective):
    cli.main(["init_only", "-n", "test_single_exp", env, "-x~uniform(0, 10)"])
    _one_of_each("test_single_exp", with_objective=with_objective)
    ids = _ids_by_status("test_single_exp")
    capsys.readouterr()
    cli.main(["status", "--all"])
    if with_objective:
        rows = "".join(f"{ids[s]}  {s:<11}" + ("          0" if s == "completed" else "") +
                       "\n" for s in STATUSES)
        head = ("id                                status         min obj\n"
                "--------------------------------  -----------  ---------\n")
    else:
        rows = "".join(f"{ids[s]}  {s}\n" for s in STATUSES)
        head = ("id                                status\n"
                "--------------------------------  -----------\n")
    want = "test_single_exp-v1\n==================\n" + head + rows + "\n\n"
    got = capsys.readouterr().out
    assert [line.rstrip() for line in got.split("\n")] == \
        [line.rstrip() for line in want.split("\n")]
