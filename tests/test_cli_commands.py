"""CLI commands on a PickledDB without running trials: init_only / insert to build experiments,
then the exact output of status (-a, -C, -e), info and list, the db setup / test / upgrade
commands and the deprecated aliases (reference: tests/functional/commands/test_status_command.py,
test_info_command.py, test_list_command.py, test_insert_command.py, test_db_commands --
behaviour re-specified on this implementation's output)."""
import datetime
import pytest
import yaml

from metaopt_amd import cli
from metaopt_amd.core.trial import Trial
from metaopt_amd.storage import protocol


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


def _run(*argv):
    return cli.main(list(argv))


def _complete(name, values, status="completed"):
    """Mark the first len(values) new trials of experiment ``name`` with objective values."""
    st = protocol.get_storage()
    exp = st.fetch_experiments({"name": name})[-1]
    trials = sorted(st.fetch_trials(uid=exp["_id"]), key=lambda t: t.params[0].value)
    for t, v in zip(trials, values):
        t.status = status
        t.results = [Trial.Result(name="loss", type="objective", value=v)]
        t.end_time = datetime.datetime.utcnow()
        st.push_trial_results(t)
    return trials


def _lines(out):
    return [line.rstrip() for line in out.strip("\n").split("\n")]


def test_status_without_experiments(env, capsys):
    _run("status")
    assert capsys.readouterr().out.strip() == "No experiment found"


def test_status_summary_and_all(env, capsys):
    _run("init_only", "-n", "exp", env, "-x~uniform(0, 10)")
    for x in ("1", "2", "3"):
        _run("insert", "-n", "exp", env, f"-x={x}")
    capsys.readouterr()
    trials = _complete("exp", [5.0, 4.0])
    _run("status")
    lines = _lines(capsys.readouterr().out)
    assert lines[0] == "exp-v1" and lines[1] == "======"
    assert lines[2].split() == ["status", "quantity", "min", "loss"]
    assert lines[4].split() == ["completed", "2", "4"]
    assert lines[5].split() == ["new", "1"]
    _run("status", "--all")
    lines = _lines(capsys.readouterr().out)
    assert lines[2].split() == ["id", "status", "min", "loss"]
    rows = [line.split() for line in lines[4:]]
    assert sorted(r[0] for r in rows) == sorted(t.id for t in trials)
    assert [r[1] for r in rows] == ["completed", "completed", "new"]


def test_status_versions_collapse_and_expand(env, capsys):
    _run("init_only", "-n", "tree", env, "-x~uniform(0, 10)")
    _run("insert", "-n", "tree", env, "-x=1")
    _complete("tree", [1.0])
    # adding a dimension makes version 2, a child of version 1
    _run("init_only", "-n", "tree", env, "-x~uniform(0, 10)", "-y~+uniform(0, 1, default_value=0)")
    _run("insert", "-n", "tree", "-v", "2", env, "-x=2", "-y=0.5")
    capsys.readouterr()
    _run("status", "--expand-versions")
    out = capsys.readouterr().out
    lines = _lines(out)
    assert lines[0] == "tree-v1" and "  tree-v2" in lines and "  =======" in lines
    _run("status", "--collapse")
    lines = _lines(capsys.readouterr().out)
    # latest version's view of the whole tree: the parent's completed trial flows through the
    # addition adapter (default value 0) next to the child's own new trial
    assert lines[0] == "tree-v2"
    rows = {line.split()[0]: line.split()[1:] for line in lines[4:] if line.strip()}
    assert rows["completed"][0] == "1" and rows["new"][0] == "1"
    _run("status", "-n", "tree", "-v", "1")
    lines = _lines(capsys.readouterr().out)
    assert lines[0] == "tree-v1"


def test_status_version_with_collapse_rejected(env):
    _run("init_only", "-n", "e", env, "-x~uniform(0, 1)")
    with pytest.raises(RuntimeError):
        _run("status", "-v", "1", "--collapse")


def test_info_sections(env, capsys):
    _run("init_only", "-n", "inf", "--max-trials", "7", env, "-x~loguniform(1e-3, 1)")
    _run("insert", "-n", "inf", env, "-x=0.1")
    _complete("inf", [0.25])
    capsys.readouterr()
    _run("info", "-n", "inf")
    out = capsys.readouterr().out
    for title in ("Identification", "Commandline", "Config", "Algorithm", "Space", "Meta-data",
                  "Parent experiment", "Stats"):
        assert f"{title}\n{'=' * len(title)}" in out
    assert "name: inf" in out and "version: 1" in out and "max trials: 7" in out
    assert "/x: reciprocal(0.001, 1)" in out or "/x: loguniform(0.001, 1)" in out
    assert "trials completed: 1" in out and "  evaluation: 0.25" in out
    assert "/x: 0.1" in out and "duration: " in out


def test_info_missing_experiment(env, capsys):
    with pytest.raises(SystemExit):
        _run("info", "-n", "nope")
    assert "not found" in capsys.readouterr().out


def test_list_tree(env, capsys):
    _run("init_only", "-n", "root", env, "-x~uniform(0, 1)")
    _run("init_only", "-n", "root", "--branch", "leaf", env, "-x~uniform(0, 1)",
         "-y~+uniform(0, 1, default_value=0.5)")
    _run("init_only", "-n", "other", env, "-z~uniform(0, 1)")
    capsys.readouterr()
    _run("list")
    out = capsys.readouterr().out
    assert "root-v1" in out and "leaf-v1" in out and "other-v1" in out
    assert out.index("root-v1") < out.index("leaf-v1")
    _run("list", "-n", "other")
    out = capsys.readouterr().out
    assert "other-v1" in out and "root" not in out


def test_insert_validates_against_space(env, capsys):
    _run("init_only", "-n", "ins", env, "-x~uniform(0, 1)")
    with pytest.raises(ValueError):
        _run("insert", "-n", "ins", env, "-x=3")        # outside the prior's support
    _run("insert", "-n", "ins", env, "-x=0.5")
    st = protocol.get_storage()
    exp = st.fetch_experiments({"name": "ins"})[0]
    trials = st.fetch_trials(uid=exp["_id"])
    assert [t.params[0].value for t in trials] == [0.5]


def test_db_setup_test_and_upgrade(env, tmp_path, capsys, monkeypatch):
    cfg_path = tmp_path / "conf" / "mopt_config.yaml"
    _run("db", "setup", "--type", "pickleddb", "--name", "n1", "--host",
         str(tmp_path / "other.pkl"), "--config-file", str(cfg_path), "-f")
    written = yaml.safe_load(cfg_path.read_text())
    assert written["database"] == {"type": "pickleddb", "name": "n1",
                                   "host": str(tmp_path / "other.pkl")}
    capsys.readouterr()
    _run("db", "test")
    out = capsys.readouterr().out
    assert out.count("Success") >= 5 and "Failure" not in out
    _run("init_only", "-n", "up", env, "-x~uniform(0, 1)")
    st = protocol.get_storage()
    exp = st.fetch_experiments({"name": "up"})[0]
    # simulate an old document: no version, no priors
    st._db.write("experiments", {"version": None}, {"_id": exp["_id"]})
    capsys.readouterr()
    _run("db", "upgrade", "-f")
    assert "completed successfully" in capsys.readouterr().out
    exp = st.fetch_experiments({"name": "up"})[0]
    assert exp["version"] in (1, None) and exp["metadata"]["priors"] == {"/x": "uniform(0, 1)"}


def test_deprecated_aliases(env, capsys):
    _run("test-db")
    assert "Success" in capsys.readouterr().out
