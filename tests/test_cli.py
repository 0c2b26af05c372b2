"""End-to-end CLI (reference tests/functional/demo and commands): hunt a black-box script with a
PickledDB, then status / list / info / insert / init_only --branch, asserting on DB documents and
printed output."""
import os
import sys
import textwrap

import pytest

from metaopt_amd import cli
from metaopt_amd.storage import protocol

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def env(tmp_path, monkeypatch):
    script = tmp_path / "black_box.py"
    script.write_text(textwrap.dedent(f"""\
        import argparse, sys
        sys.path.insert(0, {REPO!r})
        from metaopt_amd.client import report_results
        p = argparse.ArgumentParser()
        p.add_argument("-x", type=float, required=True)
        a = p.parse_args()
        report_results([{{"name": "obj", "type": "objective",
                          "value": (a.x - 34.56789) ** 2 + 23.4}}])
        """))
    broken = tmp_path / "broken_box.py"
    broken.write_text("import sys\nsys.exit(1)\n")
    monkeypatch.setenv("MOPT_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", str(tmp_path / "db.pkl"))
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(protocol, "_STORAGE", None, raising=False)
    for attr in ("_storage", "_instance"):
        if hasattr(protocol, attr):
            monkeypatch.setattr(protocol, attr, None)
    return script, broken


def _run(*argv):
    return cli.main(list(argv))


def test_hunt_status_list_info_insert_branch(env, capsys):
    script, _ = env
    assert _run("hunt", "-n", "demo", "--max-trials", "5", str(script), "-x~uniform(-50, 50)") == 0
    capsys.readouterr()
    _run("status")
    out = capsys.readouterr().out
    assert "demo-v1" in out and "completed           5" in out
    _run("info", "-n", "demo")
    out = capsys.readouterr().out
    assert "trials completed: 5" in out and "/x: uniform(-50, 100)" in out
    _run("insert", "-n", "demo", str(script), "-x=1.5")
    _run("status", "-a")
    out = capsys.readouterr().out
    assert out.count("completed") >= 5 and " new" in out
    _run("init_only", "-n", "demo", "--branch", "demo2", str(script), "-x~uniform(-10, 10)")
    capsys.readouterr()
    _run("list")
    out = capsys.readouterr().out
    assert "demo-v1" in out and "demo2-v1" in out


def test_broken_trials_stop_worker(env, capsys):
    _, broken = env
    _run("hunt", "-n", "broken", "--max-trials", "10", str(broken), "-x~uniform(-5, 5)")
    capsys.readouterr()
    _run("status", "-n", "broken")
    out = capsys.readouterr().out
    assert "broken" in out            # max_broken (3) stops the worker before max_trials
