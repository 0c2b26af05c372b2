"""The Oríon compatibility surface (VERDICT r3 "What's missing" 1).

* ``tests/boxes/orion_demo_black_box.py`` is the reference's user script
  ``tests/functional/demo/black_box.py``, byte for byte (a test fixture: it still does
  ``from orion.client import report_results``).  It runs unmodified under ``hunt`` started
  through ``orion.core.cli.main``, and gradient descent finds the quadratic's optimum 23.4 within
  the reference's tolerance in at most 15 trials (reference
  ``tests/functional/demo/test_demo.py:50-90``).
* ``pyproject.toml`` declares the ``mopt`` / ``orion`` console scripts and the
  ``OptimizationAlgorithm`` / ``Storage`` entry points of the reference's ``setup.py:39-50``;
  every declared object imports and is the registered built-in.
"""
import os
import shutil

import numpy
import pytest
import yaml

import orion.core.cli
from metaopt_amd.storage import protocol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOX = os.path.join(ROOT, "tests", "boxes", "orion_demo_black_box.py")


@pytest.fixture
def demo_dir(tmp_path, monkeypatch):
    box = tmp_path / "black_box.py"
    shutil.copy(BOX, box)
    box.chmod(0o755)
    monkeypatch.setenv("MOPT_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", str(tmp_path / "db.pkl"))
    # the trial subprocess must find ``orion`` by itself (consumer.trial_env), not through us
    monkeypatch.delenv("PYTHONPATH", raising=False)
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(protocol, "_STORAGE", None)
    return tmp_path


def test_reference_black_box_runs_unmodified(demo_dir):
    with open(BOX) as f:
        assert "from orion.client import report_results" in f.read()
    cfg = {"name": "voila_voici", "pool_size": 1, "max_trials": 100,
           "algorithms": {"gradient_descent": {"learning_rate": 0.1, "dx_tolerance": 1e-7}},
           "producer": {"strategy": "NoParallelStrategy"}}
    (demo_dir / "orion_config.yaml").write_text(yaml.safe_dump(cfg))
    user_args = ["-x~uniform(-50, 50)", "--test-env",
                 "--experiment-id", "{exp.id}", "--experiment-name", "{exp.name}",
                 "--experiment-version", "{exp.version}", "--trial-id", "{trial.id}",
                 "--working-dir", "{trial.working_dir}"]
    rc = orion.core.cli.main(["hunt", "--config", "./orion_config.yaml", "./black_box.py"]
                             + user_args)
    assert rc == 0
    st = protocol.get_storage()
    exp, = st.fetch_experiments({"name": "voila_voici"})
    assert exp["metadata"]["user_args"] == user_args
    assert exp["algorithms"]["gradient_descent"]["learning_rate"] == 0.1
    trials = sorted(st.fetch_trials(uid=exp["_id"]), key=lambda t: t.submit_time)
    assert 0 < len(trials) <= 15
    last = trials[-1]
    assert last.status == "completed"
    for r in last.results:
        if r.type == "objective":
            assert r.name == "example_objective" and abs(r.value - 23.4) < 1e-6
        elif r.type == "gradient":
            g = numpy.asarray(r.value)
            assert 0.1 * numpy.sqrt(g.dot(g)) < 1e-7
    (p,) = last.params
    assert p.name == "/x" and p.type == "real" and abs(p.value - 34.56789) < 1e-5


def _pyproject():
    try:
        import tomllib
    except ImportError:          # python < 3.11
        import tomli as tomllib
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as f:
        return tomllib.load(f)


def _resolve(target):
    import importlib
    mod, attr = target.split(":")
    return getattr(importlib.import_module(mod), attr)


def test_declared_console_scripts_and_entry_points_resolve():
    proj = _pyproject()["project"]
    scripts = proj["scripts"]
    from metaopt_amd.cli import main
    assert _resolve(scripts["mopt"]) is main and _resolve(scripts["orion"]) is main
    from metaopt_amd.algo.base import ALGORITHMS
    eps = proj["entry-points"]
    # the reference declares random and asha (setup.py:43-46); every built-in is declared here
    assert {"random", "asha"} <= set(eps["OptimizationAlgorithm"])
    assert set(eps["OptimizationAlgorithm"]) == set(ALGORITHMS.names())
    for name, target in eps["OptimizationAlgorithm"].items():
        assert ALGORITHMS.get(name) is _resolve(target)
    assert _resolve(eps["Storage"]["legacy"]) is protocol.STORAGES.get("legacy")


def test_orion_plugin_surface():
    from orion.algo.base import BaseAlgorithm
    from orion.algo.space import Real, Space
    from orion.client import insert_trials, report_results  # noqa: F401
    from metaopt_amd.algo.base import BaseAlgorithm as B
    assert BaseAlgorithm is B
    space = Space()
    space.register(Real("x", "uniform", -1, 2))
    assert "x" in space
