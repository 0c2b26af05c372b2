"""End-to-end functional suites against the reference's own functional tests, run through this
framework's CLI with real worker processes, user-script subprocesses and a shared PickledDB:

* two ``hunt`` workers on one experiment (reference tests/functional/demo/test_demo.py:149-190):
  one experiment, 100-101 completed trials, fewer than 5 left ``new``;
* 30 random-search trials finish within the reference's CI bound of 10 s (test_demo.py:483-491);
* random search and ASHA (with a fidelity) reach the noisy quadratic's optimum 23.4 within 1e-5
  in 100 trials, ASHA's best at full fidelity, and ASHA refuses a space without a fidelity
  (reference tests/functional/algos/test_algos.py:20-116);
* the branching chain of the reference's tests/functional/branching/test_branching.py:14-400:
  adding, changing, renaming and removing dimensions across branches, each child seeing its
  ancestors' and descendants' trials through the EVC adapters.
"""
import os
import shutil
import subprocess
import sys
import time
from collections import Counter

import pytest
import yaml

from metaopt_amd import cli
from metaopt_amd.io.experiment_builder import ExperimentBuilder
from metaopt_amd.storage import protocol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOX = os.path.join(ROOT, "tests", "boxes", "quadratic.py")


@pytest.fixture
def db_env(tmp_path, monkeypatch):
    box = tmp_path / "black_box.py"
    shutil.copy(BOX, box)
    box.chmod(0o755)
    db = tmp_path / "db.pkl"
    monkeypatch.setenv("MOPT_DB_TYPE", "pickleddb")
    monkeypatch.setenv("MOPT_DB_ADDRESS", str(db))
    monkeypatch.setenv("PYTHONPATH", ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    monkeypatch.chdir(tmp_path)
    for attr in ("_STORAGE", "_storage", "_instance"):
        if hasattr(protocol, attr):
            monkeypatch.setattr(protocol, attr, None)
    return tmp_path


def _hunt_process(*args):
    return subprocess.Popen([sys.executable, "-m", "metaopt_amd", "hunt", *args],
                            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)


def _trials(name):
    if not protocol.storage_is_set():
        protocol.setup_storage({"database": {"type": "pickleddb",
                                             "host": os.environ["MOPT_DB_ADDRESS"]}})
    st = protocol.get_storage()
    exps = st.fetch_experiments({"name": name})
    assert len(exps) == 1
    return exps[0], st.fetch_trials(uid=exps[0]["_id"])


def test_two_concurrent_workers(db_env):
    procs = [_hunt_process("-n", "two_workers_demo", "--max-trials", "100", "--pool-size", "2",
                           "./black_box.py", "-x~norm(34, 3)") for _ in range(2)]
    for p in procs:
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, err.decode()[-2000:]
    exp, trials = _trials("two_workers_demo")
    assert exp["max_trials"] == 100 and exp["pool_size"] == 2
    assert exp["metadata"]["user_args"] == ["-x~norm(34, 3)"]
    assert os.path.isabs(exp["metadata"]["user_script"])
    status = Counter(t.status for t in trials)
    assert 100 <= status["completed"] <= 101, status
    assert status["new"] < 5, status
    assert len({t.id for t in trials}) == len(trials)          # no trial registered twice
    assert trials[-1].params[0].name == "/x" and trials[-1].params[0].type == "real"


@pytest.mark.xdist_group("timing")   # `-n N --dist loadgroup`: never beside other timing tests
def test_thirty_trials_within_ten_seconds(db_env):
    """The reference's CI bound (10 s for 30 trials on an idle VM).  The bound scales with how
    busy the machine was during the run, so a parallel test session that oversubscribes the CPUs
    does not fail a test that measures wall time: by the 1-minute load average (lags a session
    that just started) and by the mean CPU utilisation over the run itself (psutil; the hunt
    keeps about one CPU busy, so above half the CPUs busy the others competed with it).  The
    hunt's own process tree's CPU time is subtracted first (os.times() of the waited children),
    so only competing load loosens the bound."""
    psutil = pytest.importorskip("psutil")
    load0 = os.getloadavg()[0]
    ncpu = os.cpu_count() or 1
    psutil.cpu_percent(interval=None)          # starts the utilisation window
    c0 = os.times()
    t0 = time.perf_counter()
    p = _hunt_process("-n", "quick", "--max-trials", "30", "./black_box.py",
                      "-x~uniform(-50, 50)")
    _, err = p.communicate(timeout=120)
    elapsed = time.perf_counter() - t0
    util = psutil.cpu_percent(interval=None) / 100.0
    c1 = os.times()
    own = (c1.children_user - c0.children_user) + (c1.children_system - c0.children_system)
    other = max(0.0, util - own / (ncpu * max(elapsed, 1e-6)))   # competing CPU share
    assert p.returncode == 0, err.decode()[-2000:]
    busy = max(load0, os.getloadavg()[0]) / ncpu
    scale = max(1.0, busy, 2.0 * other)
    assert elapsed < 10.0 * scale, (elapsed, busy, util, own)
    _, trials = _trials("quick")
    assert Counter(t.status for t in trials)["completed"] == 30


def _config(tmp_path, name, algorithms, **extra):
    cfg = {"name": name, "pool_size": 1, "max_trials": 100, "algorithms": algorithms, **extra}
    path = tmp_path / f"{name}.yaml"
    path.write_text(yaml.safe_dump(cfg))
    return str(path), cfg


@pytest.mark.parametrize("algo", ["random", "asha"])
def test_algorithms_reach_the_optimum(db_env, algo):
    if algo == "random":
        path, cfg = _config(db_env, "demo_random", {"random": {"seed": 1}})
        space = ["-x~uniform(-50, 50)"]
    else:
        path, cfg = _config(db_env, "demo_asha",
                            {"asha": {"seed": 1, "num_rungs": 4, "num_brackets": 1}},
                            producer={"strategy": "StubParallelStrategy"})
        space = ["-x~uniform(-50, 50)", "--fidelity~fidelity(1,10,4)"]
    assert cli.main(["hunt", "--config", path, "./black_box.py", *space, "--noise"]) == 0
    exp, trials = _trials(cfg["name"])
    assert exp["pool_size"] == 1 and exp["max_trials"] == 100
    (name, given), = cfg["algorithms"].items()
    stored = exp["algorithms"][name]                # the full configuration, defaults included
    assert {k: stored[k] for k in given} == given
    assert exp["metadata"]["user_args"] == space + ["--noise"]
    assert len(trials) <= 100 and trials[-1].status == "completed"
    best = min((t for t in trials if t.status == "completed"), key=lambda t: t.objective.value)
    assert best.objective.name == "example_objective"
    assert abs(best.objective.value - 23.4) < 1e-5
    params = {p.name: p for p in best.params}
    assert params["/x"].type == "real"
    if algo == "asha":
        assert params["/fidelity"].type == "fidelity" and params["/fidelity"].value == 10


def test_asha_requires_a_fidelity(db_env):
    path, _ = _config(db_env, "no_fidelity", {"asha": {"seed": 1}})
    with pytest.raises(Exception, match="fidelity"):
        cli.main(["hunt", "--config", path, "./black_box.py", "-x~uniform(-50, 50)"])


# ---------------------------------------------------------------------------------- branching
def _pairs(trials):
    return tuple(tuple((p.name, p.value) for p in sorted(t.params, key=lambda p: p.name))
                 for t in trials)


def _view(name):
    return ExperimentBuilder().build_view_from({"name": name})


def _branch(parent, child, *space):
    argv = ["init_only", "-n", parent]
    if child:
        argv += ["--branch", child]
    assert cli.main(argv + ["./black_box.py", *space]) is not None


def _insert(name, *values):
    assert cli.main(["insert", "-n", name, "./black_box.py", *values]) is not None


@pytest.fixture
def chain(db_env):
    """The reference's branching fixtures, full tree (init_entire)."""
    _branch("full_x", None, "-x~uniform(-10,10)")
    _insert("full_x", "-x=0")
    _branch("full_x", "full_x_full_y", "-x~uniform(-10,10)",
            "-y~+uniform(-10,10,default_value=1)")
    for x, y in ((1, 1), (-1, 1), (1, -1), (-1, -1)):
        _insert("full_x_full_y", f"-x={x}", f"-y={y}")
    _branch("full_x_full_y", "half_x_full_y", "-x~+uniform(0,10)",
            "-y~uniform(-10,10,default_value=1)")
    for x, y in ((2, 2), (2, -2)):
        _insert("half_x_full_y", f"-x={x}", f"-y={y}")
    _branch("full_x_full_y", "full_x_half_y", "-x~uniform(-10,10)",
            "-y~+uniform(0,10,default_value=1)")
    for x, y in ((3, 3), (-3, 3)):
        _insert("full_x_half_y", f"-x={x}", f"-y={y}")
    _branch("full_x_full_y", "full_x_rename_y_z", "-x~uniform(-10,10)", "-y~>z",
            "-z~uniform(-10,10,default_value=1)")
    for x, z in ((4, 4), (-4, 4), (4, -4), (-4, -4)):
        _insert("full_x_rename_y_z", f"-x={x}", f"-z={z}")
    _branch("full_x_half_y", "full_x_rename_half_y_half_z", "-x~uniform(-10,10)", "-y~>z",
            "-z~uniform(0,10,default_value=1)")
    for x, z in ((5, 5), (-5, 5)):
        _insert("full_x_rename_half_y_half_z", f"-x={x}", f"-z={z}")
    _branch("full_x_half_y", "full_x_rename_half_y_full_z", "-x~uniform(-10,10)", "-y~>z",
            "-z~+uniform(-10,10,default_value=1)")
    for x, z in ((6, 6), (-6, 6), (6, -6), (-6, -6)):
        _insert("full_x_rename_half_y_full_z", f"-x={x}", f"-z={z}")
    _branch("full_x_full_y", "full_x_remove_y", "-x~uniform(-10,10)", "-y~-")
    for x in (7, -7):
        _insert("full_x_remove_y", f"-x={x}")
    _branch("full_x_rename_y_z", "full_x_remove_z", "-x~uniform(-10,10)", "-z~-")
    for x in (8, -8):
        _insert("full_x_remove_z", f"-x={x}")
    _branch("full_x_rename_y_z", "full_x_remove_z_default_4", "-x~uniform(-10,10)", "-z~-4")
    for x in (9, -9):
        _insert("full_x_remove_z_default_4", f"-x={x}")
    return db_env


def _xy(*vals):
    return tuple(((("/x", x),) if y is None else (("/x", x), (name, y)))
                 for x, y, name in vals)


def test_branching_children_see_their_parents(chain):
    assert _pairs(_view("full_x").fetch_trials()) == ((("/x", 0),),)
    exp = _view("full_x_full_y")
    assert set(_pairs(exp.fetch_trials())) == {(("/x", 1), ("/y", 1)), (("/x", -1), ("/y", 1)),
                                               (("/x", 1), ("/y", -1)), (("/x", -1), ("/y", -1))}
    # half_x: the parent's trials outside x in [0, 10] are filtered out by the prior change
    assert set(_pairs(_view("half_x_full_y").fetch_trials(with_evc_tree=True))) >= {
        (("/x", 0), ("/y", 1)), (("/x", 1), ("/y", 1)), (("/x", 1), ("/y", -1)),
        (("/x", 2), ("/y", 2)), (("/x", 2), ("/y", -2))}
    assert (("/x", -1), ("/y", 1)) not in _pairs(
        _view("half_x_full_y").fetch_trials(with_evc_tree=True))
    renamed = set(_pairs(_view("full_x_rename_y_z").fetch_trials(with_evc_tree=True)))
    assert renamed == {(("/x", 0), ("/z", 1)), (("/x", 1), ("/z", 1)), (("/x", -1), ("/z", 1)),
                       (("/x", 1), ("/z", -1)), (("/x", -1), ("/z", -1)),
                       (("/x", 4), ("/z", 4)), (("/x", -4), ("/z", 4)),
                       (("/x", 4), ("/z", -4)), (("/x", -4), ("/z", -4)),
                       # its children: z removed (default 1 / default 4) adapted back
                       (("/x", 8), ("/z", 1)), (("/x", -8), ("/z", 1)),
                       (("/x", 9), ("/z", 4)), (("/x", -9), ("/z", 4))}
    half_z = set(_pairs(_view("full_x_rename_half_y_half_z").fetch_trials(with_evc_tree=True)))
    assert half_z == {(("/x", 0), ("/z", 1)), (("/x", 1), ("/z", 1)), (("/x", -1), ("/z", 1)),
                      (("/x", 3), ("/z", 3)), (("/x", -3), ("/z", 3)),
                      (("/x", 5), ("/z", 5)), (("/x", -5), ("/z", 5))}
    removed = set(_pairs(_view("full_x_remove_y").fetch_trials(with_evc_tree=True)))
    assert removed == {(("/x", 0),), (("/x", 1),), (("/x", -1),), (("/x", 7),), (("/x", -7),)}
    # removing z with default 4 keeps only the ancestors' trials whose z was 4
    rz4 = set(_pairs(_view("full_x_remove_z_default_4").fetch_trials(with_evc_tree=True)))
    assert rz4 == {(("/x", 4),), (("/x", -4),), (("/x", 9),), (("/x", -9),)}


def test_branching_parent_sees_every_descendant(chain):
    exp = _view("full_x_full_y")
    pairs = set(_pairs(exp.fetch_trials(with_evc_tree=True)))
    want = {(("/x", 0), ("/y", 1))}
    want |= {(("/x", x), ("/y", y)) for x, y in ((1, 1), (-1, 1), (1, -1), (-1, -1), (2, 2),
                                                  (2, -2), (3, 3), (-3, 3), (4, 4), (-4, 4),
                                                  (4, -4), (-4, -4), (5, 5), (-5, 5), (6, 6),
                                                  (-6, 6), (7, 1), (-7, 1), (8, 1), (-8, 1),
                                                  (9, 4), (-9, 4))}
    assert pairs == want
    assert len(exp.fetch_trials(with_evc_tree=True)) == 23 and len(exp.fetch_trials()) == 4


def test_branched_experiment_runs_without_branching_again(chain):
    assert cli.main(["hunt", "--max-trials", "20", "--pool-size", "1", "-n", "full_x_full_y",
                     "./black_box.py", "-x~uniform(-10,10)",
                     "-y~uniform(-10,10,default_value=1)"]) == 0
    exp = _view("full_x_full_y")
    assert len(exp.fetch_trials()) == 20
    assert len(exp.fetch_trials(with_evc_tree=True)) == 39
    assert len(protocol.get_storage().fetch_experiments({"name": "full_x_full_y"})) == 1
