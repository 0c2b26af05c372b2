"""JSONL event log and rank-failure watchdog (observability, failure detection)."""
import math
import time

import pytest

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.models.mlp import MLPSweepTask
from metaopt_amd.ops.population import PopulationMLP
from metaopt_amd.parallel.watchdog import Watchdog
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.utils.events import EventLog, read_events
from metaopt_amd.worker.population_sweep import PopulationSweep

PRIORS = {"/lr": "loguniform(1e-3, 1.0)", "/width": "loguniform(64, 128, discrete=True)",
          "/dropout": "uniform(0, 0.5)", "/steps": "fidelity(16, 64, 2)"}


@pytest.fixture(scope="module")
def data():
    return TeacherClassification(n_train=512, n_val=128, batch_size=128, seed=3)


def _sweep(data, name, max_trials, **kw):
    storage = DocumentStorage(EphemeralDB())
    exp = build_experiment(name, priors=PRIORS,
                           algorithms={"asha": {"seed": 2, "repetitions": float("inf")}},
                           max_trials=max_trials, storage=storage)
    pop = PopulationMLP(4, max_width=128, eval_batch=128, device="cpu")
    sweep = PopulationSweep(pop, MLPSweepTask(priors=PRIORS, max_width=128), data,
                            experiment=exp, sync_every=16, **kw)
    return exp, sweep


def test_event_log_roundtrip_and_json_safety(tmp_path):
    import numpy as np
    path = tmp_path / "ev" / "log.jsonl"
    with EventLog(str(path), flush_every=2) as ev:
        ev.emit("sync", step=np.int64(3), best=float("inf"), ms={"a": np.float32(1.5)})
        ev.emit("trial", id="x", objective=math.nan)
    recs = list(read_events(str(path)))
    assert [r["event"] for r in recs] == ["sync", "trial"]
    assert recs[0]["step"] == 3 and recs[0]["best"] is None and recs[0]["ms"]["a"] == 1.5
    assert recs[1]["objective"] is None and recs[1]["rank"] == 0
    assert [r["id"] for r in read_events(str(path), "trial")] == ["x"]


def test_sweep_writes_event_log(tmp_path, data):
    path = str(tmp_path / "sweep.jsonl")
    ev = EventLog(path)
    exp, sweep = _sweep(data, "ev-sweep", 12, events=ev, trial_events=True)
    summary = sweep.run(1000)
    sweep.close()
    ev.close()
    kinds = [r["event"] for r in read_events(path)]
    assert kinds[0] == "sweep_start" and kinds[-1] == "sweep_end"
    syncs = list(read_events(path, "sync"))
    assert len(syncs) == sweep.n_syncs
    assert syncs[-1]["completed"] == summary["completed"] == 12
    assert set(syncs[0]["ms"]) >= {"decide", "apply", "c1_allgather", "c5_broadcast"}
    trials = list(read_events(path, "trial"))
    assert len(trials) == 12 and all(t["status"] == "completed" for t in trials)
    ids = {t.id for t in exp.fetch_trials()}
    assert {t["id"] for t in trials} == ids
    end = list(read_events(path, "sweep_end"))[0]
    assert end["completed"] == 12 and end["best_val_loss"] == pytest.approx(
        summary["best_val_loss"])


def test_watchdog_fires_once_on_stall_and_not_while_beating():
    fired = []
    wd = Watchdog(0.3, exit_code=None, poll_s=0.02)
    wd.on_stall.append(lambda s, ph: fired.append((s, ph)))
    with wd:
        for _ in range(10):           # regular beats: no stall
            time.sleep(0.05)
            wd.beat("sync")
        assert not fired
        time.sleep(0.6)               # silence: fires exactly once
    assert wd.fired and len(fired) == 1
    assert fired[0][0] >= 0.3 and fired[0][1] == "sync"
    with pytest.raises(ValueError):
        Watchdog(0)


def test_watchdog_interrupts_in_flight_trials(tmp_path, data):
    """A stall (e.g. a peer rank died inside a collective) leaves no trial ``reserved``: rank 0
    marks the in-flight ones ``interrupted`` so another worker or a re-run picks them up."""
    path = str(tmp_path / "wd.jsonl")
    ev = EventLog(path)
    wd = Watchdog(3600, exit_code=None, poll_s=0.05)
    exp, sweep = _sweep(data, "wd-sweep", 40, events=ev, watchdog=wd)
    sweep.run(20)                     # mid-sweep: members in flight
    in_flight = len(sweep.trials)
    assert in_flight > 0
    wd.timeout_s = 0.1                # simulate the stall: no more syncs arrive
    deadline = time.time() + 10
    while not wd.fired and time.time() < deadline:
        time.sleep(0.05)
    assert wd.fired
    statuses = [t.status for t in exp.fetch_trials()]
    assert statuses.count("interrupted") == in_flight
    assert "reserved" not in statuses
    assert [r["n_trials"] for r in read_events(path, "interrupted")] == [in_flight]
    assert len(list(read_events(path, "watchdog"))) == 1
    sweep.close()
    ev.close()


def test_watchdog_exits_process_cleanly():
    """Default mode: the stuck process terminates with the watchdog's exit code."""
    import subprocess
    import sys
    code = ("import time; from metaopt_amd.parallel.watchdog import Watchdog\n"
            "Watchdog(0.2, exit_code=75, poll_s=0.02).start()\n"
            "time.sleep(30)\n")
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    proc = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True,
                          text=True, timeout=60)
    assert proc.returncode == 75
    assert "no progress" in proc.stderr


def test_launch_check_reports_kernel_name():
    from metaopt_amd.ops import _lib
    _lib.check(0, "mopt_ok")
    with pytest.raises(RuntimeError, match="mopt_bad.*hipError_t 98"):
        _lib.check(98, "mopt_bad")


@pytest.mark.gpu
def test_sync_check_mode_runs_population_step(monkeypatch):
    """MOPT_SYNC_CHECK: every launch synchronises (outside graph capture) and still trains."""
    import torch
    from metaopt_amd.ops import _lib
    from metaopt_amd.ops.population import MemberConfig
    monkeypatch.setattr(_lib, "SYNC_CHECK", True)
    dev = torch.device("cuda:0")
    d = TeacherClassification(n_train=256, n_val=128, batch_size=128, seed=0, device=dev)
    pop = PopulationMLP(2, max_width=128, eval_batch=128, device=dev, backend="hip")
    for s, w in enumerate((64, 128)):
        pop.set_member(s, MemberConfig(width=w, lr=0.1, dropout=0.0, seed=s + 1))
    x, y = d.batch(0)
    pop.train_step(x, y)
    torch.cuda.synchronize()
    assert all(math.isfinite(v) for v in pop.train_loss()[:2])


def _canon(v):
    import numpy as np
    if isinstance(v, dict):
        return {str(k): _canon(x) for k, x in sorted(v.items(), key=lambda kv: str(kv[0]))}
    if isinstance(v, (list, tuple)):
        return [_canon(x) for x in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


def test_sweep_persists_and_restores_algorithm_state(data):
    """close() stores the algorithm's FULL state (ASHA rungs, not only the RNG) and the sweep's
    step counter; a re-run restores both."""
    exp, sweep = _sweep(data, "state-sweep", 12)
    sweep.run(1000)
    sweep.close()
    state = exp.storage.get_algorithm_state(exp)
    assert state is not None
    assert _canon(state["algorithm"]) == _canon(exp.algorithms.full_state())
    assert state["sweep"]["global_step"] == sweep.global_step
    rungs = state["algorithm"]["rungs"]
    assert sum(len(r) for br in rungs for _, r in br) >= 12     # the search itself is persisted
    pop = PopulationMLP(4, max_width=128, eval_batch=128, device="cpu")
    fresh = build_experiment("state-sweep-2", priors=PRIORS,
                             algorithms={"asha": {"seed": 9, "repetitions": float("inf")}},
                             max_trials=12, storage=exp.storage)
    fresh.storage.save_algorithm_state(fresh, state=state)
    assert _canon(fresh.algorithms.full_state()) != _canon(state["algorithm"])
    sweep2 = PopulationSweep(pop, MLPSweepTask(priors=PRIORS, max_width=128), data,
                             experiment=fresh, sync_every=16, restore_algorithm=True)
    restored = fresh.algorithms.full_state()
    # completed entries come back; pending ones (never reported) are dropped
    want = _canon(state["algorithm"])
    for br in want["rungs"]:
        for rung in br:
            rung[1] = {k: v for k, v in rung[1].items() if v[0] is not None}
    got = _canon(restored)
    assert got["rungs"] == want["rungs"] and got["rng_state"] == want["rng_state"]
    assert sweep2.global_step == sweep.global_step
    sweep2.close()


@pytest.mark.parametrize("task,steps", [("logreg", 288)])
def test_sweep_cli_event_log_and_watchdog_flags(tmp_path, capsys, task, steps):
    """``mopt --debug sweep ... --event-log --trial-events --watchdog`` on the CPU backend."""
    import json
    from metaopt_amd.cli import main
    path = str(tmp_path / "cli.jsonl")
    rc = main(["--debug", "sweep", "--task", task, "--population", "4", "--steps", str(steps),
               "--max-trials", "8", "--sync-every", "16", "--event-log", path,
               "--trial-events", "--watchdog", "600"])
    assert rc == 0
    summary = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    kinds = [r["event"] for r in read_events(path)]
    assert kinds[0] == "sweep_start" and kinds[-1] == "sweep_end"
    n_trials = len(list(read_events(path, "trial")))
    assert n_trials == summary["completed"] + summary["broken"] > 0
    assert "watchdog" not in kinds
