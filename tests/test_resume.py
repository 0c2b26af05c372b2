"""Resuming a device sweep from the database (SURVEY.md §5 "Checkpoint / resume"; reference:
completed trials replayed through ``observe``, src/orion/core/worker/producer.py:103-132, and
interrupted/lost trials re-reserved, src/orion/storage/legacy.py:206-273).

* a 2-rank (gloo) ASHA sweep stopped mid-run and restarted from its storage, device-state
  sidecars and saved algorithm state ends with the same completed trials (same ids, same
  objectives) and the same ASHA rungs as the same sweep run without interruption;
* a crashed sweep (no close: trials left ``reserved``) is resumed: its lost trials are
  re-reserved and finished, none is left behind;
* promotions of a stopped run resume from the sidecar of the lower-rung trial.
"""
import datetime
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.models.data import TeacherClassification
from metaopt_amd.models.mlp import MLPSweepTask
from metaopt_amd.ops.population import PopulationMLP
from metaopt_amd.storage.database import EphemeralDB, PickledDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.worker.population_sweep import PopulationSweep

PRIORS = {"/lr": "loguniform(1e-3, 0.3)", "/width": "loguniform(64, 128, discrete=True)",
          "/dropout": "uniform(0, 0.5)", "/steps": "fidelity(16, 64, 2)"}
ALGO = {"asha": {"seed": 5, "repetitions": float("inf")}}
MAX_TRIALS = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data():
    return TeacherClassification(n_train=512, n_val=128, batch_size=128, seed=11)


def _make(storage, data, comm=None, cap=4, max_trials=MAX_TRIALS, **kw):
    exp = None
    if comm is None or comm.is_root:
        exp = build_experiment("resume-sweep", priors=PRIORS, algorithms=ALGO,
                               max_trials=max_trials, storage=storage)
    pop = PopulationMLP(cap, max_width=128, eval_batch=128, device="cpu")
    return exp, PopulationSweep(pop, MLPSweepTask(priors=PRIORS, max_width=128), data,
                                comm=comm, experiment=exp, sync_every=16,
                                ckpt_capacity=64, **kw)


def _phase_worker(rank, world, port, db_path, ckpt_dir, max_steps, resume, q, cap=4,
                  max_trials=MAX_TRIALS, stagger=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)    # same BLAS reduction order whatever the world size
    from metaopt_amd.parallel.comm import init_from_env, shutdown
    comm = init_from_env(backend="gloo")
    storage = DocumentStorage(PickledDB(host=db_path)) if comm.is_root else None
    _, sweep = _make(storage, _data(), comm=comm, cap=cap, resume=resume,
                     restore_algorithm=resume, ckpt_dir=ckpt_dir, max_trials=max_trials,
                     stagger=stagger)
    sweep.run(max_steps)
    sweep.close()
    q.put((rank, sweep.done, sweep.n_resumed, sweep.n_resume_missing))
    shutdown()


def _run_phase(db_path, ckpt_dir, max_steps, resume, world=2, cap=4, max_trials=MAX_TRIALS,
               stagger=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_phase_worker,
                         args=(r, world, port, db_path, ckpt_dir, max_steps, resume, q, cap,
                               max_trials, stagger))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _outcome(db_path, max_trials=MAX_TRIALS, fidelities=None):
    storage = DocumentStorage(PickledDB(host=db_path))
    exp = build_experiment("resume-sweep", priors=PRIORS, algorithms=ALGO,
                           max_trials=max_trials, storage=storage)
    trials = storage.fetch_trials(exp)
    done = {t.id: t.objective.value for t in trials if t.status == "completed"}
    stati = sorted(t.status for t in trials)
    if fidelities is not None:
        fidelities.update(t.params_dict["/steps"] for t in trials if t.status == "completed")
    rungs = storage.get_algorithm_state(exp)["algorithm"]["rungs"]
    completed_rungs = [[(b, sorted((k, round(v[0], 12)) for k, v in r.items()
                                   if v[0] is not None)) for b, r in br] for br in rungs]
    return done, stati, completed_rungs


def test_two_rank_sweep_stopped_and_resumed_equals_uninterrupted(tmp_path):
    ref_db = str(tmp_path / "ref.pkl")
    res = _run_phase(ref_db, None, 100000, resume=False)
    assert all(r[1] for r in res)                       # ran to completion
    ref_done, ref_stati, ref_rungs = _outcome(ref_db)
    assert len(ref_done) == MAX_TRIALS

    db = str(tmp_path / "stopped.pkl")
    ckpt = str(tmp_path / "sidecars")
    _run_phase(db, ckpt, 4 * 16 + 3, resume=False)     # stopped mid-interval 5
    mid_done, mid_stati, _ = _outcome(db)
    assert 0 < len(mid_done) < MAX_TRIALS
    assert "reserved" not in mid_stati and "interrupted" in mid_stati
    res = _run_phase(db, ckpt, 100000, resume=True)
    assert all(r[1] for r in res)
    assert sum(r[2] for r in res) > 0 and sum(r[3] for r in res) == 0   # resumed from sidecars
    done, stati, rungs = _outcome(db)
    assert "reserved" not in stati
    assert set(done) == set(ref_done)
    for tid, obj in ref_done.items():
        assert done[tid] == pytest.approx(obj, rel=1e-6, abs=1e-9), tid
    assert rungs == ref_rungs


def test_crashed_sweep_requeues_lost_trials():
    data = _data()
    storage = DocumentStorage(EphemeralDB())
    exp, sweep = _make(storage, data, pipelined=False)
    sweep.run(3 * 16)
    sweep.flush()                     # a crash: no close(), in-flight trials stay reserved
    lost = [t for t in storage.fetch_trials(exp) if t.status == "reserved"]
    assert lost
    # their heartbeats expire (the reference's lost-trial rule)
    old = datetime.datetime.utcnow() - datetime.timedelta(hours=1)
    for t in lost:
        storage.update_trial_doc(t.id, {"heartbeat": old})
    n_done_before = sum(t.status == "completed" for t in storage.fetch_trials(exp))
    exp2, sweep2 = _make(storage, data, resume=True, pipelined=False)
    assert sweep2._prior_done >= n_done_before and len(sweep2._requeue) == len(lost)
    sweep2.run(100000)
    sweep2.close()
    trials = storage.fetch_trials(exp2)
    assert not [t for t in trials if t.status in ("reserved", "new", "interrupted")]
    finished = {t.id for t in trials if t.status in ("completed", "broken")}
    assert {t.id for t in lost} <= finished
    assert sum(t.status == "completed" for t in trials) >= MAX_TRIALS - sweep2.broken


def test_promotion_resumes_from_sidecar(tmp_path):
    data = _data()
    storage = DocumentStorage(EphemeralDB())
    ckpt = str(tmp_path / "sc")
    exp, sweep = _make(storage, data, ckpt_dir=ckpt)
    sweep.run(2 * 16)
    sweep.close()
    with_state = [t for t in storage.fetch_trials(exp) if t.working_dir]
    assert with_state and all(os.path.exists(os.path.join(t.working_dir, "device_state.pt"))
                              for t in with_state)
    st = torch.load(os.path.join(with_state[0].working_dir, "device_state.pt"),
                    weights_only=True)
    assert {"config", "t", "p32", "m32"} <= set(st)
    exp2, sweep2 = _make(storage, data, resume=True, restore_algorithm=True, ckpt_dir=ckpt)
    assert sweep2._sidecar_paths
    sweep2.run(100000)
    sweep2.close()
    assert sweep2.n_resumed > 0 and sweep2.n_resume_missing == 0
    assert math.isfinite(sweep2.best[0])


def test_sweep_cli_resume(tmp_path, capsys):
    """``mopt sweep --ckpt-dir D`` stopped by ``--steps``, then ``--resume``: the experiment is
    finished without losing or duplicating trials."""
    import json
    from metaopt_amd.cli import main
    from metaopt_amd.storage.protocol import get_storage
    name = "cli-resume-logreg"
    common = ["--debug", "sweep", "-n", name, "--task", "logreg", "--population", "4",
              "--max-trials", "40", "--sync-every", "16", "--ckpt-dir", str(tmp_path)]
    assert main(common + ["--steps", "300"]) == 0
    first = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert 0 < first["completed"] < 40
    assert main(common + ["--steps", "100000", "--resume"]) == 0
    second = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    storage = get_storage()
    exp = storage.fetch_experiments({"name": name})[0]
    trials = storage.fetch_trials(uid=exp["_id"])
    stati = [t.status for t in trials]
    assert "reserved" not in stati and "interrupted" not in stati and "new" not in stati
    assert stati.count("completed") + stati.count("broken") >= 40
    assert len({t.id for t in trials}) == len(trials)
    assert second["completed"] > 0


def test_two_rank_sweep_equals_one_rank_with_the_same_slots(tmp_path):
    """The trial-parallel engine is placement-invariant: 2 ranks x 4 slots (gloo) and 1 rank x
    8 slots finish the same trials with the same objectives and build the same ASHA rungs."""
    one = str(tmp_path / "one.pkl")
    two = str(tmp_path / "two.pkl")
    assert all(r[1] for r in _run_phase(one, None, 100000, resume=False, world=1, cap=8))
    assert all(r[1] for r in _run_phase(two, None, 100000, resume=False, world=2, cap=4))
    done1, _, rungs1 = _outcome(one)
    done2, _, rungs2 = _outcome(two)
    assert len(done1) == MAX_TRIALS and set(done1) == set(done2)
    for tid, obj in done1.items():
        assert done2[tid] == pytest.approx(obj, rel=1e-6, abs=1e-9), tid
    assert rungs1 == rungs2


def test_staggered_two_rank_sweep_equals_one_rank(tmp_path):
    """The staggered start (first fill spread over 3 syncs) is decided on rank 0 alone and
    broadcast like any placement: 2 ranks x 4 slots and 1 rank x 8 slots, both staggered, finish
    the same trials with the same objectives and ASHA rungs."""
    one = str(tmp_path / "one.pkl")
    two = str(tmp_path / "two.pkl")
    assert all(r[1] for r in _run_phase(one, None, 100000, resume=False, world=1, cap=8,
                                        stagger=3))
    assert all(r[1] for r in _run_phase(two, None, 100000, resume=False, world=2, cap=4,
                                        stagger=3))
    done1, _, rungs1 = _outcome(one)
    done2, _, rungs2 = _outcome(two)
    assert len(done1) == MAX_TRIALS and set(done1) == set(done2)
    for tid, obj in done1.items():
        assert done2[tid] == pytest.approx(obj, rel=1e-6, abs=1e-9), tid
    assert rungs1 == rungs2


def test_eight_rank_sweep_equals_one_rank_with_the_same_slots(tmp_path):
    """The 8-rank control path (placement over 8 ranks, C1/C5 at W=8, C4 copies between many
    rank pairs, the writer child under 8 ranks' completions): 8 gloo ranks x 4 slots finish
    the same trials with the same objectives and ASHA rungs as 1 rank x 32 slots."""
    import collections
    n = 160
    one = str(tmp_path / "one.pkl")
    eight = str(tmp_path / "eight.pkl")
    assert all(r[1] for r in _run_phase(one, None, 100000, resume=False, world=1, cap=32,
                                        max_trials=n))
    out = _run_phase(eight, None, 100000, resume=False, world=8, cap=4, max_trials=n)
    assert len(out) == 8 and all(r[1] for r in out)
    fid = collections.Counter()
    done1, _, rungs1 = _outcome(one, n)
    done8, stati8, rungs8 = _outcome(eight, n, fid)
    assert len(done1) == n and set(done1) == set(done8)
    for tid, obj in done1.items():
        assert done8[tid] == pytest.approx(obj, rel=1e-6, abs=1e-9), tid
    assert rungs1 == rungs8
    assert "reserved" not in stati8
    # every ASHA rung was reached: promotions resumed from checkpoints (in place or over C4,
    # spread over the 8 ranks), none lost its checkpoint on the way
    assert fid[32] > 0 and fid[64] > 0
    assert sum(r[2] for r in out) > 0 and sum(r[3] for r in out) == 0
    assert sum(r[2] > 0 for r in out) >= 4


def test_failed_sweep_close_releases_trials_without_collectives():
    """close(failed=True) after an exception on one rank: no drain/spill collectives, the
    in-flight trials are released (interrupted) and the watchdog stops."""
    data = _data()
    storage = DocumentStorage(EphemeralDB())
    exp, sweep = _make(storage, data)
    sweep.run(2 * 16)

    def boom(*a, **k):
        raise AssertionError("a collective ran during failed close")
    sweep.drain = sweep.spill = boom
    in_flight = [doc[0] for doc in sweep.trials.values()]
    assert in_flight
    sweep.close(failed=True)
    by_id = {t.id: t.status for t in storage.fetch_trials(exp)}
    assert all(by_id[tid] == "interrupted" for tid in in_flight)
    assert "reserved" not in by_id.values()
