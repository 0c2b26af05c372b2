"""Experiment life cycle beyond registration races: lost-trial recovery and its race, reserve
order and exclusivity, done/broken accounting, stats, and the read-only view (behaviour of
the reference's tests/unittests/core/worker/test_experiment.py:716-833 -- fix_lost_trials and
its race -- plus its stats and view tests; written fresh against this package's API)."""
import datetime
import threading

import pytest

from metaopt_amd.core.experiment import ExperimentView
from metaopt_amd.core.trial import Trial
from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.storage.database import EphemeralDB, PickledDB
from metaopt_amd.storage.protocol import DocumentStorage, FailedUpdate


def _exp(storage=None, name="life", max_trials=10):
    return build_experiment(name, priors={"/x": "uniform(0, 1)"}, max_trials=max_trials,
                            storage=storage or DocumentStorage(EphemeralDB()))


def _add(exp, x, status="new", **fields):
    t = Trial(experiment=exp.id, params=[dict(name="/x", type="real", value=x)])
    exp.register_trial(t)
    if status != "new" or fields:
        exp.storage.update_trial_doc(t.id, dict({"status": status}, **fields))
    return t


def _age(exp, trial, seconds):
    stale = datetime.datetime.utcnow() - datetime.timedelta(seconds=seconds)
    exp.storage.update_trial_doc(trial.id, {"heartbeat": stale})


def _status(exp, trial):
    return exp.get_trial(trial).status


# ------------------------------------------------------------------------ lost trials
class TestLostTrials:
    def test_stale_reserved_trial_becomes_interrupted(self):
        exp = _exp()
        t = _add(exp, 0.1, "reserved", heartbeat=datetime.datetime.utcnow())
        _age(exp, t, 10_000)
        exp.fix_lost_trials()
        assert _status(exp, t) == "interrupted"

    def test_fresh_heartbeat_is_not_lost(self):
        exp = _exp()
        t = _add(exp, 0.1, "reserved", heartbeat=datetime.datetime.utcnow())
        exp.fix_lost_trials()
        assert _status(exp, t) == "reserved"

    def test_only_reserved_trials_can_be_lost(self):
        exp = _exp()
        done = _add(exp, 0.2, "completed", heartbeat=datetime.datetime.utcnow())
        _age(exp, done, 10_000)
        exp.fix_lost_trials()
        assert _status(exp, done) == "completed"

    def test_lost_trial_is_reserved_again(self):
        exp = _exp()
        t = _add(exp, 0.3, "reserved", heartbeat=datetime.datetime.utcnow())
        _age(exp, t, 10_000)
        again = exp.reserve_trial()         # reserve runs the lost-trial sweep first
        assert again is not None and again.id == t.id and again.status == "reserved"

    def test_race_on_a_lost_trial_is_won_once(self):
        """Two workers see the same lost trial: the compare-and-swap lets exactly one of them
        mark it, the other's update fails and is ignored by fix_lost_trials."""
        exp = _exp()
        t = _add(exp, 0.4, "reserved", heartbeat=datetime.datetime.utcnow())
        _age(exp, t, 10_000)
        (seen_a,) = exp.storage.fetch_lost_trials(exp)
        (seen_b,) = exp.storage.fetch_lost_trials(exp)
        exp.storage.set_trial_status(seen_a, status="interrupted")
        with pytest.raises(FailedUpdate):
            exp.storage.set_trial_status(seen_b, status="interrupted")
        exp.fix_lost_trials()                # nothing lost any more: a no-op
        assert _status(exp, t) == "interrupted"

    def test_fix_lost_trials_tolerates_a_concurrent_recovery(self, monkeypatch):
        """The trial is recovered by someone else between the fetch and the update."""
        exp = _exp()
        t = _add(exp, 0.5, "reserved", heartbeat=datetime.datetime.utcnow())
        _age(exp, t, 10_000)
        real = exp.storage.fetch_lost_trials

        def fetch_then_race(experiment):
            lost = real(experiment)
            exp.storage.update_trial_doc(t.id, {"status": "interrupted"})
            return lost
        monkeypatch.setattr(exp.storage, "fetch_lost_trials", fetch_then_race)
        exp.fix_lost_trials()                # FailedUpdate swallowed
        assert _status(exp, t) == "interrupted"

    def test_threads_recovering_lost_trials(self, tmp_path):
        """Eight threads on one PickledDB file sweep the same lost trials at once: every trial
        ends interrupted and reservable exactly once."""
        st = DocumentStorage(PickledDB(host=str(tmp_path / "db.pkl")))
        exp = _exp(st, name="lost-threads")
        lost = [_add(exp, 0.05 * i, "reserved", heartbeat=datetime.datetime.utcnow())
                for i in range(6)]
        for t in lost:
            _age(exp, t, 10_000)
        errors = []

        def work():
            try:
                exp.fix_lost_trials()
            except Exception as exc:  # pragma: no cover - the failure being tested for
                errors.append(exc)
        threads = [threading.Thread(target=work) for _ in range(8)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        assert not errors
        assert all(_status(exp, t) == "interrupted" for t in lost)
        got = [exp.reserve_trial() for _ in range(7)]
        assert sorted(g.id for g in got if g) == sorted(t.id for t in lost)


# ------------------------------------------------------------------------ reservation
class TestReservation:
    def test_reservation_sets_timestamps(self):
        exp = _exp()
        _add(exp, 0.1)
        t = exp.reserve_trial()
        assert t.status == "reserved" and t.start_time is not None and t.heartbeat is not None

    def test_interrupted_and_suspended_are_reservable(self):
        exp = _exp()
        for s in ("interrupted", "suspended"):
            _add(exp, 0.2 if s == "interrupted" else 0.3, s)
        got = {exp.reserve_trial().id for _ in range(2)}
        assert len(got) == 2 and exp.reserve_trial() is None

    def test_broken_and_completed_are_not_reservable(self):
        exp = _exp()
        _add(exp, 0.1, "broken")
        _add(exp, 0.2, "completed")
        assert exp.reserve_trial() is None

    def test_score_handle_is_deprecated_but_accepted(self, caplog):
        exp = _exp()
        _add(exp, 0.1)
        assert exp.reserve_trial(score_handle=lambda t: 0) is not None
        assert "deprecated" in caplog.text


# ------------------------------------------------------------------------ done / broken / stats
class TestAccounting:
    def test_is_done_by_max_trials(self):
        exp = _exp(max_trials=2)
        assert not exp.is_done
        for x in (0.1, 0.2):
            t = _add(exp, x)
            t = exp.reserve_trial()
            t.results = [dict(name="o", type="objective", value=x)]
            exp.update_completed_trial(t)
        assert exp.is_done

    def test_is_broken_by_max_broken(self):
        exp = _exp()
        for i in range(3):
            _add(exp, 0.1 * (i + 1), "broken")
        assert exp.is_broken

    def test_stats_of_completed_trials(self):
        exp = _exp()
        assert exp.stats == {}
        for x in (0.7, 0.2, 0.5):
            _add(exp, x)
            t = exp.reserve_trial()
            t.results = [dict(name="o", type="objective", value=x * 10)]
            exp.update_completed_trial(t)
        s = exp.stats
        assert s["trials_completed"] == 3 and s["best_evaluation"] == pytest.approx(2.0)
        best = exp.get_trial(uid=s["best_trials_id"])
        assert best.params[0].value == pytest.approx(0.2)
        assert s["finish_time"] >= s["start_time"] and s["duration"] >= datetime.timedelta(0)

    def test_stats_ignore_unfinished(self):
        exp = _exp()
        _add(exp, 0.1, "reserved", heartbeat=datetime.datetime.utcnow())
        _add(exp, 0.2, "broken")
        assert exp.stats == {}

    def test_register_trials_skips_duplicates(self):
        exp = _exp()
        a = Trial(params=[dict(name="/x", type="real", value=0.5)])
        b = Trial(params=[dict(name="/x", type="real", value=0.5)])
        c = Trial(params=[dict(name="/x", type="real", value=0.6)])
        done = exp.register_trials([a, b, c])
        assert [t.params[0].value for t in done] == [0.5, 0.6]
        assert len(exp.fetch_trials()) == 2


# ------------------------------------------------------------------------ read-only view
class TestView:
    def test_view_reads_the_same_trials(self):
        st = DocumentStorage(EphemeralDB())
        exp = _exp(st, name="viewed")
        _add(exp, 0.1)
        view = ExperimentView("viewed", storage=st)
        assert [t.id for t in view.fetch_trials()] == [t.id for t in exp.fetch_trials()]
        assert view.id == exp.id and view.space is not None
        assert "ExperimentView(name=viewed" in repr(view)

    def test_view_cannot_write(self):
        st = DocumentStorage(EphemeralDB())
        _exp(st, name="viewed2")
        view = ExperimentView("viewed2", storage=st)
        for attr in ("reserve_trial", "register_trial", "update_completed_trial",
                     "set_trial_status", "fix_lost_trials", "configure"):
            with pytest.raises(AttributeError, match="view-only"):
                getattr(view, attr)

    def test_view_storage_is_read_only(self):
        st = DocumentStorage(EphemeralDB())
        _exp(st, name="viewed3")
        view = ExperimentView("viewed3", storage=st)
        with pytest.raises(AttributeError):
            view.storage.register_trial(Trial(params=[dict(name="/x", type="real",
                                                           value=0.1)]))

    def test_view_of_unknown_experiment(self):
        with pytest.raises(ValueError, match="No experiment"):
            ExperimentView("nobody-here", storage=DocumentStorage(EphemeralDB()))
