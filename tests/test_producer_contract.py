"""Producer contract, case by case (the behaviour the reference pins in
tests/unittests/core/test_producer.py): completed trials are observed once by the algorithm and
the strategy, in-flight trials get lies seen only by the naive copy (rebuilt every update and
recorded once), broken trials get none, duplicates inside one pool and against the database are
skipped, several producers on one experiment never register a point twice, the real algorithm
inherits the naive copy's RNG state, and a finished algorithm stops production.  Written
against this package's API."""
import datetime

import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.utils.exceptions import SampleTimeout
from metaopt_amd.worker.producer import Producer


def _exp(pool_size=3, priors=None, algorithms=None, strategy=None, storage=None, name="p"):
    kw = {"strategy": strategy} if strategy else {}
    return build_experiment(name, priors=priors or {"/x": "uniform(-5, 5)"},
                            algorithms=algorithms or {"random": {"seed": 1}},
                            pool_size=pool_size, storage=storage or DocumentStorage(EphemeralDB()),
                            **kw)


def _set(exp, trial, status, value=None):
    if value is not None:
        trial.results = [Trial.Result(name="obj", type="objective", value=value)]
        trial.end_time = datetime.datetime.utcnow()
    trial.status = status
    if status == "completed":
        exp.storage.push_trial_results(trial)
    exp.storage.update_trial_doc(trial.id, {"status": status})


def test_completed_trials_are_observed_once(monkeypatch):
    exp = _exp()
    prod = Producer(exp)
    prod.produce()
    seen = []
    cls = type(prod.algorithm)
    real = cls.observe

    def observe(self, points, results, *a, **kw):     # the real algorithm's calls only
        if self is prod.algorithm:
            seen.extend(points)
        return real(self, points, results, *a, **kw)
    monkeypatch.setattr(cls, "observe", observe)
    a, b, c = exp.fetch_trials()
    _set(exp, a, "completed", 1.0)
    prod.update()
    prod.update()
    assert len(seen) == 1


def test_strategy_observes_completed():
    exp = _exp(strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    a = exp.fetch_trials()[0]
    _set(exp, a, "completed", 7.0)
    prod.update()
    assert prod.strategy.max_result == 7.0


def test_no_lies_when_everything_completed():
    exp = _exp(pool_size=2, strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    for i, t in enumerate(exp.fetch_trials()):
        _set(exp, t, "completed", float(i))
    prod.update()
    assert exp.storage.fetch_lies(exp) == []


def test_one_lie_per_in_flight_trial():
    exp = _exp(pool_size=3, strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    a, b, c = exp.fetch_trials()
    _set(exp, a, "completed", 2.0)
    _set(exp, b, "reserved")
    prod.update()
    lies = exp.storage.fetch_lies(exp)
    assert sorted(l.params[0].value for l in lies) == sorted(t.params[0].value for t in (b, c))
    assert all(l.lie.value == 2.0 for l in lies)


def test_lies_recorded_once_across_updates():
    exp = _exp(pool_size=2, strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    a, _ = exp.fetch_trials()
    _set(exp, a, "completed", 1.0)
    prod.update()
    prod.update()
    assert len(exp.storage.fetch_lies(exp)) == 1


def test_broken_trials_get_no_lie():
    exp = _exp(pool_size=2, strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    a, b = exp.fetch_trials()
    _set(exp, a, "completed", 1.0)
    _set(exp, b, "broken")
    prod.update()
    assert exp.storage.fetch_lies(exp) == []


def test_naive_copy_sees_lies_the_real_algorithm_does_not():
    exp = _exp(pool_size=3, strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    a, _, _ = exp.fetch_trials()
    _set(exp, a, "completed", 1.0)
    prod.update()
    assert len(prod.trials_history.ids) == 1 and len(prod.naive_trials_history.ids) == 3


def test_naive_copy_rebuilt_on_every_update():
    exp = _exp()
    prod = Producer(exp)
    prod.update()
    first = prod.naive_algorithm
    prod.update()
    assert prod.naive_algorithm is not first and prod.naive_algorithm is not prod.algorithm


def test_pool_is_filled_in_one_produce():
    exp = _exp(pool_size=5)
    assert Producer(exp).produce() == 5 and len(exp.fetch_trials()) == 5


def test_produce_updates_first_when_needed():
    exp = _exp(pool_size=1)
    prod = Producer(exp)
    assert prod.naive_algorithm is None
    prod.produce()
    assert prod.naive_algorithm is not None


def test_new_trials_descend_from_the_naive_frontier():
    exp = _exp(pool_size=2, strategy={"MaxParallelStrategy": {}})
    prod = Producer(exp)
    prod.produce()
    a, b = exp.fetch_trials()
    _set(exp, a, "completed", 1.0)
    prod.update()
    frontier = list(prod.naive_trials_history.children)
    (lie,) = exp.storage.fetch_lies(exp)
    assert lie.parents == [a.id] and frontier == [lie.id]   # completed a -> lie of b -> new
    prod.produce()
    newest = [t for t in exp.fetch_trials() if t.parents]
    assert len(newest) == 2 and all(t.parents == frontier for t in newest)


def test_real_algorithm_inherits_the_naive_rng_state():
    e1, e2 = _exp(pool_size=2, name="s1"), _exp(pool_size=2, name="s2")
    p1, p2 = Producer(e1), Producer(e2)
    p1.produce()
    p2.produce()
    p1.update()
    p2.update()
    p1.produce()
    p2.produce()
    v1 = sorted(t.params[0].value for t in e1.fetch_trials())
    v2 = sorted(t.params[0].value for t in e2.fetch_trials())
    assert v1 == v2 and len(set(v1)) == 4          # same seed: same, and no repeat


def test_duplicates_within_a_pool_are_skipped():
    exp = _exp(pool_size=4, priors={"/c": "choices(['a', 'b'])"},
               algorithms={"random": {"seed": 3}})
    prod = Producer(exp, max_idle_time=0.5, backoff_max=0.01)
    with pytest.raises(SampleTimeout):
        prod.produce()                 # only 2 distinct points exist
    vals = [t.params[0].value for t in exp.fetch_trials()]
    assert sorted(vals) == ["a", "b"]


def test_duplicates_against_the_database_are_skipped():
    st = DocumentStorage(EphemeralDB())
    exp = _exp(pool_size=2, priors={"/c": "choices(['a', 'b', 'c'])"}, storage=st)
    exp.register_trial(Trial(experiment=exp.id, params=[dict(name="/c", type="categorical",
                                                             value="a")]))
    prod = Producer(exp, max_idle_time=0.5, backoff_max=0.01)
    prod.produce()
    vals = sorted(t.params[0].value for t in exp.fetch_trials())
    assert len(vals) == len(set(vals)) == 3


def test_concurrent_producers_never_duplicate():
    st = DocumentStorage(EphemeralDB())
    exp = _exp(pool_size=3, storage=st, algorithms={"random": {"seed": 5}})
    twin = build_experiment("p", storage=st)          # a second worker on the same experiment
    p1, p2 = Producer(exp, backoff_max=0.01), Producer(twin, backoff_max=0.01)
    p1.produce()
    p2.produce()
    ids = [t.id for t in exp.fetch_trials()]
    assert len(ids) == len(set(ids)) and len(ids) >= 3


def test_stops_when_the_algorithm_is_done():
    exp = _exp(pool_size=3)
    prod = Producer(exp)
    type(prod.algorithm).is_done = property(lambda self: True)
    try:
        assert prod.produce() == 0
    finally:
        del type(prod.algorithm).is_done


def test_unconfigured_experiment_is_refused():
    class _Bare:
        space = None
    with pytest.raises(RuntimeError, match="not configured"):
        Producer(_Bare())
