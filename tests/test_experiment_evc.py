"""Experiment life cycle and EVC adapters (reference tests: core/worker/test_experiment.py,
core/evc/test_adapters.py, core/evc/test_conflicts.py)."""
import datetime

import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.evc.adapters import (Adapter, CompositeAdapter, DimensionAddition,
                                      DimensionDeletion, DimensionPriorChange, DimensionRenaming)
from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage


@pytest.fixture
def exp():
    return build_experiment("life", priors={"/x": "uniform(0, 1)"}, max_trials=3,
                            storage=DocumentStorage(EphemeralDB()))


def _t(exp, x, status="new"):
    t = Trial(experiment=exp.id, status=status,
              params=[dict(name="/x", type="real", value=x)])
    t.submit_time = datetime.datetime.utcnow()
    return t


def test_reserve_complete_and_done(exp):
    for x in (0.1, 0.2, 0.3):
        exp.register_trial(_t(exp, x))
    got = [exp.reserve_trial() for _ in range(4)]
    assert sum(t is not None for t in got) == 3
    assert not exp.is_done
    for t in got[:3]:
        t.results = [Trial.Result(name="o", type="objective", value=t.params[0].value)]
        t.status = "completed"
        exp.storage.push_trial_results(t)
    assert exp.is_done
    st = exp.stats
    assert st["trials_completed"] == 3 and st["best_evaluation"] == pytest.approx(0.1)


def test_fix_lost_trials(exp):
    exp.register_trial(_t(exp, 0.5))
    t = exp.reserve_trial()
    old = datetime.datetime.utcnow() - datetime.timedelta(seconds=10_000)
    exp.storage._db.write("trials", {"heartbeat": old}, {"_id": t.id})
    exp.fix_lost_trials()
    assert exp.get_trial(t).status == "interrupted"
    assert exp.reserve_trial().id == t.id          # interrupted trials are reservable again


def test_is_broken(exp):
    for x in (0.1, 0.2, 0.3):
        exp.storage.register_trial(_t(exp, x, status="broken"))
    assert exp.is_broken


def test_same_name_new_version_on_conflicting_space():
    storage = DocumentStorage(EphemeralDB())
    e1 = build_experiment("evc", priors={"/x": "uniform(0, 1)"}, storage=storage)
    e2 = build_experiment("evc", priors={"/x": "uniform(0, 1)", "/y": "+uniform(0, 2)"},
                          storage=storage)
    assert e2.version == e1.version + 1
    assert e2.refers["parent_id"] == e1.id


def _trial(**params):
    return Trial(experiment=1, params=[dict(name=k, type="real", value=v)
                                       for k, v in sorted(params.items())])


def test_dimension_addition_and_deletion():
    add = DimensionAddition(dict(name="/y", type="real", value=1.0))
    fwd = add.forward([_trial(**{"/x": 0.5})])
    assert [p.name for p in fwd[0].params] == ["/x", "/y"]
    back = add.backward([_trial(**{"/x": 0.5, "/y": 1.0}), _trial(**{"/x": 0.5, "/y": 2.0})])
    assert len(back) == 1 and [p.name for p in back[0].params] == ["/x"]
    dele = DimensionDeletion(dict(name="/y", type="real", value=1.0))
    assert len(dele.forward([_trial(**{"/x": 0.5, "/y": 1.0})])) == 1
    with pytest.raises(RuntimeError):
        add.forward([_trial(**{"/y": 0.5})])


def test_prior_change_renaming_and_composite_roundtrip():
    prior = DimensionPriorChange("/x", "uniform(0, 1)", "uniform(0, 0.5)")
    kept = prior.forward([_trial(**{"/x": 0.2}), _trial(**{"/x": 0.8})])
    assert [t.params[0].value for t in kept] == [0.2]
    ren = DimensionRenaming("/x", "/z")
    assert ren.forward([_trial(**{"/x": 0.2})])[0].params[0].name == "/z"
    assert ren.backward([_trial(**{"/z": 0.2})])[0].params[0].name == "/x"
    comp = CompositeAdapter(prior, ren)
    rebuilt = Adapter.build(comp.configuration)
    assert rebuilt.configuration == comp.configuration
    assert [t.params[0].name for t in rebuilt.forward([_trial(**{"/x": 0.1})])] == ["/z"]
