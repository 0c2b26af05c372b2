"""Experiment registration races and configuration life cycle (behaviour of the reference's
tests/unittests/core/worker/test_experiment.py:418-509 and :642-715: who wins when two workers
configure the same experiment, what the loser sees, how a reload recovers, and the version
increment race), plus truly concurrent builders on one PickledDB file."""
import copy
import threading

import pytest

from metaopt_amd.core.experiment import Experiment, populate_priors
from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.storage.database import DuplicateKeyError, EphemeralDB, PickledDB
from metaopt_amd.storage.protocol import DocumentStorage
from metaopt_amd.utils.exceptions import RaceCondition

USER = "racer"


@pytest.fixture
def storage():
    return DocumentStorage(EphemeralDB())


def config(name="race", args=("--x~uniform(0, 1)",), version=None):
    cfg = {"name": name, "metadata": {"user": USER, "user_args": list(args)}, "max_trials": 5,
           "algorithms": "random"}
    if version is not None:
        cfg["version"] = version
    populate_priors(cfg["metadata"])
    return cfg


def n_docs(storage, name="race"):
    return len(storage.fetch_experiments({"name": name}))


def test_loser_of_registration_race_gets_duplicate_key(storage):
    loser = Experiment("race", user=USER, storage=storage)
    winner = Experiment("race", user=USER, storage=storage)
    assert loser.id is None and winner.id is None
    winner.configure(config())
    assert winner.id is not None and n_docs(storage) == 1
    with pytest.raises(DuplicateKeyError):
        loser.configure(config())
    assert n_docs(storage) == 1                      # the loser wrote nothing
    assert not loser._init_done


def test_config_without_stored_datetime_cannot_claim_existing_experiment(storage):
    Experiment("race", user=USER, storage=storage).configure(config())
    late = Experiment("race", user=USER, storage=storage)
    assert late.id is not None and not late._init_done
    with pytest.raises(DuplicateKeyError, match="existing experiment with a new config"):
        late.configure(config())
    assert n_docs(storage) == 1


def test_reloaded_loser_configures_from_stored_identity(storage):
    winner = Experiment("race", user=USER, storage=storage)
    winner.configure(config())
    loser = Experiment("race", user=USER, storage=storage)
    again = config(version=1)
    again["metadata"]["datetime"] = winner.metadata["datetime"]
    loser.configure(again)
    assert loser._init_done and loser.id == winner.id and loser.version == winner.version
    assert loser.configuration == winner.configuration
    assert n_docs(storage) == 1


def test_configured_experiment_cannot_be_reset(storage):
    exp = Experiment("race", user=USER, storage=storage)
    exp.configure(config())
    with pytest.raises(RuntimeError, match="cannot reset"):
        exp.configure(config())


def test_config_for_other_name_or_user_is_rejected(storage):
    exp = Experiment("race", user=USER, storage=storage)
    with pytest.raises(ValueError, match="inconsistent"):
        exp.configure(config(name="other"))
    cfg = config()
    cfg["metadata"]["user"] = "someone-else"
    with pytest.raises(ValueError, match="inconsistent"):
        exp.configure(cfg)
    assert n_docs(storage) == 0 and n_docs(storage, "other") == 0


def _winner_takes_version_2(storage):
    """v1 exists; a competing worker registers v2 (one new dimension) behind the loser's back."""
    base = config()
    Experiment("race", user=USER, storage=storage).configure(copy.deepcopy(base))
    loser = Experiment("race", user=USER, version=1, storage=storage)
    assert loser.version == 1
    parent = storage.fetch_experiments({"name": "race", "version": 1})[0]
    v2 = config(args=("--x~uniform(0, 1)", "--y~+normal(0, 1)"), version=2)
    v2["refers"] = {"parent_id": parent["_id"], "root_id": parent["_id"], "adapter": []}
    v2["metadata"]["datetime"] = parent["metadata"]["datetime"]
    storage.create_experiment(v2)
    return loser, parent


def test_version_increment_race_without_version_raises_race_condition(storage):
    loser, parent = _winner_takes_version_2(storage)
    mine = config(args=("--x~uniform(0, 1)", "--z~+normal(0, 1)"))
    mine["metadata"]["datetime"] = parent["metadata"]["datetime"]
    with pytest.raises(RaceCondition, match="race condition"):
        loser.configure(mine)
    assert n_docs(storage) == 2


def test_version_increment_race_with_version_needs_branching(storage):
    loser, parent = _winner_takes_version_2(storage)
    mine = config(args=("--x~uniform(0, 1)", "--z~+normal(0, 1)"), version=1)
    mine["metadata"]["datetime"] = parent["metadata"]["datetime"]
    # the conflict cannot be resolved automatically and there is no TTY for the prompt
    with pytest.raises(ValueError, match="branching"):
        loser.configure(mine)
    assert n_docs(storage) == 2


def test_non_branching_change_updates_in_place(storage):
    exp = Experiment("race", user=USER, storage=storage)
    exp.configure(config())
    again = config(version=1)
    again["max_trials"] = 50                         # pool_size / max_trials never branch
    again["metadata"]["datetime"] = exp.metadata["datetime"]
    other = Experiment("race", user=USER, storage=storage)
    other.configure(again)
    assert other.id == exp.id and other.max_trials == 50
    assert n_docs(storage) == 1
    assert storage.fetch_experiments({"name": "race"})[0]["max_trials"] == 50


@pytest.mark.parametrize("n_workers", [4])
def test_concurrent_builders_share_one_experiment(tmp_path, n_workers):
    """N threads build the same experiment at once on one PickledDB file: the builder's
    race handling leaves exactly one document and every worker attached to it."""
    path = str(tmp_path / "race.pkl")
    ids, errors = [], []
    barrier = threading.Barrier(n_workers)

    def worker():
        try:
            st = DocumentStorage(PickledDB(host=path))
            barrier.wait()
            exp = build_experiment("shared", priors={"/x": "uniform(0, 1)"}, max_trials=10,
                                   storage=st)
            ids.append(exp.id)
        except Exception as exc:                      # pragma: no cover - reported below
            errors.append(exc)

    threads = [threading.Thread(target=worker) for _ in range(n_workers)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not errors, errors
    assert len(ids) == n_workers and len(set(ids)) == 1
    st = DocumentStorage(PickledDB(host=path))
    assert len(st.fetch_experiments({"name": "shared"})) == 1


def test_concurrent_reservations_hand_out_each_trial_once(tmp_path):
    """Workers racing on reserve_trial over one PickledDB never get the same trial twice."""
    from metaopt_amd.core.trial import Trial
    path = str(tmp_path / "reserve.pkl")
    st = DocumentStorage(PickledDB(host=path))
    exp = build_experiment("pool", priors={"/x": "uniform(0, 1)"}, storage=st)
    for i in range(24):
        t = Trial(experiment=exp.id, params=[dict(name="/x", type="real", value=i / 24)])
        exp.register_trial(t)
    got, lock = [], threading.Lock()

    def worker():
        mine = DocumentStorage(PickledDB(host=path))
        view = Experiment("pool", storage=mine)
        while True:
            t = view.reserve_trial()
            if t is None:
                return
            with lock:
                got.append(t.id)

    threads = [threading.Thread(target=worker) for _ in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert len(got) == 24 and len(set(got)) == 24
