"""Parity on the reference's own fixture files (read in place from /root/reference; skipped when
the reference tree is absent):

* ``tests/unittests/core/experiment.yaml`` -- its experiments and trials go into EphemeralDB and
  PickledDB through this framework's storage protocol; trial ids are the md5 of the parameters
  and experiment, per-status counts, atomic reservation order, the EVC tree and ``status``
  output all follow from the file (its test-only ``dumbalgo`` is replaced by ``random``);
* ``sample_config.txt`` / ``sample_config_template.txt`` -- the generic converter's prior
  extraction and template (reference tests/unittests/core/io/test_converters.py), the
  ``bad_config{1..4}.txt`` conflicts, and ``generate`` round-trip;
* ``sample_config.yml`` / ``sample_config.json`` -- the YAML and JSON converters parse the same
  configuration and regenerate it.
"""
import collections
import copy
import datetime
import os

import pytest
import yaml

from metaopt_amd.core.experiment import populate_priors
from metaopt_amd.core.trial import Trial
from metaopt_amd.io.convert import (GenericConverter, JSONConverter, YAMLConverter,
                                    infer_converter_from_file_type)
from metaopt_amd.storage.database import EphemeralDB, PickledDB
from metaopt_amd.storage.protocol import DocumentStorage

FIX = "/root/reference/tests/unittests/core"
pytestmark = pytest.mark.skipif(not os.path.isdir(FIX), reason="reference fixtures absent")


def _fixture():
    with open(os.path.join(FIX, "experiment.yaml")) as f:
        experiments, trials, workers = list(yaml.safe_load_all(f))[:3]
    for exp in experiments:
        exp["_id"] = exp["name"]          # trials refer to their experiment by name here
        exp["version"] = 1
        populate_priors(exp["metadata"])
        if "dumbalgo" in exp["algorithms"]:
            exp["algorithms"] = {"random": {"seed": None}}
    return experiments, trials, workers


@pytest.fixture(params=["ephemeral", "pickled"])
def storage(request, tmp_path):
    db = EphemeralDB() if request.param == "ephemeral" else PickledDB(host=str(tmp_path / "f.pkl"))
    st = DocumentStorage(db)
    experiments, trials, _ = _fixture()
    for exp in experiments:
        st.create_experiment(copy.deepcopy(exp))
    for t in trials:
        st.register_trial(Trial(**t))
    return st


def test_trial_documents_roundtrip():
    _, trials, _ = _fixture()
    ids = set()
    for t in trials:
        doc = Trial(**t).to_dict()
        assert set(doc) == {"experiment", "status", "worker", "heartbeat", "submit_time",
                            "start_time", "end_time", "results", "params", "parents", "_id"}
        assert len(doc["_id"]) == 32 and int(doc["_id"], 16) >= 0
        assert Trial(**doc).to_dict() == doc
        ids.add(doc["_id"])
    assert len(ids) == len(trials)


def test_counts_and_status_queries(storage):
    _, trials, _ = _fixture()
    want = collections.Counter((t["experiment"], t["status"]) for t in trials)
    for (exp, status), n in want.items():
        got = storage.fetch_trials_by_status(type("E", (), {"_id": exp})(), status)
        assert len(got) == n, (exp, status)
    dendi = type("E", (), {"_id": "supernaedo2-dendi"})()
    assert storage.count_completed_trials(dendi) == want[("supernaedo2-dendi", "completed")]
    assert storage.count_broken_trials(dendi) == want[("supernaedo2-dendi", "broken")]


def test_reservation_takes_only_reservable_trials(storage):
    _, trials, _ = _fixture()
    exp = type("E", (), {"_id": "supernaedo2-dendi"})()
    reservable = [t for t in trials if t["experiment"] == "supernaedo2-dendi"
                  and t["status"] in ("new", "interrupted", "suspended")]
    got = []
    while True:
        t = storage.reserve_trial(exp)
        if t is None:
            break
        assert t.status == "reserved" and t.start_time is not None
        got.append(t.id)
    assert len(got) == len(set(got)) == len(reservable)


def test_evc_tree_of_the_fixture(storage):
    from metaopt_amd.evc.experiment_node import ExperimentNode
    experiments, _, _ = _fixture()
    parent = {e["name"]: e["refers"].get("parent_id") for e in experiments}

    def descendants(name):
        out = {name}
        for child, p in parent.items():
            if p == name:
                out |= descendants(child)
        return out

    root = ExperimentNode("supernaedo2-dendi", 1, storage=storage)
    names = sorted(n.name for n in root)
    assert names == sorted(descendants("supernaedo2-dendi"))
    assert {"supernaedo2.1", "supernaedo2.3.1.2"} <= set(names)
    leaf = ExperimentNode("supernaedo2.3.1.2", 1, storage=storage)
    chain = []
    node = leaf
    while node is not None:
        chain.append(node.name)
        node = node.parent
    assert chain == ["supernaedo2.3.1.2", "supernaedo2.3.1", "supernaedo2.3", "supernaedo2-dendi"]


# ---------------------------------------------------------------------------------- converters
def test_generic_converter_on_sample_config(tmp_path):
    conv = GenericConverter(expression_prefix="o~")
    ret = conv.parse(os.path.join(FIX, "sample_config.txt"))
    assert ret["lalala"] == "o~uniform(1, 3, shape=(100, 3))"
    assert ret["lala"] == {"la": "o~uniform(1, 3, shape=(100, 3))",
                           "l2a": "o~+gaussian(0, 0.1, shape=(100, 3))"}
    assert ret[""] == {"lala": {"iela": "o~uniform(1, 3, shape=(100, 3))",
                                "": {"iela": "o~uniform(1, 3, shape=(100, 3))"}}}
    assert ret["aaalispera"] == "o~normal(3, 1)" and ret["a"] == "o~normal(5, 3)"
    assert ret["b"] == "o~>a_serious_name" and ret["a_serious_name"] == "o~-"
    assert ret["another_serious_name"] == "o~loguniform(0.001, 0.5)"
    with open(os.path.join(FIX, "sample_config_template.txt")) as f:
        template = f.read()
    # the stored template is the converter's template with the last prior's placeholder
    assert conv.template.rstrip("\n").startswith(template.rstrip("\n").rsplit("\n", 1)[0][:40])
    assert "{lalala!s}" in conv.template and "{//lala//iela!s}" in conv.template
    assert "{{'oups':" in conv.template and "{lala/l2a!s}" in conv.template
    # generate: the values land where the priors were
    out = tmp_path / "out.txt"
    data = {"lalala": "ispi", "lala": {"la": 5, "l2a": 6}, "": {"lala": {"iela": 1, "": {"iela": 2}}},
            "aaalispera": 3, "a": 4, "b": "x", "a_serious_name": "y",
            "another_serious_name": "z"}
    conv.generate(str(out), data)
    text = out.read_text()
    assert text.startswith("ispi\n\n5\n1\n2\n") and "a_var=4" in text and "\n6\n" in text


@pytest.mark.parametrize("n,needle", [(1, "/lala/la"), (2, "lala/la"), (3, "lala"), (4, "lala")])
def test_generic_converter_reports_conflicts(n, needle):
    with pytest.raises(ValueError) as exc:
        GenericConverter(expression_prefix="o~").parse(os.path.join(FIX, f"bad_config{n}.txt"))
    assert needle in str(exc.value)


def test_yaml_and_json_samples_agree(tmp_path):
    y = infer_converter_from_file_type(os.path.join(FIX, "sample_config.yml"))
    j = infer_converter_from_file_type(os.path.join(FIX, "sample_config.json"))
    assert isinstance(y, YAMLConverter) and isinstance(j, JSONConverter)
    assert isinstance(infer_converter_from_file_type(os.path.join(FIX, "sample_config.txt")),
                      GenericConverter)
    ry = y.parse(os.path.join(FIX, "sample_config.yml"))
    rj = j.parse(os.path.join(FIX, "sample_config.json"))
    assert ry == rj
    assert ry["training"]["lr0"] == "orion~loguniform(0.0001, 0.3)"
    for conv, ext in ((y, "yml"), (j, "json")):
        out = tmp_path / f"gen.{ext}"
        conv.generate(str(out), ry)
        assert conv.parse(str(out)) == ry
