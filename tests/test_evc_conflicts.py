"""EVC conflict detection, marker-driven and manual resolution, branch builder, adapters chain
and branching through the experiment builder (reference: tests/unittests/core/evc/
test_conflicts.py, test_resolutions.py, core/test_branch_config.py -- behaviour, not code)."""
import copy

import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.evc import conflicts as C
from metaopt_amd.evc.adapters import (Adapter, AlgorithmChange, CodeChange, CompositeAdapter,
                                      DimensionAddition, DimensionDeletion)
from metaopt_amd.evc.branch_builder import ExperimentBranchBuilder
from metaopt_amd.io.experiment_builder import build_experiment
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage


def _config(priors, algorithms=None, vcs=None, name="exp", version=1, user="tester"):
    # the markers a user types on the command line travel in user_args, as with `mopt hunt`
    return {"name": name, "version": version, "_id": f"{name}-{version}",
            "algorithms": algorithms or {"random": {"seed": None}},
            "metadata": {"priors": dict(priors), "user": user,
                         "user_args": [f"--{k.lstrip('/')}~{v}" for k, v in priors.items()],
                         **({"VCS": vcs} if vcs is not None else {})}}


OLD = _config({"/x": "uniform(0, 1)", "/y": "uniform(0, 1)"})


def _types(conflicts):
    return sorted(type(c).__name__ for c in conflicts.get())


@pytest.fixture
def storage():
    st = DocumentStorage(EphemeralDB())
    with C.using_storage(st):
        yield st


class TestDetection:
    def test_identical_configs_only_name_conflict(self, storage):
        assert _types(C.detect_conflicts(OLD, copy.deepcopy(OLD))) == ["ExperimentNameConflict"]

    def test_new_missing_changed_dimensions(self, storage):
        new = _config({"/x": "uniform(0, 2)", "/z": "uniform(0, 1)"})
        types = _types(C.detect_conflicts(OLD, new))
        assert types == ["ChangedDimensionConflict", "ExperimentNameConflict",
                         "MissingDimensionConflict", "NewDimensionConflict"]

    def test_algorithm_and_code_conflicts(self, storage):
        new = _config(OLD["metadata"]["priors"], algorithms={"asha": {"seed": 1}},
                      vcs={"type": "git", "HEAD_sha": "abc"})
        types = _types(C.detect_conflicts(OLD, new))
        assert "AlgorithmConflict" in types and "CodeConflict" in types


class TestResolution:
    def test_markers_resolve_automatically(self, storage):
        new = _config({"/x": "uniform(0, 1)", "/y": "-", "/w": "+uniform(0, 3, default_value=1)"})
        conflicts = C.detect_conflicts(OLD, new)
        builder = ExperimentBranchBuilder(conflicts)
        assert builder.is_resolved
        reprs = sorted(repr(r) for r in conflicts.get_resolutions())
        assert "w~+uniform(0, 3, default_value=1)" in reprs and "y~-" in reprs
        assert new["version"] == 2 and new["name"] == "exp"     # version bump, same name

    def test_rename_marker(self, storage):
        new = _config({"/x": "uniform(0, 1)", "/y": ">yy", "/yy": "uniform(0, 1)"})
        conflicts = C.detect_conflicts(OLD, new)
        ExperimentBranchBuilder(conflicts)
        assert conflicts.are_resolved
        ren = [r for r in conflicts.get_resolutions()
               if type(r).__name__ == "RenameDimensionResolution"]
        assert len(ren) == 1 and repr(ren[0]) == "y~>yy"

    def test_new_dimension_without_default_needs_marker_for_auto(self, storage):
        new = _config({"/x": "uniform(0, 1)", "/y": "uniform(0, 1)", "/z": "uniform(0, 1)"})
        conflicts = C.detect_conflicts(OLD, new)
        b = ExperimentBranchBuilder(conflicts, {"manual_resolution": True})
        # unmarked resolutions are reverted in manual mode; the name conflict is always marked
        assert conflicts.get_remaining([C.NewDimensionConflict])
        b.add_dimension("z", default_value=0.5)
        assert not conflicts.get_remaining([C.NewDimensionConflict])
        adapters = b.create_adapters()
        assert any(isinstance(a, DimensionAddition) for a in adapters.adapters)

    def test_branch_to_new_name(self, storage):
        new = _config({"/x": "uniform(0, 1)", "/y": "uniform(0, 1)"})
        conflicts = C.detect_conflicts(OLD, new)
        b = ExperimentBranchBuilder(conflicts, {"branch": "child"})
        assert b.is_resolved and new["name"] == "child" and new["version"] == 1

    def test_change_types_and_revert(self, storage):
        new = _config(OLD["metadata"]["priors"], vcs={"type": "git", "HEAD_sha": "abc"},
                      algorithms={"asha": {}})
        conflicts = C.detect_conflicts(OLD, new)
        b = ExperimentBranchBuilder(conflicts, {"manual_resolution": True})
        b.set_code_change_type("noeffect")
        b.set_algo()
        kinds = [type(a) for a in b.create_adapters().adapters]
        assert CodeChange in kinds and AlgorithmChange in kinds
        code_res = conflicts.get_resolved([C.CodeConflict])[0].resolution
        conflicts.revert(code_res)
        assert conflicts.get_remaining([C.CodeConflict])
        b.set_code_change_type("sideways")     # invalid: traceback printed, conflict stays open
        assert conflicts.get_remaining([C.CodeConflict])
        b.set_code_change_type("break")
        assert not conflicts.get_remaining([C.CodeConflict])

    def test_remove_with_default(self, storage):
        new = _config({"/x": "uniform(0, 1)"})
        conflicts = C.detect_conflicts(OLD, new)
        b = ExperimentBranchBuilder(conflicts, {"manual_resolution": True})
        b.remove_dimension("y", default_value=0.5)
        dele = [a for a in b.create_adapters().adapters if isinstance(a, DimensionDeletion)]
        assert len(dele) == 1
        keep = dele[0].forward([Trial(params=[dict(name="/x", type="real", value=0.1),
                                              dict(name="/y", type="real", value=0.5)]),
                                Trial(params=[dict(name="/x", type="real", value=0.2),
                                              dict(name="/y", type="real", value=0.9)])])
        assert [t.params[0].value for t in keep] == [0.1]   # only the default survives


class TestAdapters:
    def test_code_change_types(self):
        trials = [Trial(params=[dict(name="/x", type="real", value=0.1)])]
        assert len(CodeChange("noeffect").forward(trials)) == 1
        assert CodeChange("break").forward(trials) == []
        assert len(CodeChange("noeffect").backward(trials)) == 1
        assert CodeChange("unsure").backward(trials) == []     # children may not flow back
        with pytest.raises(ValueError):
            CodeChange.validate("bogus")

    def test_configuration_roundtrip(self):
        comp = CompositeAdapter(DimensionAddition(dict(name="/z", type="real", value=1.0)),
                                AlgorithmChange(), CodeChange("noeffect"))
        again = Adapter.build(comp.configuration)
        assert again.configuration == comp.configuration


class TestBuilderBranching:
    def test_versions_and_tree(self):
        st = DocumentStorage(EphemeralDB())
        e1 = build_experiment("tree", priors={"/x": "uniform(0, 1)"}, storage=st)
        e2 = build_experiment("tree", priors={"/x": "uniform(0, 1)", "/y": "+uniform(0, 1)"},
                              storage=st)
        e3 = build_experiment("tree", priors={"/x": "uniform(0, 1)", "/y": "uniform(0, 1)"},
                              storage=st, branch="tree-b")
        assert (e1.version, e2.version) == (1, 2)
        assert e3.name == "tree-b" and e3.refers["parent_id"] == e2.id
        assert e3.refers["root_id"] == e1.id
        # reusing the stored configuration does not branch
        same = build_experiment("tree-b", priors={"/x": "uniform(0, 1)", "/y": "uniform(0, 1)"},
                                storage=st)
        assert same.id == e3.id

    def test_parent_trials_visible_through_adapters(self):
        st = DocumentStorage(EphemeralDB())
        e1 = build_experiment("vis", priors={"/x": "uniform(0, 1)"}, storage=st)
        for v in (0.1, 0.2):
            t = Trial(experiment=e1.id, status="completed",
                      params=[dict(name="/x", type="real", value=v)],
                      results=[dict(name="o", type="objective", value=v)])
            e1.register_trial(t)
        e2 = build_experiment("vis", priors={"/x": "uniform(0, 1)",
                                             "/y": "+uniform(0, 1, default_value=0.5)"},
                              storage=st)
        mine = e2.fetch_trials()
        tree = e2.fetch_trials(with_evc_tree=True)
        assert mine == [] and len(tree) == 2
        assert all({p.name for p in t.params} == {"/x", "/y"} for t in tree)
