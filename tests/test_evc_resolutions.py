"""EVC conflicts, resolutions, markers, the conflict list and the branch builder in depth.

Behaviour parity targets (written fresh against this package's API): the reference's
tests/unittests/core/evc/test_conflicts.py, test_resolutions.py and
tests/unittests/core/test_branch_config.py -- every conflict type's detection, each
resolution's defaults / validation / textual form / adapters, resolving twice, reverting,
side conflicts of renames, the list queries, the name conflict against stored experiments,
and automatic vs manual resolution driven by markers and flags.
"""
import copy

import pytest

from metaopt_amd.core.trial import Trial
from metaopt_amd.evc import adapters as A
from metaopt_amd.evc import conflicts as C
from metaopt_amd.evc.branch_builder import ExperimentBranchBuilder
from metaopt_amd.space.builder import DimensionBuilder
from metaopt_amd.storage.database import EphemeralDB
from metaopt_amd.storage.protocol import DocumentStorage

NO_DEFAULT = C.NO_DEFAULT


def cfg(priors, name="exp", version=1, user="tester", algorithms=None, vcs=None, extra_args=(),
        **flags):
    """An experiment configuration as the builder stores it; markers ride in user_args."""
    args = [f"--{k.lstrip('/')}~{v}" for k, v in priors.items()] + list(extra_args)
    clean = {k: v.lstrip("+") for k, v in priors.items() if v[:1] not in "->"}
    out = {"name": name, "version": version, "_id": f"{name}-v{version}",
           "algorithms": algorithms or {"random": {"seed": None}},
           "metadata": {"priors": clean, "user": user, "user_args": args}}
    if vcs is not None:
        out["metadata"]["VCS"] = vcs
    out.update(flags)
    return out


BASE = {"/x": "uniform(0, 1)", "/y": "uniform(0, 10, default_value=5)"}


@pytest.fixture
def storage():
    st = DocumentStorage(EphemeralDB())
    with C.using_storage(st):
        yield st


def dim(name, prior):
    return DimensionBuilder().build(name, prior)


def one(conflicts, kind):
    found = conflicts.get([kind])
    assert len(found) == 1, found
    return found[0]


def kinds(conflicts):
    return sorted(type(c).__name__ for c in conflicts.get())


def trial(**params):
    return Trial(params=[dict(name=f"/{k}", type="real", value=v)
                         for k, v in sorted(params.items())])


# =========================================================================== detection
class TestDetection:
    def test_name_conflict_is_always_there(self, storage):
        assert kinds(C.detect_conflicts(cfg(BASE), cfg(BASE))) == ["ExperimentNameConflict"]

    def test_one_new_dimension(self, storage):
        c = C.detect_conflicts(cfg(BASE), cfg({**BASE, "/z": "uniform(0, 1)"}))
        z = one(c, C.NewDimensionConflict)
        assert z.dimension.name == "/z" and z.prior == "uniform(0, 1)"

    def test_one_missing_dimension(self, storage):
        c = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)"}))
        y = one(c, C.MissingDimensionConflict)
        assert y.dimension.name == "/y" and y.prior == "uniform(0, 10, default_value=5)"

    def test_one_changed_dimension(self, storage):
        c = C.detect_conflicts(cfg(BASE), cfg({**BASE, "/x": "uniform(0, 2)"}))
        x = one(c, C.ChangedDimensionConflict)
        assert (x.old_prior, x.new_prior) == ("uniform(0, 1)", "uniform(0, 2)")

    def test_default_value_change_is_a_prior_change(self, storage):
        c = C.detect_conflicts(cfg(BASE), cfg({**BASE, "/y": "uniform(0, 10, default_value=6)"}))
        assert one(c, C.ChangedDimensionConflict).dimension.name == "/y"

    def test_several_dimensions_at_once(self, storage):
        new = {"/x": "uniform(0, 3)", "/a": "uniform(0, 1)", "/b": "uniform(0, 1)"}
        c = C.detect_conflicts(cfg(BASE), cfg(new))
        assert len(c.get([C.NewDimensionConflict])) == 2
        assert len(c.get([C.MissingDimensionConflict])) == 1
        assert len(c.get([C.ChangedDimensionConflict])) == 1

    def test_algorithm_change(self, storage):
        c = C.detect_conflicts(cfg(BASE), cfg(BASE, algorithms={"asha": {"seed": 1}}))
        assert "AlgorithmConflict" in kinds(c)

    def test_algorithm_argument_change(self, storage):
        c = C.detect_conflicts(cfg(BASE, algorithms={"random": {"seed": 1}}),
                               cfg(BASE, algorithms={"random": {"seed": 2}}))
        assert "AlgorithmConflict" in kinds(c)

    def test_code_change_needs_new_vcs(self, storage):
        vcs = {"type": "git", "HEAD_sha": "a"}
        assert "CodeConflict" not in kinds(C.detect_conflicts(cfg(BASE, vcs=vcs), cfg(BASE)))
        assert "CodeConflict" not in kinds(C.detect_conflicts(cfg(BASE, vcs=vcs),
                                                               cfg(BASE, vcs=dict(vcs))))
        assert "CodeConflict" in kinds(C.detect_conflicts(
            cfg(BASE, vcs=vcs), cfg(BASE, vcs={"type": "git", "HEAD_sha": "b"})))

    def test_code_change_from_nothing(self, storage):
        c = C.detect_conflicts(cfg(BASE), cfg(BASE, vcs={"type": "git", "HEAD_sha": "b"}))
        assert "CodeConflict" in kinds(c)

    def test_registry_priorities(self):
        order = [c.__name__ for c in C.REGISTRY]
        assert order[0] == "ExperimentNameConflict"
        assert order.index("MissingDimensionConflict") < order.index("NewDimensionConflict")
        assert len(order) == 8

    def test_detection_order_follows_priority(self, storage):
        new = {"/x": "uniform(0, 3)", "/a": "uniform(0, 1)"}
        c = C.detect_conflicts(cfg(BASE), cfg(new, algorithms={"asha": {}}))
        prios = [x.priority for x in c.get()]
        assert prios == sorted(prios)


# =========================================================================== markers
class TestMarkers:
    def test_removal_marker(self):
        m = C.Markers(cfg({"/y": "-"}))
        assert m.get("/y", "-") == "" and m.get("y", "-") == ""
        assert m.get("y", ">") is None and m.get("x", "-") is None

    def test_removal_marker_with_default(self):
        assert C.Markers(cfg({"/y": "-3.5"})).get("y", "-") == "3.5"

    def test_rename_marker(self):
        assert C.Markers(cfg({"/y": ">z"})).get("y", ">") == "z"

    def test_addition_marker(self):
        m = C.Markers(cfg({"/w": "+uniform(0, 1)"}))
        assert m.get("w", "+") == "uniform(0, 1)"

    def test_plain_priors_are_not_markers(self):
        assert C.Markers(cfg(BASE)).marks == {}

    def test_nested_names_normalised(self):
        m = C.Markers(cfg({"/model/lr": "-"}))
        assert m.get("/model/lr", "-") == ""

    def test_flags_read_live_from_config(self):
        config = cfg(BASE)
        m = C.Markers(config)
        assert m.flag("branch") is None
        config["branch"] = "other"
        assert m.flag("branch") == "other"

    def test_first_marker_wins(self):
        m = C.Markers(cfg({}, extra_args=["--y~-", "--y~>z"]))
        assert m.get("y", "-") == "" and m.get("y", ">") is None


# =========================================================================== new dimension
class TestNewDimension:
    @pytest.fixture
    def conflict(self, storage):
        return one(C.detect_conflicts(cfg(BASE), cfg({**BASE, "/z": "uniform(0, 10)"})),
                   C.NewDimensionConflict)

    @pytest.fixture
    def conflict_with_default(self, storage):
        return one(C.detect_conflicts(cfg(BASE),
                                      cfg({**BASE, "/z": "uniform(0, 10, default_value=2)"})),
                   C.NewDimensionConflict)

    def test_resolve_without_default(self, conflict):
        r = conflict.try_resolve()
        assert isinstance(r, C.AddDimensionResolution) and conflict.is_resolved
        assert r.default_value is NO_DEFAULT

    def test_default_from_the_prior(self, conflict_with_default):
        assert conflict_with_default.try_resolve().default_value == 2

    def test_explicit_default(self, conflict):
        assert conflict.try_resolve(default_value=4).default_value == 4.0

    def test_explicit_default_overrides_prior(self, conflict_with_default):
        assert conflict_with_default.try_resolve(default_value=7).default_value == 7.0

    def test_default_is_cast(self, conflict):
        assert conflict.try_resolve(default_value="3").default_value == 3.0

    def test_bad_default_leaves_conflict_open(self, conflict):
        with pytest.raises(ValueError, match="outside"):
            conflict.try_resolve(default_value=11)
        assert not conflict.is_resolved and conflict.resolution is None

    def test_twice_returns_none(self, conflict):
        assert conflict.try_resolve() is not None
        assert conflict.try_resolve() is None

    def test_repr_and_diff(self, conflict):
        assert repr(conflict) == "New z"
        assert "z" in conflict.diff

    def test_resolution_repr_carries_default(self, conflict):
        assert repr(conflict.try_resolve(default_value=4)) == \
            "z~+uniform(0, 10, default_value=4.0)"

    def test_resolution_repr_without_default(self, conflict):
        assert repr(conflict.try_resolve()) == "z~+uniform(0, 10)"

    def test_adapter(self, conflict):
        (adapter,) = conflict.try_resolve(default_value=4).adapters()
        assert isinstance(adapter, A.DimensionAddition)
        assert adapter.param.to_dict() == {"name": "/z", "type": "real", "value": 4.0}

    def test_adapter_moves_parent_trials(self, conflict):
        (adapter,) = conflict.try_resolve(default_value=4).adapters()
        (t,) = adapter.forward([trial(x=0.5, y=1.0)])
        assert [p.name for p in t.params] == ["/x", "/y", "/z"]


# =========================================================================== changed dimension
class TestChangedDimension:
    @pytest.fixture
    def conflict(self, storage):
        return one(C.detect_conflicts(cfg(BASE), cfg({**BASE, "/x": "uniform(0, 2)"})),
                   C.ChangedDimensionConflict)

    def test_resolve(self, conflict):
        assert isinstance(conflict.try_resolve(), C.ChangeDimensionResolution)

    def test_twice(self, conflict):
        conflict.try_resolve()
        assert conflict.try_resolve() is None

    def test_repr(self, conflict):
        assert repr(conflict) == "x~uniform(0, 1) != x~uniform(0, 2)"
        assert repr(conflict.try_resolve()) == "x~+uniform(0, 2)"

    def test_adapter_filters_by_the_new_prior(self, conflict):
        (adapter,) = conflict.try_resolve().adapters()
        assert isinstance(adapter, A.DimensionPriorChange)
        kept = adapter.forward([trial(x=0.5, y=1.0), trial(x=1.5, y=1.0)])
        assert len(kept) == 2
        back = adapter.backward([trial(x=0.5, y=1.0), trial(x=1.5, y=1.0)])
        assert [t.params[0].value for t in back] == [0.5]

    def test_diff(self, conflict):
        assert "uniform(0, 1)" in conflict.diff and "uniform(0, 2)" in conflict.diff


# =========================================================================== missing dimension
class TestMissingDimension:
    @pytest.fixture
    def conflicts(self, storage):
        return C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)",
                                                  "/w": "uniform(0, 10, default_value=5)"}))

    @pytest.fixture
    def conflict(self, conflicts):
        return one(conflicts, C.MissingDimensionConflict)

    def test_remove_with_the_prior_default(self, conflict):
        r = conflict.try_resolve()
        assert isinstance(r, C.RemoveDimensionResolution) and r.default_value == 5

    def test_remove_with_explicit_default(self, conflict):
        assert conflict.try_resolve(default_value=1).default_value == 1.0

    def test_remove_bad_default(self, conflict):
        with pytest.raises(ValueError, match="outside"):
            conflict.try_resolve(default_value=-1)
        assert not conflict.is_resolved

    def test_remove_repr(self, conflict):
        assert repr(conflict.try_resolve(default_value=1)) == "y~-1.0"

    def test_remove_repr_without_default(self, storage):
        c = one(C.detect_conflicts(cfg({"/x": "uniform(0, 1)", "/q": "uniform(0, 1)"}),
                                   cfg({"/x": "uniform(0, 1)"})), C.MissingDimensionConflict)
        assert repr(c.try_resolve()) == "q~-"

    def test_remove_adapter_keeps_trials_at_default(self, conflict):
        (adapter,) = conflict.try_resolve(default_value=1).adapters()
        assert isinstance(adapter, A.DimensionDeletion)
        kept = adapter.forward([trial(x=0.1, y=1.0), trial(x=0.2, y=2.0)])
        assert len(kept) == 1 and [p.name for p in kept[0].params] == ["/x"]

    def test_rename(self, conflicts, conflict):
        target = one(conflicts, C.NewDimensionConflict)
        r = conflicts.try_resolve(conflict, new_dimension_conflict=target)
        assert isinstance(r, C.RenameDimensionResolution)
        assert conflict.is_resolved and target.is_resolved
        assert target.resolution is r
        assert repr(r) == "y~>w"

    def test_rename_same_prior_has_no_side_conflict(self, conflicts, conflict):
        target = one(conflicts, C.NewDimensionConflict)
        r = conflicts.try_resolve(conflict, new_dimension_conflict=target)
        assert r.side_conflicts == []

    def test_rename_with_prior_change_raises_side_conflict(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/w": "uniform(0, 3)"}))
        r = cs.try_resolve(one(cs, C.MissingDimensionConflict),
                           new_dimension_conflict=one(cs, C.NewDimensionConflict))
        (side,) = r.side_conflicts
        assert isinstance(side, C.ChangedDimensionConflict) and side in cs.get()
        assert (side.old_prior, side.new_prior) == ("uniform(0, 10, default_value=5)",
                                                     "uniform(0, 3)")

    def test_revert_rename_reopens_both_and_drops_side(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/w": "uniform(0, 3)"}))
        miss, new = one(cs, C.MissingDimensionConflict), one(cs, C.NewDimensionConflict)
        r = cs.try_resolve(miss, new_dimension_conflict=new)
        n = len(cs.get())
        cs.revert(r)
        assert not miss.is_resolved and not new.is_resolved
        assert len(cs.get()) == n - 1
        assert not cs.get([C.ChangedDimensionConflict])

    def test_rename_onto_a_resolved_dimension_is_refused(self, conflicts, conflict):
        target = one(conflicts, C.NewDimensionConflict)
        target.try_resolve()
        with pytest.raises(ValueError, match="already resolved"):
            conflict.try_resolve(new_dimension_conflict=target)
        assert not conflict.is_resolved

    def test_rename_adapter(self, conflicts, conflict):
        r = conflicts.try_resolve(conflict, new_dimension_conflict=one(conflicts,
                                                                       C.NewDimensionConflict))
        (adapter,) = r.adapters()
        assert isinstance(adapter, A.DimensionRenaming)
        (t,) = adapter.forward([trial(x=0.1, y=3.0)])
        assert [p.name for p in t.params] == ["/w", "/x"]

    def test_twice(self, conflict):
        conflict.try_resolve()
        assert conflict.try_resolve() is None

    def test_repr_and_diff(self, conflict):
        assert repr(conflict) == "Missing y"
        assert "y" in conflict.diff


# =========================================================================== algorithm
class TestAlgorithm:
    @pytest.fixture
    def conflict(self, storage):
        return one(C.detect_conflicts(cfg(BASE), cfg(BASE, algorithms={"asha": {"seed": 1}})),
                   C.AlgorithmConflict)

    def test_resolve_and_adapter(self, conflict):
        r = conflict.try_resolve()
        assert repr(r) == "--algorithm-change"
        assert [type(a) for a in r.adapters()] == [A.AlgorithmChange]

    def test_twice(self, conflict):
        conflict.try_resolve()
        assert conflict.try_resolve() is None

    def test_repr_shows_both(self, conflict):
        text = repr(conflict)
        assert "random" in text and "asha" in text and "!=" in text

    def test_diff(self, conflict):
        assert "asha" in conflict.diff

    def test_is_marked_by_flag(self, storage):
        new = cfg(BASE, algorithms={"asha": {}})
        c = one(C.detect_conflicts(cfg(BASE), new), C.AlgorithmConflict)
        r = c.try_resolve()
        assert not r.is_marked
        new["algorithm_change"] = True
        assert r.is_marked


# =========================================================================== typed changes
VCS_A = {"type": "git", "HEAD_sha": "aaa", "is_dirty": False}
VCS_B = {"type": "git", "HEAD_sha": "bbb", "is_dirty": False}


class TestTypedChanges:
    @pytest.fixture
    def code(self, storage):
        return one(C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B)),
                   C.CodeConflict)

    @pytest.mark.parametrize("kind", ["noeffect", "break", "unsure"])
    def test_each_change_type(self, code, kind):
        r = code.try_resolve(kind)
        assert r.type == kind and repr(r) == f"--code-change-type {kind}"
        (adapter,) = r.adapters()
        assert isinstance(adapter, A.CodeChange) and adapter.change_type == kind

    def test_bad_type_leaves_open(self, code):
        with pytest.raises(ValueError, match="change type"):
            code.try_resolve("often")
        assert not code.is_resolved

    def test_twice(self, code):
        code.try_resolve("break")
        assert code.try_resolve("noeffect") is None

    def test_repr(self, code):
        assert "aaa" in repr(code) and "bbb" in repr(code)

    def test_marked_arguments_default_break(self, storage):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B))
        assert cs.marked_arguments(one(cs, C.CodeConflict)) == {"change_type": "break"}

    def test_marked_arguments_from_flag(self, storage):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A),
                                cfg(BASE, vcs=VCS_B, code_change_type="noeffect"))
        assert cs.marked_arguments(one(cs, C.CodeConflict)) == {"change_type": "noeffect"}

    def test_command_line_conflict(self, storage):
        from metaopt_amd.io.space_parser import SpaceCmdlineParser
        old, new = cfg(BASE), cfg(BASE)
        for conf, extra in ((old, ["--epochs", "3"]), (new, ["--epochs", "5"])):
            p = SpaceCmdlineParser()
            p.parse(["script.py", "--x~uniform(0, 1)"] + extra)
            conf["metadata"]["parser"] = p.get_state_dict()
        cs = C.detect_conflicts(old, new)
        cli = one(cs, C.CommandLineConflict)
        assert "3" in repr(cli) and "5" in repr(cli)
        r = cli.try_resolve("unsure")
        assert repr(r) == "--cli-change-type unsure"
        assert isinstance(r.adapters()[0], A.CommandLineChange)

    def test_command_line_same_args_no_conflict(self, storage):
        from metaopt_amd.io.space_parser import SpaceCmdlineParser
        old, new = cfg(BASE), cfg(BASE)
        for conf in (old, new):
            p = SpaceCmdlineParser()
            p.parse(["script.py", "--x~uniform(0, 1)", "--epochs", "3"])
            conf["metadata"]["parser"] = p.get_state_dict()
        assert "CommandLineConflict" not in kinds(C.detect_conflicts(old, new))

    def test_command_line_prior_change_is_not_a_cli_change(self, storage):
        from metaopt_amd.io.space_parser import SpaceCmdlineParser
        old, new = cfg(BASE), cfg(BASE)
        for conf, prior in ((old, "uniform(0, 1)"), (new, "uniform(0, 2)")):
            p = SpaceCmdlineParser()
            p.parse(["script.py", f"--x~{prior}", "--epochs", "3"])
            conf["metadata"]["parser"] = p.get_state_dict()
        assert "CommandLineConflict" not in kinds(C.detect_conflicts(old, new))

    def test_script_config_conflict(self, storage, tmp_path):
        import yaml
        from metaopt_amd.io.space_parser import SpaceCmdlineParser
        old, new = cfg(BASE), cfg(BASE)
        for conf, layers in ((old, 2), (new, 3)):
            path = tmp_path / f"c{layers}.yaml"
            path.write_text(yaml.safe_dump({"lr": "orion~uniform(0, 1)", "layers": layers}))
            p = SpaceCmdlineParser()
            p.parse(["script.py", "--config", str(path)])
            conf["metadata"]["parser"] = p.get_state_dict()
        cs = C.detect_conflicts(old, new)
        sc = one(cs, C.ScriptConfigConflict)
        assert repr(sc) == "Script's configuration file changed"
        assert "layers" in sc.diff
        assert repr(sc.try_resolve("noeffect")) == "--config-change-type noeffect"

    def test_script_config_prior_only_change_is_not_a_config_change(self, storage, tmp_path):
        import yaml
        from metaopt_amd.io.space_parser import SpaceCmdlineParser
        old, new = cfg(BASE), cfg(BASE)
        for conf, prior in ((old, "uniform(0, 1)"), (new, "uniform(0, 2)")):
            path = tmp_path / f"c{prior[-2]}.yaml"
            path.write_text(yaml.safe_dump({"lr": f"orion~{prior}", "layers": 2}))
            p = SpaceCmdlineParser()
            p.parse(["script.py", "--config", str(path)])
            conf["metadata"]["parser"] = p.get_state_dict()
        assert "ScriptConfigConflict" not in kinds(C.detect_conflicts(old, new))


# =========================================================================== experiment name
class TestExperimentName:
    def _register(self, storage, name, version=1, parent=None, user="tester"):
        doc = {"name": name, "version": version, "metadata": {"user": user},
               "refers": {"parent_id": parent}}
        storage.create_experiment(doc)
        return doc

    def test_version_increment(self, storage):
        old = self._register(storage, "exp")
        cs = C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), cfg(BASE))
        r = one(cs, C.ExperimentNameConflict).try_resolve()
        assert (r.new_name, r.new_version) == ("exp", 2)
        assert repr(r) == "--branch exp"

    def test_new_name(self, storage):
        old = self._register(storage, "exp")
        new = cfg(BASE)
        cs = C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), new)
        r = one(cs, C.ExperimentNameConflict).try_resolve("fork")
        assert (new["name"], new["version"]) == ("fork", 1)
        assert repr(r) == "--branch fork"

    def test_existing_name_is_refused(self, storage):
        old = self._register(storage, "exp")
        self._register(storage, "taken")
        c = one(C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), cfg(BASE)),
                C.ExperimentNameConflict)
        with pytest.raises(ValueError, match="already exists"):
            c.try_resolve("taken")
        assert not c.is_resolved

    def test_existing_name_of_another_user_is_fine(self, storage):
        old = self._register(storage, "exp")
        self._register(storage, "theirs", user="someone-else")
        c = one(C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), cfg(BASE)),
                C.ExperimentNameConflict)
        assert c.try_resolve("theirs").new_version == 1

    def test_no_increment_when_children_exist(self, storage):
        old = self._register(storage, "exp")
        self._register(storage, "exp", version=2, parent=old["_id"])
        c = one(C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), cfg(BASE)),
                C.ExperimentNameConflict)
        with pytest.raises(ValueError, match="has children"):
            c.try_resolve()
        assert c.try_resolve("fresh").new_name == "fresh"

    def test_child_of_other_name_does_not_block(self, storage):
        old = self._register(storage, "exp")
        self._register(storage, "fork", parent=old["_id"])
        c = one(C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), cfg(BASE)),
                C.ExperimentNameConflict)
        assert c.try_resolve().new_version == 2

    def test_increment_from_latest_version(self, storage):
        self._register(storage, "exp")
        v2 = self._register(storage, "exp", version=2)
        cs = C.detect_conflicts(dict(cfg(BASE, version=2), _id=v2["_id"]), cfg(BASE))
        assert one(cs, C.ExperimentNameConflict).try_resolve().new_version == 3

    def test_revert_restores_name_and_version(self, storage):
        old = self._register(storage, "exp")
        new = cfg(BASE, name="exp", version=1)
        cs = C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), new)
        r = one(cs, C.ExperimentNameConflict).try_resolve("fork")
        cs.revert(r)
        assert (new["name"], new["version"]) == ("exp", 1)

    def test_always_marked(self, storage):
        old = self._register(storage, "exp")
        r = one(C.detect_conflicts(dict(cfg(BASE), _id=old["_id"]), cfg(BASE)),
                C.ExperimentNameConflict).try_resolve()
        assert r.is_marked and r.adapters() == []

    def test_repr(self, storage):
        c = one(C.detect_conflicts(cfg(BASE), cfg(BASE)), C.ExperimentNameConflict)
        assert repr(c) == "Experiment name 'exp' already exist for user 'tester'"

    def test_marked_arguments(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg(BASE, branch="b2"))
        assert cs.marked_arguments(one(cs, C.ExperimentNameConflict)) == {"new_name": "b2"}
        cs = C.detect_conflicts(cfg(BASE), cfg(BASE))
        assert cs.marked_arguments(one(cs, C.ExperimentNameConflict)) is None


# =========================================================================== the list
class TestConflictsList:
    @pytest.fixture
    def cs(self, storage):
        new = {"/x": "uniform(0, 3)", "/a": "uniform(0, 1)", "/b": "uniform(0, 1)"}
        return C.detect_conflicts(cfg(BASE), cfg(new, algorithms={"asha": {}}))

    def test_get_all(self, cs):
        assert len(cs.get()) == 6

    def test_get_one_type(self, cs):
        assert len(cs.get([C.NewDimensionConflict])) == 2

    def test_get_several_types(self, cs):
        assert len(cs.get([C.NewDimensionConflict, C.AlgorithmConflict])) == 3

    def test_get_by_dimension(self, cs):
        (a,) = cs.get(dimension_name="a")
        assert a.dimension.name == "/a"

    def test_get_by_dimension_and_type(self, cs):
        assert cs.get([C.ChangedDimensionConflict], dimension_name="x")
        with pytest.raises(ValueError, match="not found"):
            cs.get([C.NewDimensionConflict], dimension_name="x")

    def test_unknown_dimension(self, cs):
        with pytest.raises(ValueError, match="'nope' not found"):
            cs.get(dimension_name="nope")

    def test_callback(self, cs):
        found = cs.get(callback=lambda c: isinstance(c, C.NewDimensionConflict)
                       and c.dimension.name == "/b")
        assert len(found) == 1

    def test_remaining_and_resolved(self, cs):
        cs.try_resolve(cs.get([C.AlgorithmConflict])[0])
        assert len(cs.get_resolved()) == 1 and len(cs.get_remaining()) == 5
        assert not cs.are_resolved

    def test_resolutions_are_distinct(self, cs):
        miss = one(cs, C.MissingDimensionConflict)
        cs.try_resolve(miss, new_dimension_conflict=cs.get(dimension_name="a")[0])
        assert len(cs.get_resolved()) == 2          # the renamed pair, by one resolution
        assert len(list(cs.get_resolutions())) == 1
        # y's prior differs from a's: the rename raised an open side prior change on a
        (side,) = cs.get_remaining([C.ChangedDimensionConflict], dimension_name="a")
        assert side.new_prior == "uniform(0, 1)"

    def test_are_resolved(self, cs):
        for c in list(cs.get()):
            if isinstance(c, C.MissingDimensionConflict):
                cs.try_resolve(c, default_value=5)
            else:
                cs.try_resolve(c)
        assert cs.are_resolved

    def test_deprecate(self, cs):
        n = len(cs.get())
        cs.deprecate([cs.get([C.AlgorithmConflict])[0]])
        assert len(cs.get()) == n - 1

    def test_deprecate_unknown(self, cs):
        other = C.AlgorithmConflict(cfg(BASE), cfg(BASE))
        with pytest.raises(ValueError):
            cs.deprecate([other])

    def test_try_resolve_error_prints_traceback(self, storage, capsys):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B))
        assert cs.try_resolve(one(cs, C.CodeConflict), "never") is None
        assert "Traceback" in capsys.readouterr().out

    def test_try_resolve_error_silenced(self, storage, capsys):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B))
        assert cs.try_resolve(one(cs, C.CodeConflict), "never", silence_errors=True) is None
        assert capsys.readouterr().out == ""

    def test_try_resolve_keyboard_interrupt_propagates(self, cs, monkeypatch):
        algo = one(cs, C.AlgorithmConflict)

        def interrupt(*a, **k):
            raise KeyboardInterrupt
        monkeypatch.setattr(algo, "_resolve", interrupt)
        with pytest.raises(KeyboardInterrupt):
            cs.try_resolve(algo)

    def test_revert_by_text(self, cs):
        cs.try_resolve(one(cs, C.AlgorithmConflict))
        cs.revert("--algorithm-change")
        assert not one(cs, C.AlgorithmConflict).is_resolved

    def test_revert_unknown_text(self, cs):
        with pytest.raises(ValueError, match="no resolution"):
            cs.revert("--nothing")


# =========================================================================== branch builder
class TestBranchBuilder:
    def test_markers_resolve_removal_with_default(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/y": "-7"}))
        b = ExperimentBranchBuilder(cs)
        assert b.is_resolved
        (res,) = [r for r in cs.get_resolutions() if isinstance(r, C.RemoveDimensionResolution)]
        assert res.default_value == 7.0

    def test_rename_marker_claims_target_before_auto_addition(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/y": ">w",
                                                "/w": "uniform(0, 10, default_value=5)"}))
        ExperimentBranchBuilder(cs)
        names = sorted(repr(r) for r in cs.get_resolutions())
        assert "y~>w" in names
        assert not any(n.startswith("w~+") for n in names)

    def test_rename_with_prior_change_auto_resolves_side_conflict(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/y": ">w",
                                                "/w": "uniform(0, 3)"}))
        b = ExperimentBranchBuilder(cs)
        assert b.is_resolved
        assert any(isinstance(r, C.ChangeDimensionResolution) for r in cs.get_resolutions())

    def test_manual_mode_keeps_only_marked(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 2)", "/y": "-",
                                                "/z": "uniform(0, 1)"}))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True})
        assert one(cs, C.MissingDimensionConflict).is_resolved          # ~- typed
        assert not one(cs, C.NewDimensionConflict).is_resolved          # no ~+
        assert not one(cs, C.ChangedDimensionConflict).is_resolved
        assert not b.is_resolved

    def test_manual_mode_with_flags(self, storage):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B,
                                                           algorithms={"asha": {}}))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True, "algorithm_change": True,
                                         "code_change_type": "unsure"})
        assert b.is_resolved
        assert one(cs, C.CodeConflict).resolution.type == "unsure"

    def test_auto_code_default_break(self, storage):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B))
        ExperimentBranchBuilder(cs)
        assert one(cs, C.CodeConflict).resolution.type == "break"

    def test_branch_flag(self, storage):
        new = cfg(BASE)
        b = ExperimentBranchBuilder(C.detect_conflicts(cfg(BASE), new), {"branch": "kid"})
        assert b.is_resolved and (new["name"], new["version"]) == ("kid", 1)

    def test_auto_resolution_flag_is_accepted(self, storage):
        b = ExperimentBranchBuilder(C.detect_conflicts(cfg(BASE), cfg(BASE)),
                                    {"auto_resolution": True})
        assert b.is_resolved

    def test_experiment_and_conflicting_config(self, storage):
        old, new = cfg(BASE), cfg({**BASE, "/z": "uniform(0, 1)"})
        b = ExperimentBranchBuilder(C.detect_conflicts(old, new))
        assert b.experiment_config is old and b.conflicting_config is new

    def test_none_flags_not_copied(self, storage):
        new = cfg(BASE)
        ExperimentBranchBuilder(C.detect_conflicts(cfg(BASE), new), {"branch": None})
        assert "branch" not in new

    def test_set_code_change_type(self, storage):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A), cfg(BASE, vcs=VCS_B))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True})
        b.set_code_change_type("noeffect")
        assert one(cs, C.CodeConflict).resolution.type == "noeffect"
        with pytest.raises(RuntimeError, match="No CodeConflict"):
            b.set_code_change_type("break")

    def test_set_algo(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg(BASE, algorithms={"asha": {}}))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True})
        b.set_algo()
        assert b.is_resolved
        with pytest.raises(RuntimeError):
            b.set_algo()

    def test_change_experiment_name(self, storage):
        new = cfg(BASE)
        b = ExperimentBranchBuilder(C.detect_conflicts(cfg(BASE), new),
                                    {"manual_resolution": True})
        b.reset("--branch exp")
        b.change_experiment_name("other")
        assert new["name"] == "other"

    def test_add_changed_dimension(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({**BASE, "/x": "uniform(0, 2)"}))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True})
        b.add_dimension("x")
        assert one(cs, C.ChangedDimensionConflict).is_resolved

    def test_add_unknown_dimension(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({**BASE, "/x": "uniform(0, 2)"}))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True})
        with pytest.raises(ValueError):
            b.add_dimension("nope")

    def test_rename_dimension(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)",
                                                "/w": "uniform(0, 10, default_value=5)"}))
        b = ExperimentBranchBuilder(cs, {"manual_resolution": True})
        b.rename_dimension("y", "w")
        assert b.is_resolved
        assert [type(a) for a in b.create_adapters().adapters] == [A.DimensionRenaming]

    def test_reset_then_redo(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)"}))
        b = ExperimentBranchBuilder(cs)
        (text,) = [repr(r) for r in cs.get_resolutions()
                   if isinstance(r, C.RemoveDimensionResolution)]
        b.reset(text)
        assert not b.is_resolved
        b.remove_dimension("y", default_value=2)
        assert b.is_resolved

    def test_create_adapters_round_trip(self, storage):
        cs = C.detect_conflicts(cfg(BASE, vcs=VCS_A),
                                cfg({"/x": "uniform(0, 1)", "/z": "+uniform(0, 1, "
                                     "default_value=0.5)"}, vcs=VCS_B,
                                    algorithms={"asha": {}}, code_change_type="noeffect"))
        b = ExperimentBranchBuilder(cs)
        chain = b.create_adapters()
        again = A.Adapter.build(chain.configuration)
        assert again.configuration == chain.configuration
        kinds_ = {type(a) for a in chain.adapters}
        assert {A.DimensionDeletion, A.DimensionAddition, A.AlgorithmChange,
                A.CodeChange} <= kinds_

    def test_adapter_chain_moves_parent_trials(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/y": "-5",
                                                "/z": "+uniform(0, 1, default_value=0.5)"}))
        chain = ExperimentBranchBuilder(cs).create_adapters()
        moved = chain.forward([trial(x=0.1, y=5.0), trial(x=0.2, y=6.0)])
        assert len(moved) == 1
        assert {p.name: p.value for p in moved[0].params} == {"/x": 0.1, "/z": 0.5}
        back = chain.backward(moved)
        assert {p.name: p.value for p in back[0].params} == {"/x": 0.1, "/y": 5.0}

    def test_unknown_rename_target_is_skipped_when_silenced(self, storage):
        cs = C.detect_conflicts(cfg(BASE), cfg({"/x": "uniform(0, 1)", "/y": ">ghost"}))
        b = ExperimentBranchBuilder(cs)
        assert not one(cs, C.MissingDimensionConflict).is_resolved
        assert not b.is_resolved


# =========================================================================== CLI flags
def test_cli_branching_arguments_come_from_the_resolutions():
    import argparse
    from metaopt_amd.cli.evc import fetch_branching_configuration, get_branching_args_group
    p = argparse.ArgumentParser()
    get_branching_args_group(p)
    ns = vars(p.parse_args(["-b", "kid", "--algorithm-change", "--code-change-type", "unsure",
                            "--cli-change-type", "noeffect", "--config-change-type", "break",
                            "--manual-resolution"]))
    got = fetch_branching_configuration(ns)
    assert got == {"manual_resolution": True, "auto_resolution": False, "branch": "kid",
                   "algorithm_change": True, "code_change_type": "unsure",
                   "cli_change_type": "noeffect", "config_change_type": "break"}
    with pytest.raises(SystemExit):
        p.parse_args(["--code-change-type", "sometimes"])
    assert set(C.FLAGS.values()) == {r.flag for r in C.RESOLUTIONS if r.flag}


def test_experiment_level_branching_chain(storage):
    """Versions and branches through the experiment builder: add, remove, rename and a prior
    change along one lineage; the tree view sees the ancestors' trials through the adapters."""
    from metaopt_amd.io.experiment_builder import build_experiment
    st = storage
    e1 = build_experiment("chain", priors={"/x": "uniform(0, 1)", "/y": "uniform(0, 1)"},
                          storage=st)
    for x, y in ((0.1, 0.5), (0.2, 0.6)):
        e1.register_trial(Trial(experiment=e1.id, status="completed",
                                params=[dict(name="/x", type="real", value=x),
                                        dict(name="/y", type="real", value=y)],
                                results=[dict(name="o", type="objective", value=x)]))
    e2 = build_experiment("chain", priors={"/x": "uniform(0, 1)", "/y": "uniform(0, 1)",
                                           "/z": "+uniform(0, 1, default_value=0.3)"},
                          storage=st)
    assert e2.version == 2 and len(e2.fetch_trials(with_evc_tree=True)) == 2
    e3 = build_experiment("chain", priors={"/x": "uniform(0, 1)", "/y": "-0.5",
                                           "/z": "uniform(0, 1, default_value=0.3)"},
                          user_args=["--x~uniform(0, 1)", "--y~-0.5",
                                     "--z~uniform(0, 1, default_value=0.3)"],
                          storage=st)
    assert e3.version == 3
    tree = e3.fetch_trials(with_evc_tree=True)
    assert len(tree) == 1                       # only y == 0.5 survives the removal
    assert {p.name for p in tree[0].params} == {"/x", "/z"}
    e4 = build_experiment("chain", priors={"/x": "uniform(0, 0.15)",
                                           "/z": "uniform(0, 1, default_value=0.3)"},
                          storage=st, branch="chain-narrow")
    assert e4.name == "chain-narrow" and e4.refers["parent_id"] == e3.id
    assert len(e4.fetch_trials(with_evc_tree=True)) == 1
