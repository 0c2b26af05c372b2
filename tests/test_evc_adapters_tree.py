"""EVC adapters (forward / backward trial filtering and rewriting, construction errors,
serialisation) and the generic tree (parent / children links, traversals, map).  Behaviour
parity with the reference's tests/unittests/core/evc/test_adapters.py and test_tree.py,
written against this package's API."""
import pytest

from metaopt_amd.core.trial import Param, Trial
from metaopt_amd.evc.adapters import (Adapter, AlgorithmChange, CodeChange, CommandLineChange,
                                      CompositeAdapter, DimensionAddition, DimensionDeletion,
                                      DimensionPriorChange, DimensionRenaming, ScriptConfigChange)
from metaopt_amd.evc.tree import DepthFirstTraversal, PreOrderTraversal, TreeNode


def trial(**params):
    return Trial(params=[dict(name=f"/{k}", type="real", value=v)
                         for k, v in sorted(params.items())])


def names(t):
    return [p.name for p in t.params]


def value(t, name):
    return next(p.value for p in t.params if p.name == name)


DEFAULT = dict(name="/d", type="real", value=1.0)


@pytest.fixture
def trials():
    return [trial(x=0.1 * i, y=float(i)) for i in range(6)]


# ------------------------------------------------------------------------ construction
class TestConstruction:
    def test_addition_from_param_or_dict(self):
        a = DimensionAddition(Param(**DEFAULT))
        b = DimensionAddition(DEFAULT)
        assert a.param.to_dict() == b.param.to_dict()

    @pytest.mark.parametrize("bad", [1, "d", [DEFAULT]])
    def test_addition_rejects_non_params(self, bad):
        with pytest.raises(TypeError, match="Param"):
            DimensionAddition(bad)

    def test_deletion_wraps_an_addition(self):
        d = DimensionDeletion(DEFAULT)
        assert d.param.name == "/d" and d.param.value == 1.0

    def test_prior_change_requires_same_shape(self):
        DimensionPriorChange("/x", "uniform(0, 1)", "uniform(0, 10)")
        with pytest.raises(NotImplementedError, match="shape"):
            DimensionPriorChange("/x", "uniform(0, 1)", "uniform(0, 1, shape=2)")

    @pytest.mark.parametrize("bad", [(1, "/y"), ("/x", None)])
    def test_renaming_needs_string_names(self, bad):
        with pytest.raises(TypeError, match="strings"):
            DimensionRenaming(*bad)

    @pytest.mark.parametrize("cls", [CodeChange, CommandLineChange, ScriptConfigChange])
    def test_change_type_validated(self, cls):
        for ok in ("noeffect", "break", "unsure"):
            assert cls(ok).change_type == ok
        with pytest.raises(ValueError, match="change type"):
            cls("sometimes")

    def test_composite_accepts_only_adapters(self):
        assert CompositeAdapter().adapters == ()
        CompositeAdapter(AlgorithmChange(), CodeChange("noeffect"))
        with pytest.raises(TypeError, match="adapter objects"):
            CompositeAdapter(AlgorithmChange(), "code")

    def test_factory_by_type_name(self):
        a = Adapter(of_type="DimensionRenaming", old_name="/x", new_name="/z")
        assert isinstance(a, DimensionRenaming)
        with pytest.raises(NotImplementedError, match="BaseAdapter"):
            Adapter(of_type="teleportation")


# ------------------------------------------------------------------------ forward / backward
class TestDimensionAdditionDeletion:
    def test_addition_forward_adds_default(self, trials):
        out = DimensionAddition(DEFAULT).forward(trials)
        assert len(out) == len(trials)
        assert all(names(t) == ["/d", "/x", "/y"] and value(t, "/d") == 1.0 for t in out)
        assert all(names(t) == ["/x", "/y"] for t in trials)     # inputs untouched

    def test_addition_forward_refuses_existing_dimension(self, trials):
        with pytest.raises(RuntimeError, match="already present"):
            DimensionAddition(dict(name="/x", type="real", value=0.0)).forward(trials)

    def test_addition_backward_keeps_only_default_trials(self, trials):
        child = DimensionAddition(DEFAULT).forward(trials)
        child[0].params[0].value = 2.0                     # one child trial left the default
        back = DimensionAddition(DEFAULT).backward(child)
        assert len(back) == len(trials) - 1
        assert all(names(t) == ["/x", "/y"] for t in back)

    def test_addition_backward_needs_the_dimension(self, trials):
        with pytest.raises(RuntimeError, match="should be present"):
            DimensionAddition(DEFAULT).backward(trials)

    def test_deletion_is_addition_reversed(self, trials):
        with_d = DimensionAddition(DEFAULT).forward(trials)
        fwd = DimensionDeletion(DEFAULT).forward(with_d)
        assert [names(t) for t in fwd] == [names(t) for t in trials]
        back = DimensionDeletion(DEFAULT).backward(trials)
        assert all("/d" in names(t) for t in back)
        with pytest.raises(RuntimeError):
            DimensionDeletion(DEFAULT).forward(trials)        # nothing to delete


class TestPriorChangeAndRenaming:
    def test_prior_change_filters_by_new_and_old_priors(self, trials):
        shrink = DimensionPriorChange("/x", "uniform(0, 1)", "uniform(0, 0.25)")
        fwd = shrink.forward(trials)
        assert sorted(value(t, "/x") for t in fwd) == pytest.approx([0.0, 0.1, 0.2])
        assert len(shrink.backward(trials)) == len(trials)    # all inside the old prior

    def test_prior_change_needs_the_dimension(self, trials):
        with pytest.raises(RuntimeError):
            DimensionPriorChange("/z", "uniform(0, 1)", "uniform(0, 2)").forward(trials)

    def test_renaming_round_trip(self, trials):
        r = DimensionRenaming("/x", "/a")
        fwd = r.forward(trials)
        assert all(names(t) == ["/a", "/y"] for t in fwd)       # params stay sorted
        back = r.backward(fwd)
        assert [value(t, "/x") for t in back] == [value(t, "/x") for t in trials]

    def test_renaming_missing_dimension(self, trials):
        with pytest.raises(RuntimeError):
            DimensionRenaming("/q", "/a").forward(trials)
        with pytest.raises(RuntimeError):
            DimensionRenaming("/x", "/a").backward(trials)   # child trials would carry /a


class TestChangeTypes:
    def test_algorithm_change_passes_everything(self, trials):
        a = AlgorithmChange()
        assert a.forward(trials) == trials and a.backward(trials) == trials

    @pytest.mark.parametrize("cls", [CodeChange, CommandLineChange, ScriptConfigChange])
    @pytest.mark.parametrize("kind,fwd,bwd", [("noeffect", True, True), ("unsure", True, False),
                                              ("break", False, False)])
    def test_change_semantics(self, trials, cls, kind, fwd, bwd):
        a = cls(kind)
        assert (a.forward(trials) == trials) is fwd
        assert (a.backward(trials) == trials) is bwd
        assert a.forward(trials) in (trials, [])


class TestComposite:
    def test_empty_composite_is_identity(self, trials):
        c = CompositeAdapter()
        assert c.forward(trials) == trials and c.backward(trials) == trials

    def test_forward_in_order_backward_reversed(self, trials):
        c = CompositeAdapter(DimensionAddition(DEFAULT), DimensionRenaming("/d", "/e"))
        fwd = c.forward(trials)
        assert all(names(t) == ["/e", "/x", "/y"] for t in fwd)
        back = c.backward(fwd)             # rename /e -> /d first, then drop the default
        assert [names(t) for t in back] == [names(t) for t in trials]

    def test_break_in_chain_empties(self, trials):
        c = CompositeAdapter(DimensionAddition(DEFAULT), CodeChange("break"))
        assert c.forward(trials) == []


# ------------------------------------------------------------------------ serialisation
@pytest.mark.parametrize("adapter", [
    DimensionAddition(DEFAULT), DimensionDeletion(DEFAULT),
    DimensionPriorChange("/x", "uniform(0, 1)", "uniform(0, 2)"),
    DimensionRenaming("/x", "/z"), AlgorithmChange(), CodeChange("unsure"),
    CommandLineChange("noeffect"), ScriptConfigChange("break")])
def test_configuration_round_trips(adapter):
    cfg = adapter.configuration
    assert isinstance(cfg, list) and len(cfg) == 1
    rebuilt = Adapter.build(cfg)
    assert isinstance(rebuilt, CompositeAdapter) and rebuilt.adapters[0] == adapter
    assert rebuilt.configuration == cfg


def test_composite_configuration_flattens_singletons():
    c = CompositeAdapter(DimensionAddition(DEFAULT), AlgorithmChange())
    cfg = c.configuration
    assert [d["of_type"] for d in cfg] == ["dimensionaddition", "algorithmchange"]
    assert Adapter.build(cfg).configuration == cfg
    assert CompositeAdapter(AlgorithmChange()).configuration == [{"of_type": "algorithmchange"}]
    assert CompositeAdapter().configuration == []


# ------------------------------------------------------------------------ tree
def chain():
    """a -> (b -> (d, e), c)"""
    a = TreeNode("a")
    b = TreeNode("b", a)
    c = TreeNode("c", a)
    d = TreeNode("d", b)
    e = TreeNode("e", b)
    return a, b, c, d, e


class TestTree:
    def test_creation_and_links(self):
        a, b, c, d, e = chain()
        assert a.parent is None and b.parent is a and d.parent is b
        assert [n.item for n in a.children] == ["b", "c"]
        assert d.root is a and a.root is a

    def test_set_parent_moves_node(self):
        a, b, c, d, e = chain()
        d.set_parent(c)
        assert d.parent is c and d in c.children and d not in b.children

    def test_drop_parent(self):
        a, b, c, d, e = chain()
        b.drop_parent()
        assert b.parent is None and b not in a.children
        assert d.root is b

    def test_add_and_drop_children(self):
        a, b, c, d, e = chain()
        f, g = TreeNode("f"), TreeNode("g")
        c.add_children(f, g)
        assert f.parent is c and [n.item for n in c.children] == ["f", "g"]
        c.drop_children(f)
        assert f.parent is None and [n.item for n in c.children] == ["g"]
        b.drop_children()
        assert b.children == [] and d.parent is None and e.parent is None

    def test_reinsertion_keeps_single_link(self):
        a, b, c, d, e = chain()
        d.set_parent(b)                    # already its parent
        assert [n.item for n in b.children].count("d") == 1
        b.add_children(d)
        assert [n.item for n in b.children].count("d") == 1

    def test_traversals(self):
        a, *_ = chain()
        assert [n.item for n in PreOrderTraversal(a)] == ["a", "b", "d", "e", "c"]
        assert [n.item for n in DepthFirstTraversal(a)] == ["d", "e", "b", "c", "a"]
        assert [n.item for n in a] == ["a", "b", "d", "e", "c"]

    def test_map_builds_a_new_tree_of_the_same_shape(self):
        a, b, c, d, e = chain()
        up = a.map(lambda node: node.item.upper())
        assert [n.item for n in PreOrderTraversal(up)] == ["A", "B", "D", "E", "C"]
        assert [n.item for n in PreOrderTraversal(a)] == ["a", "b", "d", "e", "c"]  # untouched
        sub = b.map(lambda node: len(node.children))
        assert sub.parent is None and [n.item for n in sub] == [2, 0, 0]

    def test_children_must_be_nodes(self):
        with pytest.raises(TypeError, match="TreeNode"):
            TreeNode("a").add_children("b")
