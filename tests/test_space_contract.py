"""Behaviour contract of the search-space dimensions, spaces and transformers (what the
reference pins in tests/unittests/algo/test_space.py and tests/unittests/core/test_transformer.py:
random-state handling, bounds and containment, casting, defaults, priors' string forms, sampling
reproducibility, the transformer algebra and required-space building) -- written against this
package's API; expected values are this implementation's documented semantics."""
import numpy as np
import pytest

from metaopt_amd.space.dims import (Categorical, Fidelity, Integer, Real, Space,
                                    check_random_state)
from metaopt_amd.space.transformer import (Compose, Enumerate, Identity, OneHotEncode, Quantize,
                                           Reverse, TransformedDimension, TransformedSpace,
                                           build_required_space)


# ------------------------------------------------------------------ random state
class TestRandomState:
    def test_none_gives_a_fresh_state(self):
        assert isinstance(check_random_state(None), np.random.RandomState)

    def test_state_is_passed_through(self):
        rs = np.random.RandomState(3)
        assert check_random_state(rs) is rs

    def test_int_and_tuple_seed_reproducible(self):
        for seed in (7, (1, 2, 3)):
            a, b = check_random_state(seed), check_random_state(seed)
            assert a.randint(1 << 30) == b.randint(1 << 30)

    def test_invalid_seed(self):
        with pytest.raises(ValueError, match="cannot be used to seed"):
            check_random_state("seed")


# ------------------------------------------------------------------ Real
class TestReal:
    def test_uniform_is_loc_scale(self):
        d = Real("x", "uniform", -1, 2)
        lo, hi = d.interval()
        assert (float(lo), float(hi)) == (-1.0, 1.0)
        assert d.type == "real" and d.prior_name == "uniform" and d.shape == ()

    def test_contains_is_half_open(self):
        d = Real("x", "uniform", -1, 2)
        assert -1 in d and 0.999 in d
        assert 1.0 not in d and 1.5 not in d and -1.01 not in d

    def test_samples_are_inside_and_reproducible(self):
        d = Real("x", "uniform", -1, 2)
        a, b = d.sample(50, seed=4), d.sample(50, seed=4)
        assert a == b and all(v in d for v in a)
        assert d.sample(5, seed=5) != a[:5]

    def test_extra_bounds_truncate_the_prior(self):
        d = Real("x", "norm", 0, 1, low=-0.5, high=0.5)
        assert d.interval() == (-0.5, 0.5)
        assert all(-0.5 <= v <= 0.5 for v in d.sample(200, seed=1))
        assert 0.7 not in d

    def test_bad_bounds(self):
        with pytest.raises(ValueError, match="Lower bound"):
            Real("x", "uniform", 0, 1, low=0.5, high=0.2)

    @pytest.mark.parametrize("kw", ["size", "seed", "random_state"])
    def test_banned_keywords(self, kw):
        with pytest.raises(ValueError):
            Real("x", "norm", 0, 1, **{kw: 3})

    def test_default_value(self):
        assert Real("x", "uniform", 0, 1, default_value=0.5).default_value == 0.5
        assert Real("x", "uniform", 0, 1).default_value is None
        with pytest.raises(ValueError, match="Can't set default value"):
            Real("x", "uniform", 0, 1, default_value=3)

    def test_cast(self):
        d = Real("x", "uniform", 0, 2)
        assert d.cast(["0.5", 1]) == [0.5, 1.0]
        assert d.cast("1.25") == 1.25
        got = d.cast(np.array([1, 2]))
        assert list(np.asarray(got, dtype=float)) == [1.0, 2.0]

    def test_shaped_dimension(self):
        d = Real("y", "norm", 0, 1, shape=(2, 3))
        assert d.shape == (2, 3)
        assert np.asarray(d.sample(1, seed=1)[0]).shape == (2, 3)
        assert np.zeros((2, 3)) in d and np.zeros((3, 2)) not in d

    def test_string_forms(self):
        d = Real("lr", "loguniform", 1e-3, 1.0)
        assert d.get_prior_string() == "loguniform(0.001, 1.0)"
        assert d.get_string() == "lr~loguniform(0.001, 1.0)"
        assert "Real(name=lr" in repr(d)

    def test_loguniform_samples_spread_over_decades(self):
        d = Real("lr", "loguniform", 1e-4, 1.0)
        s = np.log10(d.sample(2000, seed=2))
        assert -4 <= s.min() and s.max() < 0
        counts = np.histogram(s, bins=4, range=(-4, 0))[0]
        assert counts.min() > 350            # ~500 per decade

    def test_equality_and_hash(self):
        a, b = Real("x", "uniform", 0, 1), Real("x", "uniform", 0, 1)
        assert a == b and hash(a) == hash(b)
        assert a != Real("x", "uniform", 0, 2) and a != Real("z", "uniform", 0, 1)

    def test_rename(self):
        d = Real("x", "uniform", 0, 1)
        d.name = "y"
        assert d.name == "y"
        with pytest.raises(TypeError):
            d.name = 3


# ------------------------------------------------------------------ Integer
class TestInteger:
    def test_interval_and_cardinality(self):
        d = Integer("i", "uniform", -3, 6)
        assert d.interval() == (-3, 3)
        assert d.type == "integer" and d.cardinality == 6

    def test_contains_integers_only(self):
        d = Integer("i", "uniform", -3, 6)
        assert 2 in d and -3 in d
        assert 2.5 not in d and 10 not in d

    def test_samples_are_ints(self):
        d = Integer("i", "uniform", 0, 10)
        s = d.sample(100, seed=3)
        assert all(isinstance(v, (int, np.integer)) for v in s)
        assert all(0 <= v <= 10 for v in s)

    def test_cast_rounds_down(self):
        d = Integer("i", "uniform", 0, 10)
        assert d.cast("3") == 3 and d.cast([1.7, 2.2]) == [1, 2]

    def test_discrete_keyword_is_for_the_builder(self):
        from metaopt_amd.space.builder import DimensionBuilder
        with pytest.raises(ValueError, match="discrete"):
            Real("w", "loguniform", 64, 1024, discrete=True)
        d = DimensionBuilder().build("w", "loguniform(64, 1024, discrete=True)")
        assert d.type == "integer"
        s = d.sample(300, seed=5)
        assert all(64 <= v <= 1024 and int(v) == v for v in s)

    def test_default_value(self):
        assert Integer("i", "uniform", 0, 10, default_value=4).default_value == 4
        with pytest.raises(ValueError):
            Integer("i", "uniform", 0, 10, default_value=40)

    def test_string(self):
        assert Integer("i", "uniform", -3, 6).get_prior_string() == "uniform(-3, 6)"
        assert Integer("i", "uniform", -3, 6).get_string() == "i~uniform(-3, 6)"


# ------------------------------------------------------------------ Categorical
class TestCategorical:
    def test_tuple_categories_are_uniform(self):
        d = Categorical("c", ("a", "b", 3))
        assert d.probabilities == pytest.approx((1 / 3,) * 3)
        assert d.cardinality == 3 and d.type == "categorical"

    def test_dict_probabilities(self):
        d = Categorical("c", {"x": 0.2, "y": 0.8})
        assert d.probabilities == (0.2, 0.8)
        s = d.sample(2000, seed=1)
        assert 0.74 < s.count("y") / 2000 < 0.86

    def test_contains_and_sample(self):
        d = Categorical("c", ("a", "b", 3))
        assert "a" in d and 3 in d and "z" not in d
        assert set(d.sample(60, seed=2)) <= {"a", "b", 3}

    def test_prior_strings(self):
        assert Categorical("c", ("a", "b", 3)).get_prior_string() == "choices(['a', 'b', 3])"
        assert Categorical("c", {"x": 0.2, "y": 0.8}).get_prior_string() == \
            "choices({'x': 0.20, 'y': 0.80})"

    def test_cast(self):
        d = Categorical("c", ("a", "b", 3))
        assert d.cast("a") == "a"
        with pytest.raises(ValueError, match="Invalid category"):
            d.cast("zz")

    def test_default_value(self):
        assert Categorical("c", ("a", "b"), default_value="b").default_value == "b"
        with pytest.raises(ValueError):
            Categorical("c", ("a", "b"), default_value="q")

    def test_mixed_object_types(self):
        d = Categorical("c", (None, "s", 1.5, True))
        assert None in d and 1.5 in d and "s" in d

    def test_bad_probabilities(self):
        with pytest.raises(ValueError):
            Categorical("c", {"a": 0.3, "b": 0.3})

    def test_no_categories(self):
        with pytest.raises(ValueError):
            Categorical("c", ())


# ------------------------------------------------------------------ Fidelity
class TestFidelity:
    def test_basic(self):
        f = Fidelity("epoch", 1, 16, base=4)
        assert f.interval() == (1, 16) and f.type == "fidelity"
        assert f.get_prior_string() == "fidelity(1, 16, 4)"

    def test_samples_and_default_are_the_maximum(self):
        f = Fidelity("epoch", 1, 16, base=4)
        assert f.sample(3) == [16, 16, 16] and f.default_value == 16

    def test_contains(self):
        f = Fidelity("epoch", 1, 16, base=4)
        assert 1 in f and 4 in f and 16 in f and 32 not in f and 0 not in f

    def test_cast(self):
        assert Fidelity("epoch", 1, 16).cast(3) == 3

    def test_bad_range(self):
        with pytest.raises(AttributeError):
            Fidelity("epoch", 0, 16)
        with pytest.raises(AttributeError):
            Fidelity("epoch", 8, 4)


# ------------------------------------------------------------------ Space
def _space():
    s = Space()
    s.register(Real("x", "uniform", -1, 2))
    s.register(Integer("i", "uniform", -3, 6))
    s.register(Categorical("c", ("a", "b", 3)))
    return s


class TestSpace:
    def test_keys_are_sorted(self):
        s = _space()
        assert s.keys() == ["c", "i", "x"]
        assert [d.name for d in s.values()] == ["c", "i", "x"]

    def test_sample_reproducible_and_contained(self):
        s = _space()
        a, b = s.sample(10, seed=3), s.sample(10, seed=3)
        assert a == b and all(p in s for p in a)

    def test_contains_names_and_points(self):
        s = _space()
        assert "x" in s and "nope" not in s
        assert ("a", 0, 0.5) in s and ("q", 0, 0.5) not in s and ("a", 0) not in s

    def test_interval(self):
        assert _space().interval()[0] == ("a", "b", 3)

    def test_getitem_by_name_and_index(self):
        s = _space()
        assert s["x"].name == "x" and s[0].name == "c"

    def test_bad_setitem(self):
        s = _space()
        with pytest.raises((TypeError, ValueError)):
            s["y"] = 5
        with pytest.raises(ValueError):
            s["x"] = Real("x", "uniform", 0, 1)       # already registered

    def test_repr_lists_dimensions(self):
        assert "Space([Categorical(name=c" in repr(_space())


# ------------------------------------------------------------------ transformers
class TestTransformers:
    def test_identity(self):
        t = Identity("real")
        assert t.transform(5) == 5 and t.reverse(5) == 5
        assert t.domain_type == t.target_type == "real"

    def test_quantize_floors(self):
        t = Quantize()
        assert (t.domain_type, t.target_type) == ("real", "integer")
        assert t.transform(2.6) == 2 and t.reverse(3) == 3.0
        assert t.repr_format("x") == "Quantize(x)"

    def test_reverse_swaps_types_and_directions(self):
        t = Reverse(Quantize())
        assert (t.domain_type, t.target_type) == ("integer", "real")
        assert t.transform(3) == 3.0 and t.reverse(2.7) == 2

    def test_enumerate(self):
        t = Enumerate(["a", "b", 3])
        assert (t.domain_type, t.target_type) == ("categorical", "integer")
        assert t.transform("b") == 1 and list(t.transform(["a", 3])) == [0, 2]
        assert t.reverse(2) == 3 and list(t.reverse(np.array([0, 1]))) == ["a", "b"]

    def test_onehot(self):
        t = OneHotEncode(3)
        assert list(t.transform(2)) == [0, 0, 1]
        assert t.transform(np.array([0, 1])).tolist() == [[1, 0, 0], [0, 1, 0]]
        assert t.reverse(np.array([0.1, 0.7, 0.2])) == 1
        assert t.infer_target_shape(()) == (3,)

    def test_onehot_of_two_categories_is_a_scalar(self):
        t = OneHotEncode(2)
        assert t.transform(1) == 1.0 and t.infer_target_shape(()) == ()
        assert t.reverse(0.7) == 1 and t.reverse(0.3) == 0

    def test_compose(self):
        t = Compose([Enumerate(["a", "b", "c"]), OneHotEncode(3)], "categorical")
        assert list(t.transform("b")) == [0, 1, 0]
        assert t.reverse(np.array([0, 0, 1])) == "c"
        assert (t.domain_type, t.target_type) == ("categorical", "real")
        assert t.infer_target_shape(()) == (3,)

    def test_equality(self):
        assert Quantize() == Quantize() and hash(Quantize()) == hash(Quantize())
        assert Quantize() != Identity()

    def test_roundtrip_over_samples(self):
        dim = Categorical("c", ("a", "b", "c", "d"))
        t = Compose([Enumerate(list(dim.categories)), OneHotEncode(4)], "categorical")
        for v in dim.sample(30, seed=8):
            assert t.reverse(t.transform(v)) == v


class TestTransformedDimension:
    def test_onehot_categorical(self):
        td = TransformedDimension(Compose([Enumerate(["a", "b", "c"]), OneHotEncode(3)],
                                          "categorical"), Categorical("c", ("a", "b", "c")))
        assert td.type == "real" and td.shape == (3,) and td.name == "c"
        assert np.array([0, 1, 0]) in td
        assert td.get_prior_string() == "OneHotEncode(Enumerate(choices(['a', 'b', 'c'])))"

    def test_integer_as_real(self):
        td = TransformedDimension(Reverse(Quantize()), Integer("n", "uniform", 0, 5))
        assert td.type == "real" and 2.5 in td and td.reverse(2.6) == 2

    def test_attribute_passthrough(self):
        td = TransformedDimension(Identity("real"), Real("x", "uniform", 0, 1))
        assert td.prior_name == "uniform"


class TestRequiredSpace:
    def test_real_requirement(self):
        s = build_required_space("real", _space())
        assert isinstance(s, TransformedSpace)
        types = {d.name: d.type for d in s.values()}
        assert types == {"c": "real", "i": "real", "x": "real"}

    def test_integer_requirement(self):
        s = build_required_space("integer", _space())
        assert {d.name: d.type for d in s.values()} == {"c": "integer", "i": "integer",
                                                       "x": "integer"}

    def test_none_keeps_types(self):
        s = build_required_space(None, _space())
        assert {d.name: d.type for d in s.values()} == {"c": "categorical", "i": "integer",
                                                       "x": "real"}

    def test_roundtrip_points(self):
        orig = _space()
        s = build_required_space("real", orig)
        for p in orig.sample(20, seed=9):
            back = s.reverse(s.transform(p))
            assert back[0] == p[0] and back[1] == p[1]
            assert back[2] == pytest.approx(p[2])

    def test_fidelity_untouched(self):
        orig = Space()
        orig.register(Fidelity("epoch", 1, 16))
        orig.register(Real("x", "uniform", 0, 1))
        s = build_required_space("integer", orig)
        assert {d.name: d.type for d in s.values()} == {"epoch": "fidelity", "x": "integer"}

    def test_unsupported_requirement(self):
        with pytest.raises(TypeError):
            build_required_space("complex", _space())
