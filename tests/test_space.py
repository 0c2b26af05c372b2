"""Search space, prior DSL and transformations (reference tests: tests/unittests/algo/test_space.py,
tests/unittests/core/io/test_space_builder.py, tests/unittests/core/test_transformer.py)."""
import numpy
import pytest

from metaopt_amd.space.builder import DimensionBuilder, SpaceBuilder, build_space, parse_prior
from metaopt_amd.space.dims import Categorical, Fidelity, Integer, Real, Space
from metaopt_amd.space.transformer import (Enumerate, OneHotEncode, Quantize, Reverse,
                                           build_required_space)


class TestDims:
    def test_real_bounds_and_sampling(self):
        dim = Real("yolo", "uniform", -3, 4)  # scipy convention: [-3, 1)
        assert dim.interval() == (-3.0, 1.0)
        samples = dim.sample(500, seed=1)
        assert all(-3 <= s < 1 for s in samples)
        assert 0.5 in dim and 1.0 not in dim and -3.0 in dim

    def test_real_truncation_redraws(self):
        dim = Real("x", "norm", 0, 1, low=-0.5, high=0.5)
        assert dim.interval() == (-0.5, 0.5)
        s = dim.sample(200, seed=2)
        assert all(-0.5 <= v < 0.5 for v in s)

    def test_improbable_bounds_raise(self):
        dim = Real("x", "norm", 0, 1, low=10, high=10.0001)
        with pytest.raises(ValueError, match="Improbable bounds"):
            dim.sample(5, seed=1)

    def test_invalid_bounds(self):
        with pytest.raises(ValueError):
            Real("x", "uniform", 0, 1, low=2, high=1)

    def test_integer(self):
        dim = Integer("i", "uniform", -3, 10)
        s = dim.sample(100, seed=3)
        assert all(isinstance(v, int) and -3 <= v < 7 for v in s)
        assert 3 in dim and 3.5 not in dim and 7 not in dim
        assert dim.cast(["1", "2"]) == [1, 2]

    def test_shaped_dimension(self):
        dim = Real("v", "uniform", 0, 1, shape=(2, 3))
        s = dim.sample(2, seed=0)
        assert s[0].shape == (2, 3)
        assert s[0] in dim
        assert numpy.zeros(3) not in dim

    def test_categorical(self):
        dim = Categorical("c", {"a": 0.1, "b": 0.9, 3: 0.0})
        s = dim.sample(200, seed=4)
        assert set(s) <= {"a", "b"}
        assert "a" in dim and 3 in dim and "z" not in dim
        assert dim.get_prior_string() == "choices({'a': 0.10, 'b': 0.90, 3: 0.00})"
        uni = Categorical("u", ["x", "y"])
        assert uni.get_prior_string() == "choices(['x', 'y'])"
        with pytest.raises(RuntimeError):
            dim.interval()

    def test_default_value_validated(self):
        Real("x", "uniform", 0, 1, default_value=0.5)
        with pytest.raises(ValueError):
            Real("x", "uniform", 0, 1, default_value=2.0)

    def test_seed_forbidden_in_definition(self):
        with pytest.raises(ValueError):
            Real("x", "norm", 0, 1, random_state=1)

    def test_fidelity(self):
        dim = Fidelity("epoch", 1, 16, 4)
        assert dim.sample(3) == [16, 16, 16]
        assert dim.get_prior_string() == "fidelity(1, 16, 4)"
        assert 4 in dim and 17 not in dim
        with pytest.raises(AttributeError):
            Fidelity("e", 0, 2)
        with pytest.raises(AttributeError):
            Fidelity("e", 1, 2, base=1)

    def test_space_sorted_and_contains(self):
        space = Space()
        space.register(Real("zz", "uniform", 0, 1))
        space.register(Categorical("aa", ["x", "y"]))
        space.register(Integer("mm", "uniform", 0, 5))
        assert space.keys() == ["aa", "mm", "zz"]
        assert space[0].name == "aa"
        pts = space.sample(10, seed=5)
        assert all(p in space for p in pts)
        assert ("x", 3, 2.0) not in space
        with pytest.raises(ValueError):
            space.register(Real("zz", "uniform", 0, 1))
        with pytest.raises(TypeError):
            space["k"] = 3

    def test_space_sampling_is_reproducible(self):
        space = build_space({"/x": "uniform(0, 1)", "/y": "loguniform(1e-3, 1)"})
        assert space.sample(5, seed=11) == space.sample(5, seed=11)


class TestBuilder:
    def test_parse_prior_literals_only(self):
        assert parse_prior("uniform(-3, 5, shape=2)") == ("uniform", (-3, 5), {"shape": 2})
        with pytest.raises(RuntimeError):
            parse_prior("uniform(__import__('os'))")
        with pytest.raises(TypeError):
            parse_prior("uniform(open('x'))")

    def test_aliases(self):
        b = DimensionBuilder()
        d = b.build("lr", "loguniform(0.001, 1)")
        assert isinstance(d, Real) and d.prior_name == "reciprocal"
        d = b.build("x", "uniform(-3, 5)")
        assert d.interval() == (-3.0, 5.0)
        d = b.build("i", "uniform(-3, 5, discrete=True)")
        assert isinstance(d, Integer)
        d = b.build("g", "gaussian(0, 1)")
        assert d.prior_name == "norm"
        d = b.build("c", "choices(['a', 'b'])")
        assert isinstance(d, Categorical)
        d = b.build("c2", "choices('a', 'b', 'c')")
        assert d.categories == ("a", "b", "c")
        d = b.build("f", "fidelity(1, 10, base=3)")
        assert isinstance(d, Fidelity) and d.base == 3

    def test_scipy_distributions(self):
        b = DimensionBuilder()
        assert isinstance(b.build("p", "poisson(mu=3)"), Integer)
        assert isinstance(b.build("a", "alpha(3)"), Real)
        with pytest.raises(TypeError):
            b.build("x", "notadistribution(1)")
        with pytest.raises(TypeError):
            b.build("x", "uniform(1, 2, 3, 4, 5)")

    def test_markers(self):
        space = SpaceBuilder().build({"/a": "uniform(0, 1)", "/b": "-uniform(0, 1)",
                                      "/c": ">d", "/d": "+uniform(0, 2)"})
        assert space.keys() == ["/a", "/d"]


class TestTransformer:
    def test_quantize_and_reverse(self):
        q = Quantize()
        assert q.transform(2.7) == 2
        r = Reverse(Quantize())
        assert r.target_type == "real"

    def test_onehot(self):
        oh = OneHotEncode(3)
        t = oh.transform(numpy.array([0, 2]))
        assert t.tolist() == [[1, 0, 0], [0, 0, 1]]
        assert oh.reverse(t).tolist() == [0, 2]
        two = OneHotEncode(2)
        assert float(two.transform(1)) == 1.0 and int(two.reverse(0.7)) == 1

    def test_enumerate(self):
        e = Enumerate(["a", "b", 3])
        assert int(e.transform("b")) == 1
        assert e.reverse(2) == 3

    def test_required_space_real(self):
        space = build_space({"/c": "choices(['x', 'y', 'z'])", "/i": "uniform(0, 10, discrete=True)",
                             "/r": "uniform(0, 1)", "/f": "fidelity(1, 4)"})
        ts = build_required_space("real", space)
        assert [d.type for d in ts.values()] == ["real", "fidelity", "real", "real"]
        pt = ("y", 4, 3, 0.5)
        tpt = ts.transform(pt)
        assert tpt in ts
        back = ts.reverse(tpt)
        assert back[0] == "y" and int(back[2]) == 3

    def test_required_space_integer(self):
        space = build_space({"/r": "uniform(0, 10)", "/c": "choices(['x', 'y'])"})
        ts = build_required_space("integer", space)
        assert [d.type for d in ts.values()] == ["integer", "integer"]
