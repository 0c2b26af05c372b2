"""Algorithms, primary wrapper, parallel strategies and plugin discovery (reference tests:
tests/unittests/algo/test_asha.py, test_random.py, core/test_primary_algo.py, core/test_strategy.py,
tests/functional/gradient_descent_algo)."""
import os
import sys

import numpy as np
import pytest

from metaopt_amd.algo.asha import ASHA, Bracket
from metaopt_amd.algo.base import ALGORITHMS, BaseAlgorithm, create_algo
from metaopt_amd.algo.primary import PrimaryAlgo
from metaopt_amd.core.trial import Trial
from metaopt_amd.space.builder import build_space
from metaopt_amd.worker.strategy import (MaxParallelStrategy, MeanParallelStrategy,
                                         NoParallelStrategy, StubParallelStrategy,
                                         create_strategy)


@pytest.fixture
def space():
    return build_space({"/lr": "loguniform(1e-4, 1)", "/units": "uniform(8, 64, discrete=True)",
                        "/epoch": "fidelity(1, 9, 3)"})


def quad(x):
    return (x - 34.56789) ** 2 + 23.4


class TestRandom:
    def test_seeded_reproducible(self, space):
        a, b = create_algo(space, {"random": {"seed": 5}}), create_algo(space, {"random": {"seed": 5}})
        assert a.suggest(4) == b.suggest(4)

    def test_state_dict_roundtrip(self, space):
        a = create_algo(space, {"random": {"seed": 5}})
        st = a.state_dict
        first = a.suggest(2)
        a.set_state(st)
        assert a.suggest(2) == first

    def test_configuration(self, space):
        assert create_algo(space, "random").configuration == {"random": {"seed": None}}


class TestASHA:
    def test_requires_fidelity(self):
        with pytest.raises(RuntimeError):
            ASHA(build_space({"/x": "uniform(0, 1)"}))

    def test_budgets(self, space):
        a = ASHA(space, seed=1)
        assert a.budgets == [1, 3, 9]
        assert a.num_rungs == 3

    def test_promotion_of_best(self, space):
        a = ASHA(space, seed=1)
        pts = a.suggest(9)
        assert all(p[0] == 1 for p in pts)
        objs = list(range(9))
        a.observe(pts, [{"objective": float(o)} for o in objs])
        promo = a.suggest(1)[0]
        # the best point (objective 0) is promoted to budget 3 with same hyper-parameters
        assert promo[0] == 3 and promo[1:] == pts[0][1:]

    def test_num_gt_one_never_promotes_twice(self, space):
        a = ASHA(space, seed=2)
        pts = a.suggest(9)
        a.observe(pts, [{"objective": float(i)} for i in range(9)])
        more = a.suggest(20)
        promoted = [p for p in more if p[0] == 3]
        assert len(promoted) == len({p[1:] for p in promoted}) == 3

    def test_opt_out_when_filled(self, space):
        a = ASHA(space, seed=3)
        pts = a.suggest(9)
        a.observe(pts, [{"objective": float(i)} for i in range(9)])
        a.suggest(3)                        # 3 promotions to rung 1 -> bracket filled
        assert a.suggest(1) is None         # waiting for rung 1 results

    def test_done_after_top_rung_completes(self, space):
        a = ASHA(space, seed=4)
        pts = a.suggest(9)
        a.observe(pts, [{"objective": float(i)} for i in range(9)])
        r1 = a.suggest(3)
        a.observe(r1, [{"objective": float(i)} for i in range(3)])
        top = a.suggest(1)
        assert top[0][0] == 9 and not a.is_done
        a.observe(top, [{"objective": 0.0}])
        assert a.is_done

    def test_repetitions_keep_sampling(self, space):
        a = ASHA(space, seed=5, repetitions=float("inf"))
        pts = a.suggest(9)
        a.observe(pts, [{"objective": float(i)} for i in range(9)])
        a.suggest(3)
        more = a.suggest(5)
        assert more is not None and len(more) == 5 and len(a.brackets) == 2

    def test_bracket_candidate_respects_k(self, space):
        a = ASHA(space, seed=6)
        b = a.brackets[0]
        pts = a.space.sample(5, seed=1)
        for i, p in enumerate(pts):
            p = list(p)
            p[0] = 1
            b.register(tuple(p), float(i))
        # 5 // 3 = 1 candidate: only the best
        cand = b.get_candidate(0)
        assert cand is not None and b.get_candidate(0) == cand

    def test_full_state_roundtrip(self, space):
        a = ASHA(space, seed=7)
        pts = a.suggest(9)
        a.observe(pts, [{"objective": float(i)} for i in range(9)])
        st = a.full_state()
        b = ASHA(space, seed=0)
        b.set_state(st)
        assert b.suggest(1) == a.suggest(1)


class TestTPE:
    def test_beats_random_on_quadratic(self):
        space = build_space({"/x": "uniform(-50, 50)"})
        tpe = create_algo(space, {"tpe": {"seed": 1, "n_initial_points": 10}})
        best = np.inf
        for _ in range(60):
            (p,) = tpe.suggest(1)
            y = quad(p[0])
            best = min(best, y)
            tpe.observe([p], [{"objective": y}])
        assert best < 23.4 + 1.0

    def test_batch_suggest_is_diverse_and_in_space(self):
        space = build_space({"/x": "uniform(0, 1)", "/c": "choices(['a', 'b', 'c'])",
                             "/i": "loguniform(1, 100, discrete=True)"})
        tpe = create_algo(space, {"tpe": {"seed": 2, "n_initial_points": 5}})
        pts = tpe.suggest(5)
        tpe.observe(pts, [{"objective": float(i)} for i in range(5)])
        batch = tpe.suggest(16)
        assert all(p in space for p in batch)
        assert len({round(p[2], 6) for p in batch}) > 8


class TestPrimaryAndPlugins:
    def test_primary_transforms_for_real_algorithms(self):
        space = build_space({"/c": "choices(['x', 'y', 'z'])", "/n": "uniform(0, 5, discrete=True)"})
        primary = PrimaryAlgo(space, {"gradient_descent": {"learning_rate": 0.1}})
        assert all(d.type == "real" for d in primary.transformed_space.values())
        (p,) = primary.suggest(1)
        assert p in space

    def test_gradient_descent_converges(self):
        space = build_space({"/x": "uniform(-50, 50)"})
        gd = PrimaryAlgo(space, {"gradient_descent": {"learning_rate": 0.1}})
        for _ in range(200):
            (p,) = gd.suggest(1)
            x = float(p[0])
            gd.observe([p], [{"objective": quad(x), "gradient": [2 * (x - 34.56789)],
                              "constraint": []}])
            if gd.is_done:
                break
        assert abs(x - 34.56789) < 1e-3

    def test_nested_algorithm_kwargs(self):
        space = build_space({"/x": "uniform(0, 1)"})

        class Meta(BaseAlgorithm):
            def __init__(self, space, inner="random", seed=None):
                super().__init__(space, inner=inner, seed=seed)

            def suggest(self, num=1):
                return self.inner.suggest(num)

            def observe(self, points, results):
                pass

        m = Meta(space, inner={"random": {"seed": 3}})
        assert m.configuration == {"meta": {"inner": {"random": {"seed": 3}}, "seed": None}}

    def test_entry_point_plugin_discovery(self, tmp_path, monkeypatch):
        """An external package registered through the `OptimizationAlgorithm` entry-point group
        (the reference's plugin mechanism) is discovered by name."""
        pkg = tmp_path / "myplugin"
        pkg.mkdir()
        (pkg / "__init__.py").write_text(
            "from metaopt_amd.algo.base import BaseAlgorithm\n"
            "class Constant(BaseAlgorithm):\n"
            "    def __init__(self, space, value=0.5):\n"
            "        super().__init__(space, value=value)\n"
            "    def suggest(self, num=1):\n"
            "        return [(self.value,)] * num\n"
            "    def observe(self, points, results):\n"
            "        pass\n")
        dist = tmp_path / "myplugin-0.1.dist-info"
        dist.mkdir()
        (dist / "METADATA").write_text("Metadata-Version: 2.1\nName: myplugin\nVersion: 0.1\n")
        (dist / "entry_points.txt").write_text(
            "[OptimizationAlgorithm]\nconstant = myplugin:Constant\n")
        monkeypatch.syspath_prepend(str(tmp_path))
        ALGORITHMS._loaded = False
        try:
            algo = create_algo(build_space({"/x": "uniform(0, 1)"}), {"constant": {"value": 0.25}})
            assert algo.suggest(2) == [(0.25,), (0.25,)]
        finally:
            ALGORITHMS._types.pop("constant", None)
            ALGORITHMS._loaded = False


class TestStrategies:
    def _trial(self):
        return Trial(experiment="e", params=[dict(name="/x", type="real", value=1.0)])

    def test_max_and_mean(self):
        mx, mean = MaxParallelStrategy(), MeanParallelStrategy()
        res = [{"objective": 1.0}, {"objective": 5.0}, {"objective": None}]
        for s in (mx, mean):
            s.observe([None] * 3, res)
        assert mx.lie(self._trial()).value == 5.0
        assert mean.lie(self._trial()).value == 3.0

    def test_defaults_and_stub(self):
        assert MaxParallelStrategy().lie(self._trial()).value == float("inf")
        assert NoParallelStrategy().lie(self._trial()) is None
        stub = create_strategy({"StubParallelStrategy": {"stub_value": 2}})
        assert isinstance(stub, StubParallelStrategy) and stub.lie(self._trial()).value == 2

    def test_lie_on_completed_raises(self):
        t = self._trial()
        t.results = [Trial.Result(name="o", type="objective", value=1.0)]
        with pytest.raises(RuntimeError):
            MaxParallelStrategy().lie(t)
