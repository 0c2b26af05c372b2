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


class TestPBT:
    def _space(self):
        return build_space({"/lr": "loguniform(1e-4, 1)", "/width": "choices([64, 128])",
                            "/steps": "fidelity(10, 40, 2)"})

    def test_timeline_and_initial_population(self):
        pbt = create_algo(self._space(), {"pbt": {"seed": 1, "population_size": 6,
                                                   "interval": 10}})
        assert pbt.timeline == [10, 20, 30, 40]
        pts = pbt.suggest(10)
        assert len(pts) == 6 and all(p[1] == 10 for p in pts)
        assert pbt.suggest(1) is None           # waits for results

    def test_exploit_copies_winner_and_perturbs(self):
        space = self._space()
        pbt = create_algo(space, {"pbt": {"seed": 2, "population_size": 10, "interval": 10,
                                           "min_forking_population": 10, "freeze": ["/width"]}})
        pts = pbt.suggest(10)
        objs = {p: float(i) for i, p in enumerate(sorted(pts, key=lambda p: p[0]))}
        pbt.observe(list(objs), [{"objective": o} for o in objs.values()])
        succ = pbt.suggest(10)
        assert len(succ) == 10 and all(s[1] == 20 for s in succ)
        best = min(objs, key=objs.get)
        worst = max(objs, key=objs.get)
        for s in succ:
            parent = pbt.parent_of(s)
            assert parent is not None and parent[1] == 10
            if objs[parent] <= 1.0 and parent != s[:1] + (10,) + s[2:]:
                # exploited child: copy of a top member, lr perturbed by 1.2**+-1, width frozen
                assert s[2] == parent[2]
                assert abs(s[0] / parent[0] - 1.2) < 1e-9 or abs(parent[0] / s[0] - 1.2) < 1e-9
        # the worst member never continues itself
        assert all(pbt.parent_of(s) != worst for s in succ)
        assert any(pbt.parent_of(s) == best for s in succ)
        assert all(s in space for s in succ)

    def test_done_after_last_generation(self):
        pbt = create_algo(self._space(), {"pbt": {"seed": 3, "population_size": 4,
                                                   "interval": 10, "min_forking_population": 2}})
        pts = pbt.suggest(4)
        for _ in range(4):
            pbt.observe(pts, [{"objective": float(i)} for i in range(len(pts))])
            if pbt.is_done:
                break
            pts = pbt.suggest(4)
        assert pbt.is_done

    def test_primary_forwards_parent(self):
        space = self._space()
        primary = PrimaryAlgo(space, {"pbt": {"seed": 4, "population_size": 5, "interval": 10,
                                              "min_forking_population": 5}})
        pts = primary.suggest(5)
        primary.observe(pts, [{"objective": float(i)} for i in range(5)])
        nxt = primary.suggest(5)
        assert all(primary.parent_of(p) in pts for p in nxt)


class TestGridAndHyperband:
    def test_grid(self):
        space = build_space({"/x": "uniform(0, 1)", "/c": "choices(['a', 'b'])",
                             "/lr": "loguniform(1e-3, 1)"})
        grid = create_algo(space, {"gridsearch": {"n_values": 3}})
        pts = []
        while True:
            got = grid.suggest(5)
            if got is None:
                break
            pts.extend(got)
        assert len(pts) == 2 * 3 * 3 and len(set(pts)) == 18
        lrs = sorted({p[1] for p in pts})
        assert abs(lrs[1] / lrs[0] - lrs[2] / lrs[1]) < 1e-6   # log-spaced
        grid.observe(pts, [{"objective": 0.0}] * len(pts))
        assert grid.is_done

    def test_hyperband_synchronous_halving(self):
        space = build_space({"/x": "uniform(0, 1)", "/e": "fidelity(1, 9, 3)"})
        hb = create_algo(space, {"hyperband": {"seed": 1}})
        assert [len(r) for r in hb.schedule] == [3, 2, 1]
        assert hb.schedule[0] == [(9, 1), (3, 3), (1, 9)]
        first = hb.suggest(100)
        assert len(first) == 9 and all(p[0] == 1 for p in first)
        hb.observe(first[:8], [{"objective": p[1]} for p in first[:8]])
        assert hb.suggest(5) is None            # synchronous: waits for the whole rung
        hb.observe(first[8:], [{"objective": first[8][1]}])
        promo = hb.suggest(10)
        best3 = sorted(first, key=lambda p: p[1])[:3]
        assert sorted(p[1] for p in promo) == sorted(p[1] for p in best3)
        assert all(p[0] == 3 for p in promo)
        assert all(hb.parent_of(p) in first for p in promo)
