"""ASHA bracket and rung contract (the behaviour tests/unittests/algo/test_asha.py of the reference
pins: rung creation, registration and bad fidelities, candidate promotion rules -- top
len(rung) // eta, completed only, at most once, none when the next rung is full -- bracket
done-ness, update_rungs, the non-fidelity id, suggest's new / promote / opt-out paths, seeding and
state).  Written against this package's API (suggest(num) registers points as pending)."""
import logging

import pytest

from metaopt_amd.algo.asha import ASHA, Bracket
from metaopt_amd.space.builder import build_space


@pytest.fixture
def space():
    # sorted keys: /epoch (fidelity, index 0), /lr, /units
    return build_space({"/lr": "loguniform(1e-4, 1)", "/units": "uniform(8, 64, discrete=True)",
                        "/epoch": "fidelity(1, 9, 3)"})


@pytest.fixture
def asha(space):
    return ASHA(space, seed=1)


@pytest.fixture
def bracket(asha):
    return asha.brackets[0]


def _pt(epoch, lr, units=16):
    return (epoch, lr, units)


def _fill_rung0(bracket, n=9):
    for i in range(n):
        bracket.register(_pt(1, 0.01 * (i + 1)), float(i))


class TestBracket:
    def test_rungs_creation(self, bracket):
        assert [b for b, _ in bracket.rungs] == [1, 3, 9]
        assert all(not r for _, r in bracket.rungs)

    def test_register(self, asha, bracket):
        p = _pt(1, 0.1)
        bracket.register(p, 0.5)
        rung = bracket.rungs[0][1]
        assert rung[asha.get_id(p)] == (0.5, p)

    def test_register_higher_rung(self, asha, bracket):
        p = _pt(3, 0.1)
        bracket.register(p, 0.2)
        assert asha.get_id(p) in bracket.rungs[1][1]

    def test_bad_fidelity(self, bracket):
        with pytest.raises(IndexError, match="Bad fidelity level 2"):
            bracket.register(_pt(2, 0.1), 0.5)

    def test_candidate_is_the_best_of_the_top_third(self, bracket):
        _fill_rung0(bracket)
        cand = bracket.get_candidate(0)
        assert cand == _pt(1, 0.01)

    def test_no_promotion_without_enough_points(self, bracket):
        _fill_rung0(bracket, n=2)                 # 2 // 3 == 0 slots for promotion
        assert bracket.get_candidate(0) is None

    def test_no_promotion_of_pending_points(self, bracket):
        for i in range(9):
            bracket.register(_pt(1, 0.01 * (i + 1)), None)
        assert bracket.get_candidate(0) is None

    def test_promoted_point_is_not_promoted_again(self, asha, bracket):
        _fill_rung0(bracket)
        bracket.register(_pt(3, 0.01), None)      # the best one already entered rung 1
        assert bracket.get_candidate(0) == _pt(1, 0.02)

    def test_only_top_k_are_promotable(self, bracket):
        _fill_rung0(bracket)
        for i in range(3):                        # the top 3 of 9 are all promoted
            bracket.register(_pt(3, 0.01 * (i + 1)), None)
        assert bracket.get_candidate(0) is None

    def test_update_rungs_returns_next_fidelity(self, bracket):
        _fill_rung0(bracket)
        assert bracket.update_rungs() == _pt(3, 0.01)

    def test_update_rungs_none_when_top_taken(self, bracket):
        _fill_rung0(bracket)
        bracket.register(_pt(9, 0.5), None)
        assert bracket.update_rungs() is None

    def test_update_rungs_prefers_higher_rung(self, bracket):
        _fill_rung0(bracket)
        for i in range(3):
            bracket.register(_pt(3, 0.01 * (i + 1)), float(i))
        assert bracket.update_rungs() == _pt(9, 0.01)

    def test_is_done_needs_a_completed_top_point(self, bracket):
        assert not bracket.is_done
        bracket.register(_pt(9, 0.3), None)
        assert not bracket.is_done
        bracket.register(_pt(9, 0.3), 1.0)
        assert bracket.is_done

    def test_is_filled_means_the_penultimate_rung_is_full(self, bracket):
        _fill_rung0(bracket)
        assert not bracket.is_filled              # rung 0 full, rung 1 (needs eta = 3) empty
        for i in range(2):
            bracket.register(_pt(3, 0.01 * (i + 1)), None)
        assert not bracket.is_filled
        bracket.register(_pt(3, 0.03), None)
        assert bracket.is_filled and bracket.has_rung_filled(0)

    def test_overwrite_flag(self, asha, bracket):
        p = _pt(1, 0.1)
        bracket.register(p, None, overwrite=False)
        bracket.register(p, 0.7, overwrite=False)
        assert bracket.rungs[0][1][asha.get_id(p)][0] is None
        bracket.register(p, 0.7)
        assert bracket.rungs[0][1][asha.get_id(p)][0] == 0.7

    def test_rebuild_index_matches_incremental(self, bracket):
        _fill_rung0(bracket)
        bracket.register(_pt(3, 0.01), 0.1)
        before = (bracket._sorted, bracket._free)
        bracket.rebuild_index()
        assert (bracket._sorted, bracket._free) == before

    def test_repr(self, bracket):
        assert repr(bracket) == "Bracket([1, 3, 9])"


class TestASHA:
    def test_get_id_ignores_fidelity(self, asha):
        assert asha.get_id(_pt(1, 0.1)) == asha.get_id(_pt(9, 0.1))
        assert asha.get_id(_pt(1, 0.1)) != asha.get_id(_pt(1, 0.2))

    def test_get_id_numpy_and_python_scalars_agree(self, asha):
        import numpy as np
        assert asha.get_id((1, np.float64(0.1), np.int64(16))) == asha.get_id((1, 0.1, 16))

    def test_observe_routes_to_the_bracket(self, asha):
        p = _pt(1, 0.1)
        asha.observe([p], [{"objective": 0.3}])
        assert asha.brackets[0].rungs[0][1][asha.get_id(p)][0] == 0.3

    def test_observe_unknown_fidelity_raises(self, asha):
        with pytest.raises(ValueError, match="No bracket found"):
            asha.observe([_pt(3, 0.4)], [{"objective": 0.3}])

    def test_observe_corrupted_fidelity_warns(self, asha, caplog):
        p = _pt(1, 0.1)
        asha.observe([p], [{"objective": 0.3}])
        with caplog.at_level(logging.WARNING):
            asha.observe([_pt(2, 0.1)], [{"objective": 0.3}])
        assert "wrong bracket" in caplog.text

    def test_suggest_new_points_at_the_lowest_fidelity(self, asha):
        pts = asha.suggest(5)
        assert len(pts) == 5 and all(p[0] == 1 for p in pts)
        assert len({asha.get_id(p) for p in pts}) == 5

    def test_suggest_promotes_first(self, asha):
        pts = asha.suggest(9)
        asha.observe(pts, [{"objective": float(i)} for i in range(9)])
        nxt = asha.suggest(1)
        assert nxt == [(3,) + tuple(pts[0][1:])]

    def test_suggest_opts_out_when_filled(self, space):
        a = ASHA(space, seed=2)
        for i in range(3):
            a.brackets[0].register(_pt(3, 0.01 * (i + 1)), None)
        assert a.suggest(1) is None

    def test_seed_reproducible(self, space):
        assert ASHA(space, seed=7).suggest(4) == ASHA(space, seed=7).suggest(4)
        assert ASHA(space, seed=7).suggest(4) != ASHA(space, seed=8).suggest(4)

    def test_state_roundtrip(self, space):
        a = ASHA(space, seed=3)
        st = a.state_dict
        first = a.suggest(3)
        b = ASHA(space, seed=99)
        b.set_state(st)
        assert b.suggest(3) == first

    def test_full_state_restores_rungs(self, space):
        a = ASHA(space, seed=3)
        pts = a.suggest(9)
        a.observe(pts, [{"objective": float(i)} for i in range(9)])
        b = ASHA(space, seed=0)
        b.set_state(a.full_state())
        assert b.suggest(1) == a.suggest(1)

    def test_reduction_factor_and_grace_period(self, space):
        a = ASHA(space, seed=1, grace_period=1, max_resources=9, reduction_factor=3)
        assert a.budgets == [1, 3, 9]
        with pytest.raises(AttributeError):
            ASHA(space, seed=1, reduction_factor=1)

    def test_num_brackets(self, space):
        a = ASHA(space, seed=1, num_brackets=2)
        assert [repr(b) for b in a.brackets] == ["Bracket([1, 3, 9])", "Bracket([3, 9])"]
        pts = a.suggest(12)
        assert {p[0] for p in pts} <= {1, 3}

    def test_is_done(self, space):
        a = ASHA(space, seed=1)
        assert not a.is_done
        a.brackets[0].register(_pt(9, 0.2), 0.1)
        assert a.is_done
