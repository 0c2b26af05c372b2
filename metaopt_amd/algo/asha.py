"""Asynchronous Successive Halving (reference: ``src/orion/algo/asha.py:36-365``).

Li et al., "A System for Massively Parallel Hyperparameter Tuning" (arXiv:1810.05934).

Same rung/bracket logic as the reference -- budgets ``logspace(log_b(min), log_b(max), n_rungs,
base=b)``, promotion of the top ``len(rung) // b`` completed points of the highest promotable rung,
softmax-of-size bracket choice for new samples, opt-out (``None``) once every bracket is filled --
with three changes made for device populations:

* ``suggest(num)`` supports ``num > 1`` (the reference raises): a population asks for hundreds
  of points at once.  Each suggested point is registered immediately as *pending* (objective
  None) in its rung, so one call never promotes the same point twice and fills count pending
  work exactly like the reference counts lies;
* ``Bracket.is_done`` returns a bool (the reference returns ``len(rung)``, quirk 4);
* the full rung state round-trips through ``state_dict``/``set_state`` when ``full=True`` is
  requested (device checkpoints resume the search without replaying trials).

``unbounded=True`` selects the asynchronous algorithm of Li et al. (Algorithm 2) instead of the
reference's bounded brackets: each bracket's rungs grow without limit (a bracket is never
"filled", its top rung never closes), a configuration is promoted from rung k as soon as it ranks
in the top ``n_k // eta`` of the rung's *completed* entries (``n_k`` = completed, not pending --
otherwise the first completions of a rung full of pending work would all qualify), and a new
configuration is sampled only when nothing is promotable.  With the bounded default every bracket
promotes exactly one configuration to the top budget and ``repetitions=inf`` turns the search
into a chain of tiny brackets: at the device sweep's budget that spent the budget on bottom-rung
runs and lost to random search ("What's weak" 2).  The default stays bounded, the
reference's semantics (``/root/reference/src/orion/algo/asha.py:156-202,317-361``).
"""
from __future__ import annotations

import bisect
import copy
import hashlib
import logging

import numpy

from ..space.dims import Fidelity
from .base import ALGORITHMS, BaseAlgorithm

log = logging.getLogger(__name__)

SPACE_ERROR = ("ASHA cannot be used if space does not contain a fidelity dimension.")


def _is_fidelity(dim) -> bool:
    return isinstance(dim, Fidelity) or isinstance(getattr(dim, "original_dimension", None),
                                                   Fidelity)


@ALGORITHMS.register()
class ASHA(BaseAlgorithm):
    """Asynchronous Successive Halving over the space's single ``fidelity`` dimension."""

    trusted_suggestions = True   # space samples and promotions of already-validated points

    def __init__(self, space, seed=None, grace_period=None, max_resources=None,
                 reduction_factor=None, num_rungs=None, num_brackets=1, repetitions=1,
                 unbounded=False):
        super().__init__(space, seed=seed, max_resources=max_resources,
                         grace_period=grace_period, reduction_factor=reduction_factor,
                         num_rungs=num_rungs, num_brackets=num_brackets, repetitions=repetitions,
                         unbounded=unbounded)
        self.trial_info = {}  # id (non-fidelity params) -> Bracket
        try:
            fid = self.space.values()[self.fidelity_index]
        except IndexError as exc:
            raise RuntimeError(SPACE_ERROR) from exc
        min_r = grace_period if grace_period is not None else fid.low
        max_r = max_resources if max_resources is not None else fid.high
        eta = reduction_factor if reduction_factor is not None else fid.base
        if eta < 2:
            raise AttributeError("Reduction factor for ASHA needs to be at least 2.")
        if num_rungs is None:
            num_rungs = int(numpy.log(max_r / min_r) / numpy.log(eta) + 1)
        self.num_rungs = num_rungs
        budgets = numpy.logspace(numpy.log(min_r) / numpy.log(eta), numpy.log(max_r) / numpy.log(eta),
                                 num_rungs, base=eta).astype(int)
        self.budgets = [int(b) for b in budgets]
        self.eta = eta
        self.brackets = [self._bracket(self.budgets[i:]) for i in range(num_brackets)]
        self._repetition = 1

    def _bracket(self, budgets):
        return (AsyncBracket if self.unbounded else Bracket)(self, self.eta, budgets)

    def seed_rng(self, seed):
        self.rng = numpy.random.RandomState(seed)

    @property
    def state_dict(self):
        return {"rng_state": self.rng.get_state()}

    def set_state(self, state_dict):
        self.seed_rng(0)
        self.rng.set_state(state_dict["rng_state"])
        if "rungs" in state_dict:
            while len(self.brackets) < len(state_dict["rungs"]):
                self.brackets.append(self._bracket(self.budgets[:1]))
            self._repetition = state_dict.get("repetition", 1)
            for bracket, rungs in zip(self.brackets, state_dict["rungs"]):
                bracket.rungs = [(b, {k: (o, tuple(p)) for k, (o, p) in r.items()})
                                 for b, r in rungs]
                bracket.rebuild_index()
            self.trial_info = {k: self.brackets[i] for k, i in state_dict["trial_info"].items()}

    def full_state(self) -> dict:
        """RNG + rungs (for persisting the search itself, not only its RNG)."""
        st = self.state_dict
        st["rungs"] = [[(b, {k: (o, list(p)) for k, (o, p) in r.items()}) for b, r in br.rungs]
                       for br in self.brackets]
        st["trial_info"] = {k: self.brackets.index(b) for k, b in self.trial_info.items()}
        st["repetition"] = self._repetition
        return copy.deepcopy(st)

    def clear_pending(self) -> None:
        """Drop the entries suggested but never reported (objective None) -- after a restore
        the stored trials without a result (waiting or broken) are observed again as
        pending, so only points whose trial never reached the storage disappear."""
        for bracket in self.brackets:
            for _, rung in bracket.rungs:
                for k in [k for k, (o, _) in rung.items() if o is None]:
                    del rung[k]
            bracket.rebuild_index()
        # ``trial_info`` keeps every id's bracket: a point observed again lands where it was

    def suggest(self, num=1):
        """Promotions first (one at a time, each registered as pending), then all remaining new
        points drawn in ONE vectorised ``space.sample`` call and spread over the brackets."""
        out = []
        if self.unbounded:       # batched: every eligible promotion of a rung in one query
            for bracket in self.brackets:
                out.extend(bracket.promote(num - len(out)))
                if len(out) >= num:
                    break
        while len(out) < num and not self.unbounded:
            cand = None
            for bracket in self.brackets:
                cand = bracket.update_rungs()
                if cand is not None:
                    bracket.register(cand, None, overwrite=False)
                    break
            if cand is None:
                break
            out.append(cand)
        remaining = num - len(out)
        if remaining > 0:
            out.extend(self._sample_new(remaining))
        return out or None

    def _suggest_one(self):
        pts = self.suggest(1)
        return pts[0] if pts else None

    def _current_brackets(self):
        current = self.brackets[-self.num_brackets:]
        if all(b.is_filled for b in current):
            if self._repetition >= (self.repetitions if self.repetitions is not None else 1):
                log.debug("All brackets are filled.")
                return None
            # ``repetitions > 1``: run another set of brackets (the population keeps sampling
            # instead of idling, as in the original ASHA which never stops adding configs)
            self._repetition += 1
            self.brackets += [self._bracket(self.budgets[i:]) for i in range(self.num_brackets)]
            current = self.brackets[-self.num_brackets:]
        return current

    def _sample_new(self, n):
        current = self._current_brackets()
        if current is None:
            return []
        fi = self.fidelity_index
        out = []
        for _attempt in range(100):
            need = n - len(out)
            if need <= 0:
                break
            pts = self.space.sample(need, seed=tuple(self.rng.randint(0, 1000000, size=3)))
            sizes = numpy.array([len(b.rungs) for b in current])
            probs = numpy.e ** (sizes - sizes.max())
            probs = numpy.array([p * int(not b.is_filled) for p, b in zip(probs, current)])
            if probs.sum() <= 0:
                break
            picks = self.rng.choice(len(current), size=len(pts), p=probs / probs.sum()).tolist()
            info, get_id = self.trial_info, self.get_id
            rung0 = [b.rungs[0][0] for b in current]
            for point, idx in zip(pts, picks):
                point = (*point[:fi], rung0[idx], *point[fi + 1:])
                _id = get_id(point)
                if _id in info:
                    continue
                b = current[idx]
                info[_id] = b
                b._register_at(0, point, None, False, _id)   # fidelity = rung 0's
                out.append(point)
        else:
            if len(out) < n:
                raise RuntimeError("ASHA keeps sampling already existing points.")
        return out

    def get_id(self, point) -> str:
        """md5 of the non-fidelity values (the bracket key); memoised per point -- every point is
        looked up at suggest, registration and observation."""
        try:
            cache = self.__dict__["_id_cache"]
        except KeyError:
            cache = self.__dict__["_id_cache"] = {}
        key = point if type(point) is tuple else tuple(point)
        _id = cache.get(key)
        if _id is None:
            fi = self.fidelity_index
            # python scalars: numpy 2 reprs np.float64 values as 'np.float64(..)', which would
            # give a sampled point and the same point observed back from storage two ids
            p = [v.item() if isinstance(v, numpy.generic) else v for v in key]
            del p[fi]
            _id = hashlib.md5(str(p).encode("utf-8")).hexdigest()
            if len(cache) > 1 << 20:
                cache.clear()
            cache[key] = _id
        return _id

    def observe(self, points, results):
        self.observe_objectives(points, [r["objective"] for r in results])

    def observe_objectives(self, points, objectives, ids=None):
        """:meth:`observe` with bare objective values (the device sweep's fast path); ``ids``:
        the points' :meth:`get_id` values when the caller kept them (no second lookup)."""
        get_id = self.get_id
        for j, (point, objective) in enumerate(zip(points, objectives)):
            _id = ids[j] if ids is not None else get_id(point)
            bracket = self.trial_info.get(_id)
            if bracket is None:
                fid = point[self.fidelity_index]
                cands = [b for b in self.brackets if b.rungs[0][0] == fid]
                if not cands:
                    raise ValueError(f"No bracket found for point {_id} with fidelity {fid}")
                bracket = cands[0]
            try:
                bracket.register(point, objective, _id=_id)
            except IndexError:
                log.warning("Point registered to wrong bracket (corrupted timestamps?).")
                continue
            self.trial_info.setdefault(_id, bracket)

    @property
    def is_done(self):
        if self.unbounded:        # asynchronous ASHA never runs out of configurations
            return False
        reps = self.repetitions if self.repetitions is not None else 1
        return self._repetition >= reps and all(b.is_done for b in self.brackets)

    @property
    def space(self):
        return self._space

    @space.setter
    def space(self, space):
        self._space = space
        self.__dict__.pop("_fidelity_index", None)   # re-derived for the new space
        self.__dict__.pop("_id_cache", None)

    @property
    def fidelity_index(self) -> int:
        try:
            return self.__dict__["_fidelity_index"]
        except KeyError:
            idx = [i for i, d in enumerate(self.space.values()) if _is_fidelity(d)][0]
            self.__dict__["_fidelity_index"] = idx
            return idx


class Bracket:
    """Rungs ``[(budget, {id: (objective, point)})]`` of one ASHA bracket.

    Each rung also keeps its completed entries sorted by objective, and separately the completed
    entries not yet present in the next rung (``bisect``): a promotion query is then the best
    un-promoted entry, checked against the top-k rank by one binary search -- O(log n) instead of
    re-sorting or scanning the rung.  (Plain lists: a bracket's rungs stay small -- with
    ``repetitions`` a filled bracket is followed by a new one -- and ``sortedcontainers`` was
    measured slower at these sizes.)"""

    def __init__(self, asha, reduction_factor, budgets):
        self.asha = asha
        self.reduction_factor = reduction_factor
        self.rungs = [(int(b), dict()) for b in budgets]
        self._sorted = [[] for _ in budgets]
        self._free = [[] for _ in budgets]

    def rebuild_index(self):
        """Recompute the sorted views after the rungs were replaced wholesale (set_state)."""
        self._sorted = [sorted((o, k) for k, (o, _) in r.items() if o is not None)
                        for _, r in self.rungs]
        self._free = [[e for e in self._sorted[i]
                       if i + 1 >= len(self.rungs) or e[1] not in self.rungs[i + 1][1]]
                      for i in range(len(self.rungs))]

    @staticmethod
    def _discard(lst, entry):
        j = bisect.bisect_left(lst, entry)
        if j < len(lst) and lst[j] == entry:
            del lst[j]

    def register(self, point, objective, overwrite=True, _id=None):
        fid = point[self.asha.fidelity_index]
        if fid == self.rungs[0][0]:
            i = 0
        else:
            idx = [i for i, (b, _) in enumerate(self.rungs) if b == fid]
            if not idx:
                raise IndexError(f"Bad fidelity level {fid}. Should be in "
                                 f"{[b for b, _ in self.rungs]}. Params: {point}")
            i = idx[0]
        self._register_at(i, point, objective, overwrite, _id)

    def _register_at(self, i, point, objective, overwrite, _id=None):
        rung = self.rungs[i][1]
        if _id is None:
            _id = self.asha.get_id(point)
        if not overwrite and _id in rung:
            return
        old = rung.get(_id)
        if old is not None and old[0] is not None:
            self._discard(self._sorted[i], (old[0], _id))
            self._discard(self._free[i], (old[0], _id))
        rung[_id] = (objective, tuple(point))
        if objective is not None:
            bisect.insort(self._sorted[i], (objective, _id))
            if i + 1 >= len(self.rungs) or _id not in self.rungs[i + 1][1]:
                bisect.insort(self._free[i], (objective, _id))
        if i > 0 and old is None:   # entering rung i = promoted out of rung i - 1
            below = self.rungs[i - 1][1].get(_id)
            if below is not None and below[0] is not None:
                self._discard(self._free[i - 1], (below[0], _id))

    def get_candidate(self, rung_id):
        """Best completed entry of the rung's top ``len(rung) // eta`` not promoted yet
        (unbounded: top ``completed // eta``)."""
        free = self._free[rung_id]
        if not free:
            return None
        _, rung = self.rungs[rung_id]
        n = len(self._sorted[rung_id]) if self.asha.unbounded else len(rung)
        k = min(n // self.reduction_factor, len(self._sorted[rung_id]))
        best = free[0]
        if bisect.bisect_left(self._sorted[rung_id], best) < k:
            return rung[best[1]][1]
        return None

    @property
    def is_done(self) -> bool:
        """A point has COMPLETED at the top budget (the reference counts pending ones too)."""
        return any(o is not None for o, _ in self.rungs[-1][1].values())

    @property
    def is_filled(self) -> bool:
        if self.asha.unbounded:
            return False
        return self.has_rung_filled(len(self.rungs) - 2)

    def has_rung_filled(self, rung_id) -> bool:
        n = len(self.rungs)
        return len(self.rungs[rung_id][1]) >= self.reduction_factor ** (n - rung_id - 1)

    def update_rungs(self):
        # bounded: the top rung is taken (pending or completed) -> no more promotions
        if self.rungs[-1][1] and not self.asha.unbounded:
            return None
        for rung_id in range(len(self.rungs) - 2, -1, -1):
            cand = self.get_candidate(rung_id)
            if cand is not None:
                cand = list(cand)       # a tuple of scalars: a shallow copy is a full copy
                cand[self.asha.fidelity_index] = self.rungs[rung_id + 1][0]
                return tuple(cand)
        return None

    def __repr__(self):
        return f"Bracket({[b for b, _ in self.rungs]})"


class AsyncBracket(Bracket):
    """The rungs of asynchronous (unbounded) ASHA, with the promotion query over numpy arrays.

    Unbounded rungs grow by every completion of the sweep (about a thousand per sync at 8 GPUs),
    so the sorted-list index of :class:`Bracket` (``bisect.insort``: O(n) per insert) became the
    rank-0 decision's largest cost.  Here each rung keeps its objectives in a growable float64
    array (NaN = pending) with a "promoted" flag per entry; registering a result is O(1), and a
    promotion query is one ``argpartition`` over the rung's completed objectives -- the top
    ``completed // eta`` -- recomputed only when the rung received a result since the last query.
    The eligible, not yet promoted entries are then handed out best first (ties by arrival)."""

    def __init__(self, asha, reduction_factor, budgets):
        super().__init__(asha, reduction_factor, budgets)
        self.rebuild_index()

    def rebuild_index(self):
        R = len(self.rungs)
        self._pos = [dict() for _ in range(R)]
        self._obj = [numpy.full(64, numpy.nan) for _ in range(R)]
        self._prom = [numpy.zeros(64, dtype=bool) for _ in range(R)]
        self._ids = [[] for _ in range(R)]
        self._queue = [None] * R          # eligible positions, best first (None = recompute)
        for i, (_, rung) in enumerate(self.rungs):
            for _id, (obj, _) in rung.items():
                self._slot(i, _id, obj)
        for i in range(1, R):
            for _id in self.rungs[i][1]:
                j = self._pos[i - 1].get(_id)
                if j is not None:
                    self._prom[i - 1][j] = True

    def _slot(self, i, _id, objective):
        pos = self._pos[i]
        j = pos.get(_id)
        if j is None:
            j = len(self._ids[i])
            if j == len(self._obj[i]):
                self._obj[i] = numpy.concatenate([self._obj[i], numpy.full(j, numpy.nan)])
                self._prom[i] = numpy.concatenate([self._prom[i], numpy.zeros(j, dtype=bool)])
            pos[_id] = j
            self._ids[i].append(_id)
        if objective is not None:
            self._obj[i][j] = objective
            self._queue[i] = None
        return j

    def _register_at(self, i, point, objective, overwrite, _id=None):
        rung = self.rungs[i][1]
        if _id is None:
            _id = self.asha.get_id(point)
        if not overwrite and _id in rung:
            return
        new = _id not in rung
        rung[_id] = (objective, tuple(point))
        self._slot(i, _id, objective)
        if i > 0 and new:   # entering rung i = promoted out of rung i - 1
            j = self._pos[i - 1].get(_id)
            if j is not None:
                self._prom[i - 1][j] = True

    def _eligible(self, i):
        q = self._queue[i]
        if q is None:
            n = len(self._ids[i])
            obj = self._obj[i][:n]
            done = numpy.flatnonzero(~numpy.isnan(obj))
            k = len(done) // self.reduction_factor
            if k == 0:
                q = []
            else:
                top = done[numpy.argpartition(obj[done], k - 1)[:k]] if k < len(done) else done
                top = top[numpy.lexsort((top, obj[top]))]      # best first, ties by arrival
                q = top[~self._prom[i][top]].tolist()
            q.reverse()                                         # pop() from the best end
            self._queue[i] = q
        return q

    def get_candidate(self, rung_id):
        q = self._eligible(rung_id)
        while q and self._prom[rung_id][q[-1]]:
            q.pop()
        return self.rungs[rung_id][1][self._ids[rung_id][q[-1]]][1] if q else None

    def promote(self, num):
        """Up to ``num`` promotions, highest rung first, each registered as pending above."""
        out = []
        fi = self.asha.fidelity_index
        for rung_id in range(len(self.rungs) - 2, -1, -1):
            q = self._eligible(rung_id)
            nxt = self.rungs[rung_id + 1][0]
            while q and len(out) < num:
                j = q.pop()
                if self._prom[rung_id][j]:
                    continue
                cand = list(self.rungs[rung_id][1][self._ids[rung_id][j]][1])
                cand[fi] = nxt
                cand = tuple(cand)
                self._register_at(rung_id + 1, cand, None, False, self._ids[rung_id][j])
                out.append(cand)
            if len(out) >= num:
                break
        return out

    def update_rungs(self):
        out = self.promote(1)
        if out:   # promote() registered it already; suggest() registers again (no-op)
            return out[0]
        return None
