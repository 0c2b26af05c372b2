"""Hyperband (Li et al., JMLR 2018) -- synchronous successive-halving brackets.

Not in the reference (Oríon added it later); implemented here on the same fidelity conventions as
:mod:`~metaopt_amd.algo.asha`: budgets ``low * eta**i`` up to the fidelity's ``high`` with
``eta`` = the fidelity ``base``.  Bracket ``s`` (``s = s_max .. 0``) starts ``n_s =
ceil((s_max + 1) / (s + 1) * eta**s)`` configurations at budget ``R * eta**-s`` and, once EVERY
configuration of a rung is observed, promotes the best ``floor(n_i / eta)`` to the next rung
(the synchronous rule that distinguishes Hyperband from ASHA).  Brackets run one after another;
``repetitions`` restarts the whole schedule.  Like ASHA here, ``suggest(num)`` may return many
points at once, and promoted points keep their hyper-parameters, so :meth:`parent_of` lets a
device population resume them from the lower-budget checkpoint.
"""
from __future__ import annotations

import logging
import math

import numpy

from .asha import _is_fidelity
from .base import ALGORITHMS, BaseAlgorithm

log = logging.getLogger(__name__)


def _nonfid_key(point, fi):
    return repr(tuple(v for i, v in enumerate(point) if i != fi))


@ALGORITHMS.register()
class Hyperband(BaseAlgorithm):
    synchronous = True   # one bracket at a time: a rung advances when all its results are in

    def __init__(self, space, seed=None, repetitions=1):
        super().__init__(space, seed=seed, repetitions=repetitions)
        fids = [i for i, d in enumerate(self.space.values()) if _is_fidelity(d)]
        if len(fids) != 1:
            raise RuntimeError("Hyperband needs exactly one fidelity dimension")
        self.fidelity_index = fi = fids[0]
        fid = self.space.values()[fi]
        self.eta = eta = int(fid.base)
        low, high = float(fid.low), float(fid.high)
        self.s_max = s_max = int(math.floor(math.log(high / low) / math.log(eta) + 1e-9))
        self.schedule = []  # per bracket: [(n_i, budget_i)]
        for s in range(s_max, -1, -1):
            n = int(math.ceil((s_max + 1) / (s + 1) * eta ** s))
            rungs = []
            for i in range(s + 1):
                b = int(round(high * eta ** (i - s)))
                rungs.append((max(1, int(n * eta ** -i)), max(int(low), min(int(high), b))))
            self.schedule.append(rungs)
        self._rep = 0
        self._bracket = 0
        self._rung = 0
        self._issued = {}     # nonfid key -> point of the current rung
        self._results = {}    # nonfid key -> objective of the current rung
        self._prev = {}       # nonfid key -> point of the previous rung (for parent_of)
        self._sent = {}       # promoted points of the current rung already handed out
        self._done = False

    def seed_rng(self, seed):
        self.rng = numpy.random.RandomState(seed)

    @property
    def state_dict(self):
        return {"rng_state": self.rng.get_state(), "rep": self._rep, "bracket": self._bracket,
                "rung": self._rung, "issued": dict(self._issued),
                "results": dict(self._results), "prev": dict(self._prev), "sent": dict(self._sent),
                "done": self._done}

    def set_state(self, state_dict):
        self.seed_rng(0)
        self.rng.set_state(state_dict["rng_state"])
        for k in ("rep", "bracket", "rung", "issued", "results", "prev", "sent", "done"):
            if k in state_dict:
                setattr(self, "_" + k, state_dict[k])

    @property
    def budgets(self):
        return sorted({b for rungs in self.schedule for _, b in rungs})

    def _rung_spec(self):
        return self.schedule[self._bracket][self._rung]

    def suggest(self, num=1):
        if self._done:
            return None
        n_target, budget = self._rung_spec()
        out = []
        if self._rung == 0:
            missing = n_target - len(self._issued)
            if missing > 0:
                n = min(num, missing)
                pts = self.space.sample(n, seed=tuple(self.rng.randint(0, 1000000, size=3)))
                for p in pts:
                    p = list(p)
                    p[self.fidelity_index] = budget
                    p = tuple(p)
                    k = _nonfid_key(p, self.fidelity_index)
                    if k in self._issued:
                        continue
                    self._issued[k] = p
                    out.append(p)
        else:
            pending = [(k, p) for k, p in self._issued.items()
                       if k not in self._results and k not in self._sent]
            for k, p in pending[:num]:
                self._sent[k] = True
                out.append(p)
        return out or None

    def observe(self, points, results):
        for p, r in zip(points, results):
            k = _nonfid_key(p, self.fidelity_index)
            if k in self._issued and tuple(p) == tuple(self._issued[k]) and \
                    r.get("objective") is not None:
                self._results[k] = float(r["objective"])
        self._advance()

    def _advance(self):
        while not self._done:
            n_target, _ = self._rung_spec()
            if len(self._results) < n_target or len(self._results) < len(self._issued):
                return
            rungs = self.schedule[self._bracket]
            if self._rung + 1 < len(rungs):
                n_next, b_next = rungs[self._rung + 1]
                best = sorted(self._results.items(), key=lambda kv: kv[1])[:n_next]
                self._prev = dict(self._issued)
                self._issued = {}
                for k, _ in best:
                    p = list(self._prev[k])
                    p[self.fidelity_index] = b_next
                    self._issued[k] = tuple(p)
                self._results = {}
                self._sent = {}
                self._rung += 1
                return
            # bracket finished
            self._issued, self._results, self._prev, self._sent = {}, {}, {}, {}
            self._rung = 0
            self._bracket += 1
            if self._bracket >= len(self.schedule):
                self._bracket = 0
                self._rep += 1
                if self._rep >= self.repetitions:
                    self._done = True
            return

    def parent_of(self, point):
        if self._rung == 0:
            return None
        k = _nonfid_key(point, self.fidelity_index)
        return self._prev.get(k)

    @property
    def is_done(self):
        return self._done
