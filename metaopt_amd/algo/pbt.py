"""Population-Based Training (Jaderberg et al., arXiv:1711.09846) as a suggest/observe algorithm.

The reference has no PBT (north-star config 5 adds it); this follows the study API of every other
algorithm here, so the same code drives host black-box workers and device populations:

* the space needs a ``fidelity`` dimension -- the *cumulative* training budget (e.g. steps).
  The fork timeline is ``low, low + interval, ...`` (``interval`` defaults to ``low``) up to
  ``high``: every ``interval`` units each member is ready to be exploited;
* generation 0 is ``population_size`` points sampled from the priors at the first budget;
* when a member completes generation ``g`` (observed objective) it gets a successor at the next
  budget.  **Exploit** (truncation selection): once at least ``min_forking_population`` members
  of generation ``g`` are observed, a member in the worst ``1 - truncation_quantile`` fraction
  is replaced by a copy of a member drawn from the best ``candidate_pool_ratio`` fraction;
  **explore**: the copy's hyper-parameters are perturbed (x or / ``factor``, clipped to the
  prior's bounds; categorical resampled with ``resample_probability``).  Other members continue
  unchanged;
* :meth:`parent_of` returns the point whose trained state (weights, optimizer, step counter) the
  successor must resume from -- the member itself, or the exploited winner.  Dimensions listed
  in ``freeze`` (architecture, e.g. ``/width``) are never perturbed, so a resumed state always
  fits the successor.
"""
from __future__ import annotations

import copy
import logging
from typing import Dict, List, Optional

import numpy

from .asha import _is_fidelity
from .base import ALGORITHMS, BaseAlgorithm

log = logging.getLogger(__name__)


def _key(point) -> tuple:
    return tuple(v.tolist() if isinstance(v, numpy.ndarray) else v for v in point)


@ALGORITHMS.register()
class PBT(BaseAlgorithm):
    synchronous = True   # a generation's exploit needs that generation's results

    def __init__(self, space, seed=None, population_size=16, interval=None,
                 min_forking_population=5, truncation_quantile=0.8, candidate_pool_ratio=0.2,
                 factor=1.2, resample_probability=0.2, freeze=()):
        super().__init__(space, seed=seed, population_size=population_size, interval=interval,
                         min_forking_population=min_forking_population,
                         truncation_quantile=truncation_quantile,
                         candidate_pool_ratio=candidate_pool_ratio, factor=factor,
                         resample_probability=resample_probability, freeze=list(freeze))
        fids = [i for i, d in enumerate(self.space.values()) if _is_fidelity(d)]
        if len(fids) != 1:
            raise RuntimeError("PBT needs exactly one fidelity dimension (the training budget)")
        self.fidelity_index = fids[0]
        fid = self.space.values()[self.fidelity_index]
        low, high = int(fid.low), int(fid.high)
        step = int(interval) if interval else low
        if step <= 0:
            raise ValueError("PBT interval must be positive")
        self.timeline = list(range(low, high + 1, step))
        if self.timeline[-1] != high:
            self.timeline.append(high)
        # lineage bookkeeping: point key -> {"point", "gen", "objective", "parent"}
        self.nodes: Dict[tuple, dict] = {}
        self.generations: List[Dict[tuple, Optional[float]]] = [{} for _ in self.timeline]
        self._ready: List[tuple] = []      # observed members waiting for their successor
        self._forked = set()               # members whose successor was issued
        # exploit / explore record: (generation forked from, loser key, winner key), and the
        # number of perturbed hyper-parameter sets (explore) per generation forked from
        self.exploit_log: List[tuple] = []
        self.explores: Dict[int, int] = {}

    # ------------------------------------------------------------------ RNG / state
    def seed_rng(self, seed):
        self.rng = numpy.random.RandomState(seed)

    @property
    def state_dict(self):
        return {"rng_state": self.rng.get_state(), "nodes": copy.deepcopy(self.nodes),
                "ready": list(self._ready), "forked": sorted(self._forked, key=repr),
                "exploit_log": list(self.exploit_log), "explores": dict(self.explores)}

    def set_state(self, state_dict):
        self.seed_rng(0)
        self.rng.set_state(state_dict["rng_state"])
        if "nodes" in state_dict:
            self.nodes = copy.deepcopy(state_dict["nodes"])
            self.generations = [{} for _ in self.timeline]
            for k, n in self.nodes.items():
                self.generations[n["gen"]][k] = n["objective"]
            self._ready = [tuple(k) for k in state_dict["ready"]]
            self._forked = set(tuple(k) for k in state_dict["forked"])
            self.exploit_log = [tuple(e) for e in state_dict.get("exploit_log", [])]
            self.explores = {int(g): int(n) for g, n in state_dict.get("explores", {}).items()}

    # ------------------------------------------------------------------ study API
    def suggest(self, num=1):
        out = []
        gen0 = self.generations[0]
        n_init = min(num, self.population_size - len(gen0))
        if n_init > 0:
            pts = self.space.sample(n_init, seed=tuple(self.rng.randint(0, 1000000, size=3)))
            for p in pts:
                p = list(p)
                p[self.fidelity_index] = self.timeline[0]
                p = tuple(p)
                if _key(p) in self.nodes:
                    continue
                self._add(p, 0, None)
                out.append(p)
        still_waiting = []
        for k in self._ready:
            if len(out) >= num:
                still_waiting.append(k)
                continue
            succ = self._successor(k)
            if succ is None:
                still_waiting.append(k)
            else:
                out.append(succ)
        self._ready = still_waiting
        return out or None

    def observe(self, points, results):
        for point, result in zip(points, results):
            k = _key(point)
            node = self.nodes.get(k)
            if node is None:  # a point this instance did not suggest (e.g. replayed history)
                fid = point[self.fidelity_index]
                if fid not in self.timeline:
                    continue
                node = self._add(tuple(point), self.timeline.index(fid), None)
            obj = result.get("objective")
            if obj is None:
                continue
            node["objective"] = float(obj)
            self.generations[node["gen"]][k] = float(obj)
            if node["gen"] < len(self.timeline) - 1 and k not in self._forked \
                    and k not in self._ready:
                self._ready.append(k)

    def parent_of(self, point):
        """The point whose trained state ``point`` resumes from (None: train from scratch)."""
        node = self.nodes.get(_key(point))
        if node is None or node["parent"] is None:
            return None
        return self.nodes[node["parent"]]["point"]

    def exploit_counts(self) -> Dict[int, tuple]:
        """{generation forked from: (#exploits, #explores)} -- an exploit replaces a bottom
        member by a copy of a top one; an explore perturbs a copy's hyper-parameters."""
        out: Dict[int, list] = {}
        for g, _, _ in self.exploit_log:
            out.setdefault(g, [0, 0])[0] += 1
        for g, n in self.explores.items():
            out.setdefault(g, [0, 0])[1] += n
        return {g: tuple(v) for g, v in sorted(out.items())}

    @property
    def is_done(self):
        last = self.generations[-1]
        done = sum(1 for v in last.values() if v is not None)
        return done >= self.population_size

    # ------------------------------------------------------------------ internals
    def _add(self, point, gen, parent):
        k = _key(point)
        node = {"point": tuple(point), "gen": gen, "objective": None, "parent": parent}
        self.nodes[k] = node
        self.generations[gen].setdefault(k, None)
        return node

    def _successor(self, k):
        node = self.nodes[k]
        g = node["gen"]
        done = sorted((v, kk) for kk, v in self.generations[g].items() if v is not None)
        if len(done) < min(self.min_forking_population, self.population_size):
            return None
        rank = [kk for _, kk in done].index(k)
        n = len(done)
        source = k
        params = list(node["point"])
        explored = 0
        if rank >= int(numpy.ceil(self.truncation_quantile * n)):       # bottom fraction: exploit
            pool = max(1, int(numpy.floor(self.candidate_pool_ratio * n)))
            source = done[self.rng.randint(pool)][1]
            params = self._explore(list(self.nodes[source]["point"]))
            explored = 1
        params[self.fidelity_index] = self.timeline[g + 1]
        succ = tuple(params)
        tries = 0
        while _key(succ) in self.nodes and tries < 10:  # identical child: explore again
            succ = list(self._explore(list(self.nodes[source]["point"])))
            succ[self.fidelity_index] = self.timeline[g + 1]
            succ = tuple(succ)
            tries += 1
            explored = 1
        if _key(succ) in self.nodes:
            return None
        self._forked.add(k)
        self._add(succ, g + 1, source)
        if source != k:
            self.exploit_log.append((g, k, source))
        if explored:
            self.explores[g] = self.explores.get(g, 0) + 1
        return succ

    def _explore(self, params):
        out = list(params)
        for i, dim in enumerate(self.space.values()):
            if i == self.fidelity_index or dim.name in self.freeze:
                continue
            if dim.type == "categorical" or getattr(dim, "prior_name", "") == "choices":
                if self.rng.rand() < self.resample_probability:
                    out[i] = dim.sample(1, seed=tuple(self.rng.randint(0, 1000000, size=3)))[0]
                continue
            low, high = dim.interval()
            f = self.factor if self.rng.rand() < 0.5 else 1.0 / self.factor
            v = numpy.asarray(out[i], dtype=float) * f
            if dim.type == "integer":
                v = numpy.round(v)
                v = numpy.clip(v, low, high - 1)
                out[i] = v.astype(int).tolist() if v.shape else int(v)
            else:
                hi = numpy.nextafter(high, -numpy.inf) if numpy.isfinite(high) else high
                v = numpy.clip(v, low, hi)
                out[i] = v.tolist() if v.shape else float(v)
        return out
