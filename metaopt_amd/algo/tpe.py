"""Tree-structured Parzen Estimator (north-star config 3; not in the reference snapshot, listed in
its ROADMAP "More Optimizers").

Bergstra et al., "Algorithms for Hyper-Parameter Optimization" (NeurIPS 2011).  Observations are
split at the ``gamma`` quantile of the objective into "good" (l) and "bad" (g) sets; each
dimension gets an independent Parzen estimator per set (truncated Gaussians with the hyperopt
neighbour-gap bandwidth plus one prior component; a smoothed histogram for categoricals), and
each suggestion is the best of ``n_ei_candidates`` draws from l by the ratio l(x)/g(x), which is
monotone in expected improvement.

Log-scaled priors (``loguniform``) are modelled in log space; integers are modelled as reals
and rounded.  ``suggest(num)`` for populations uses a constant-liar scheme: every point picked
in the same call is added to the "bad" set before the next pick, so one call spreads over the
space instead of returning near-duplicates.
"""
from __future__ import annotations

import math
from typing import List

import numpy

from ..space.dims import Categorical, Fidelity, Integer
from .base import ALGORITHMS, BaseAlgorithm

_LOG_PRIORS = ("reciprocal", "loguniform")


def _norm_logpdf_trunc(x, mu, sigma, low, high):
    """log pdf of N(mu, sigma) truncated to [low, high]; x [n], mu/sigma [m] -> [n, m]."""
    from scipy.special import log_ndtr, ndtr
    z = (x[:, None] - mu[None, :]) / sigma[None, :]
    logp = -0.5 * z * z - numpy.log(sigma[None, :]) - 0.5 * math.log(2 * math.pi)
    mass = ndtr((high - mu) / sigma) - ndtr((low - mu) / sigma)
    return logp - numpy.log(numpy.maximum(mass, 1e-12))[None, :]


class _Parzen1D:
    """Mixture of truncated Gaussians on [low, high] with a prior component."""

    def __init__(self, obs, low, high, prior_weight=1.0, equal_weight=False, full_weight_num=25):
        obs = numpy.asarray(obs, dtype=float)
        prior_mu = 0.5 * (low + high)
        prior_sigma = high - low
        mus = numpy.concatenate([obs, [prior_mu]])
        order = numpy.argsort(mus)
        srt = mus[order]
        if len(srt) > 1:
            left = numpy.diff(srt, prepend=low)
            right = numpy.diff(srt, append=high)
            sig_sorted = numpy.maximum(left, right)
        else:
            sig_sorted = numpy.array([prior_sigma])
        sigmas = numpy.empty_like(sig_sorted)
        sigmas[order] = sig_sorted
        n = len(obs)
        maxs = prior_sigma
        mins = prior_sigma / min(100.0, 1.0 + n)
        sigmas = numpy.clip(sigmas, mins, maxs)
        sigmas[-1] = prior_sigma
        if equal_weight or n <= full_weight_num:
            w = numpy.ones(n)
        else:  # older observations fade linearly (hyperopt's forgetting ramp)
            ramp = numpy.linspace(1.0 / n, 1.0, num=n - full_weight_num)
            w = numpy.concatenate([ramp, numpy.ones(full_weight_num)])
        weights = numpy.concatenate([w, [prior_weight]])
        self.weights = weights / weights.sum()
        self.mus, self.sigmas, self.low, self.high = mus, sigmas, low, high

    def sample(self, n, rng):
        from scipy.stats import truncnorm
        comp = rng.choice(len(self.mus), size=n, p=self.weights)
        mu, sg = self.mus[comp], self.sigmas[comp]
        a, b = (self.low - mu) / sg, (self.high - mu) / sg
        return truncnorm.rvs(a, b, loc=mu, scale=sg, random_state=rng)

    def logpdf(self, x):
        lp = _norm_logpdf_trunc(numpy.asarray(x, float), self.mus, self.sigmas, self.low, self.high)
        lw = numpy.log(self.weights)[None, :]
        m = (lp + lw).max(axis=1, keepdims=True)
        return (m + numpy.log(numpy.exp(lp + lw - m).sum(axis=1, keepdims=True)))[:, 0]


@ALGORITHMS.register()
class TPE(BaseAlgorithm):
    """TPE with per-dimension Parzen estimators."""

    requires = None

    def __init__(self, space, seed=None, n_initial_points=20, n_ei_candidates=24, gamma=0.25,
                 equal_weight=False, prior_weight=1.0, full_weight_num=25):
        super().__init__(space, seed=seed, n_initial_points=n_initial_points,
                         n_ei_candidates=n_ei_candidates, gamma=gamma, equal_weight=equal_weight,
                         prior_weight=prior_weight, full_weight_num=full_weight_num)
        self._points: List[tuple] = []
        self._objectives: List[float] = []
        self._seen = set()

    def seed_rng(self, seed):
        self.rng = numpy.random.RandomState(seed)

    @property
    def state_dict(self):
        return {"rng_state": self.rng.get_state()}

    def set_state(self, state_dict):
        self.seed_rng(0)
        self.rng.set_state(state_dict["rng_state"])
        if "points" in state_dict:
            self._points = [tuple(p) for p in state_dict["points"]]
            self._objectives = [float(o) for o in state_dict["objectives"]]
            self._seen = {repr(p) for p in self._points}

    def full_state(self):
        """RNG + every observation (the model TPE fits is a function of them)."""
        return {"rng_state": self.rng.get_state(), "points": [list(p) for p in self._points],
                "objectives": list(self._objectives)}

    def observe(self, points, results):
        for p, r in zip(points, results):
            obj = r.get("objective") if isinstance(r, dict) else r
            if obj is None or (isinstance(obj, float) and not math.isfinite(obj)):
                continue
            key = repr(tuple(p))
            if key in self._seen:
                continue
            self._seen.add(key)
            self._points.append(tuple(p))
            self._objectives.append(float(obj))

    # -- per-dimension helpers ----------------------------------------------------------------
    def _dim_bounds(self, dim):
        low, high = dim.interval()
        logscale = dim.prior_name in _LOG_PRIORS
        if not (numpy.isfinite(low) and numpy.isfinite(high)):
            low, high = dim.interval(0.999)
        if isinstance(dim, Integer):
            high = high - 1e-9 if numpy.isfinite(high) else high
        if logscale:
            return math.log(low), math.log(high), True
        return float(low), float(high), False

    def suggest(self, num=1):
        n_obs = len(self._objectives)
        if n_obs < self.n_initial_points:
            n_rand = min(num, self.n_initial_points - n_obs)
            pts = self.space.sample(n_rand, seed=tuple(self.rng.randint(0, 1000000, size=3)))
            if n_rand == num:
                return pts
            return pts + self._suggest_model(num - n_rand, extra_bad=pts)
        return self._suggest_model(num)

    def _suggest_model(self, num, extra_bad=()):
        pts = list(self._points)
        objs = numpy.asarray(self._objectives, dtype=float)
        if len(pts) < 2:
            return self.space.sample(num, seed=tuple(self.rng.randint(0, 1000000, size=3)))
        order = numpy.argsort(objs, kind="stable")
        n_good = max(1, int(math.ceil(self.gamma * len(pts))))
        good = [pts[i] for i in order[:n_good]]
        bad = [pts[i] for i in order[n_good:]] + list(extra_bad)
        out = []
        for _ in range(num):
            p = self._pick(good, bad)
            out.append(p)
            bad.append(p)  # constant liar: pretend the pick is bad so the next pick spreads out
        return out

    def _pick(self, good, bad):
        dims = self.space.values()
        n_cand = int(self.n_ei_candidates)
        cand_cols, score = [], numpy.zeros(n_cand)
        for i, dim in enumerate(dims):
            if isinstance(dim, Fidelity):
                cand_cols.append([dim.high] * n_cand)
                continue
            if dim.shape:
                cand_cols.append(dim.sample(n_cand, self.rng))
                continue
            if isinstance(dim, Categorical):
                cats = list(dim.categories)
                idx = {repr(c): j for j, c in enumerate(cats)}
                prior = numpy.asarray(dim.probabilities) * self.prior_weight

                def hist(points):
                    h = prior.copy()
                    for p in points:
                        h[idx[repr(p[i])]] += 1.0
                    return h / h.sum()

                pl, pg = hist(good), hist(bad)
                c = self.rng.choice(len(cats), size=n_cand, p=pl)
                score += numpy.log(pl[c]) - numpy.log(pg[c])
                cand_cols.append([cats[j] for j in c])
                continue
            low, high, logscale = self._dim_bounds(dim)
            tf = (lambda v: math.log(v)) if logscale else float
            gl = [tf(p[i]) for p in good]
            bl = [tf(p[i]) for p in bad]
            lpar = _Parzen1D(gl, low, high, self.prior_weight, self.equal_weight,
                             self.full_weight_num)
            gpar = _Parzen1D(bl, low, high, self.prior_weight, self.equal_weight,
                             self.full_weight_num)
            x = lpar.sample(n_cand, self.rng)
            score += lpar.logpdf(x) - gpar.logpdf(x)
            vals = numpy.exp(x) if logscale else x
            if isinstance(dim, Integer):
                lo, hi = dim.interval()
                vals = numpy.clip(numpy.floor(vals), lo, hi - 1).astype(int)
                cand_cols.append([int(v) for v in vals])
            else:
                lo, hi = dim.interval()
                vals = numpy.clip(vals, lo, numpy.nextafter(hi, lo))
                cand_cols.append([float(v) for v in vals])
        best = int(numpy.argmax(score))
        return tuple(col[best] for col in cand_cols)
