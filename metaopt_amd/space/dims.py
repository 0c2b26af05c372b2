"""Search-space dimensions and the :class:`Space` container.

Behavioural parity with the reference's ``src/orion/algo/space.py`` (``Dimension`` :69-275,
``Real`` :291-405, ``Integer`` :454-497, ``Categorical`` :500-647, ``Fidelity`` :650-729,
``Space`` :732-858): the same constructor signatures, prior strings, bound semantics (low
inclusive / high exclusive), sorted dimension order, and positional indexing.

Differences by design:
  * sampling is vectorised -- one ``rvs`` call per dimension for all ``n`` points plus rejection
    redraws of only the out-of-bound entries -- because device populations ask for hundreds or
    thousands of points per suggest (the reference makes one scipy call per point and dimension);
  * only public numpy 2 / scipy APIs are used (no ``numpy.object``, no ``_parse_args_rvs``).
"""
from __future__ import annotations

import numbers
from typing import Any, Iterable, List, Optional, Sequence

import numpy
from scipy.stats import distributions


def check_random_state(seed):
    """numpy global RNG for ``None``, a RandomState as is, else a RandomState seeded by ``seed``."""
    if seed is None or seed is numpy.random:
        return numpy.random.mtrand._rand  # the global RandomState (public alias)
    if isinstance(seed, numpy.random.RandomState):
        return seed
    try:
        return numpy.random.RandomState(seed)
    except Exception as exc:
        raise ValueError(f"{seed!r} cannot be used to seed a numpy.random.RandomState") from exc


class _Ellipsis:  # pragma: no cover - repr helper
    def __repr__(self):
        return "..."


def _is_numeric_array(point) -> bool:
    def _is_num(x):
        return isinstance(x, (numbers.Number, numpy.ndarray)) and not isinstance(x, bool)
    if isinstance(point, (str, bytes)):
        return False
    try:
        return all(_is_num(x) or _is_numeric_array(x) for x in point)
    except TypeError:
        return _is_num(point) or isinstance(point, numpy.number)


def _normalize_shape(shape) -> tuple:
    if shape is None:
        return ()
    if isinstance(shape, numbers.Integral):
        return (int(shape),)
    return tuple(int(s) for s in shape)


class Dimension:
    """A named dimension with a ``scipy.stats`` prior.

    ``args``/``kwargs`` are the prior's shape/loc/scale parameters; ``default_value`` and
    ``shape`` are consumed here.  ``type`` is the lower-cased class name.
    """

    NO_DEFAULT_VALUE = None

    def __init__(self, name, prior, *args, **kwargs):
        self._name = None
        self.name = name
        if isinstance(prior, str):
            self._prior_name = prior
            self.prior = getattr(distributions, prior)
        elif prior is None:
            self._prior_name = "None"
            self.prior = None
        else:
            self._prior_name = prior.name
            self.prior = prior
        self._args = tuple(args)
        self._kwargs = dict(kwargs)
        self._default_value = self._kwargs.pop("default_value", self.NO_DEFAULT_VALUE)
        self._shape = self._kwargs.pop("shape", None)
        self.validate()

    # -- validation / identity --------------------------------------------------------------
    def validate(self):
        if "random_state" in self._kwargs or "seed" in self._kwargs:
            raise ValueError("random_state/seed cannot be set in a parameter's definition! "
                             "Set seed globally!")
        if "discrete" in self._kwargs:
            raise ValueError("Do not use kwarg 'discrete' on `Dimension`, use `Integer` instead!")
        if "size" in self._kwargs:
            raise ValueError("Use 'shape' keyword only instead of 'size'.")
        if (self.default_value is not self.NO_DEFAULT_VALUE
                and self.default_value not in self):
            raise ValueError(f"{self.default_value} is not a valid value for this Dimension. "
                             "Can't set default value.")

    def _hashable(self):
        return (self.name, self.shape, self.type, tuple(self._args),
                tuple(sorted(self._kwargs.items())), self.default_value, self._prior_name)

    def __eq__(self, other):
        return isinstance(other, Dimension) and self._hashable() == other._hashable()

    def __hash__(self):
        return hash(self._hashable())

    # -- sampling ------------------------------------------------------------------------------
    def _rvs(self, n: int, rng) -> numpy.ndarray:
        """``n`` raw prior draws, shape (n,) + self.shape."""
        return numpy.asarray(self.prior.rvs(*self._args, size=(n,) + self.shape,
                                            random_state=rng, **self._kwargs))

    def sample(self, n_samples=1, seed=None) -> List[Any]:
        rng = check_random_state(seed)
        draws = self._rvs(n_samples, rng)
        return [self._post(d) for d in draws]

    def _post(self, value):
        """Scalar dims yield Python/numpy scalars, shaped dims numpy arrays."""
        if self.shape:
            return value
        return value.item() if isinstance(value, numpy.ndarray) else value

    def cast(self, point):
        raise NotImplementedError

    def interval(self, alpha=1.0):
        """(low inclusive, high exclusive) covering ``alpha`` of the prior's mass (cached: priors
        are immutable and scipy's ``interval`` costs tens of microseconds)."""
        cache = self.__dict__.setdefault("_interval_cache", {})
        if alpha not in cache:
            cache[alpha] = self._compute_interval(alpha)
        return cache[alpha]

    def _compute_interval(self, alpha=1.0):
        return self.prior.interval(alpha, *self._args, **self._kwargs)

    def __contains__(self, point):
        raise NotImplementedError

    # -- strings -------------------------------------------------------------------------------
    def __repr__(self):
        return (f"{self.__class__.__name__}(name={self.name}, prior={{{self._prior_name}: "
                f"{self._args}, {self._kwargs}}}, shape={self.shape}, "
                f"default value={self._default_value})")

    def get_prior_string(self) -> str:
        args = [str(a) for a in self._args]
        args += [f"{k}={v}" for k, v in self._kwargs.items()]
        if self._shape is not None:
            args.append(f"shape={self._shape}")
        if self.default_value is not self.NO_DEFAULT_VALUE:
            args.append(f"default_value={self.default_value!r}")
        return f"{self._prior_name}({', '.join(args)})"

    def get_string(self) -> str:
        return f"{self.name}~{self.get_prior_string()}"

    # -- attributes ----------------------------------------------------------------------------
    @property
    def name(self):
        return self._name

    @name.setter
    def name(self, value):
        if isinstance(value, str) or value is None:
            self._name = value
        else:
            raise TypeError("Dimension's name must be either string or None. "
                            f"Provided: {value}, of type: {type(value)}")

    @property
    def default_value(self):
        return self._default_value

    @property
    def type(self) -> str:
        return self.__class__.__name__.lower()

    @property
    def prior_name(self) -> str:
        return self._prior_name

    @property
    def shape(self) -> tuple:
        return _normalize_shape(self._shape)

    @property
    def cardinality(self):
        return numpy.inf


class Real(Dimension):
    """Real-valued dimension; optional ``low``/``high`` kwargs truncate the prior's support."""

    MAX_TRIES = 4  # reference space.py:371-391 gives each draw 4 tries; here 4 rounds that
    #               accept nothing abort (per-entry tries make large batches fail spuriously)

    def __init__(self, name, prior, *args, **kwargs):
        self._low = kwargs.pop("low", -numpy.inf)
        self._high = kwargs.pop("high", numpy.inf)
        if self._high <= self._low:
            raise ValueError(f"Lower bound {self._low} has to be less than upper bound {self._high}")
        super().__init__(name, prior, *args, **kwargs)

    def __contains__(self, point):
        if not self.shape and isinstance(point, (int, float, numpy.number)) and \
                not isinstance(point, (bool, numpy.bool_)):
            low, high = self.interval()  # scalar fast path (the common case, no numpy)
            return bool(low <= point < high)
        if not _is_numeric_array(point):
            return False
        low, high = self.interval()
        p = numpy.asarray(point)
        if p.shape != self.shape:
            return False
        return bool(numpy.all(p < high) and numpy.all(p >= low))

    def _compute_interval(self, alpha=1.0):
        lo, hi = super()._compute_interval(alpha)
        return (max(lo, self._low), min(hi, self._high))

    def _in_bounds(self, draws: numpy.ndarray) -> numpy.ndarray:
        low, high = self.interval()
        axes = tuple(range(1, draws.ndim))
        ok = (draws >= low) & (draws < high)
        return numpy.all(ok, axis=axes) if axes else ok

    def sample(self, n_samples=1, seed=None):
        rng = check_random_state(seed)
        draws = self._rvs(n_samples, rng).astype(float, copy=False)
        draws = self._redraw(draws, rng, lambda k: self._rvs(k, rng).astype(float, copy=False))
        if not self.shape:
            return draws.tolist()       # python floats in one C pass (no per-value .item())
        return [self._post(d) for d in draws]

    def _redraw(self, draws, rng, draw_fn):
        """Replace out-of-bound entries by in-bound candidates drawn in batches of at least 64
        (4x the missing count); give up after MAX_TRIES batches that accept nothing -- an
        acceptance rate below ~1/256.  (Redrawing only the missing entries made the last few
        of a large sample fail spuriously: at 38 % acceptance one entry is rejected four times
        in a row 15 % of the time.)"""
        ok = self._in_bounds(draws)
        stalled = 0
        while not ok.all():
            if stalled >= self.MAX_TRIES:
                raise ValueError(f"Improbable bounds: (low={self._low}, high={self._high}). "
                                 "Please make interval larger.")
            bad = numpy.nonzero(~ok)[0]
            cand = draw_fn(max(4 * len(bad), 64))
            good = cand[self._in_bounds(cand)][:len(bad)]
            fill = bad[:len(good)]
            draws[fill] = good
            ok[fill] = True
            stalled = 0 if len(good) else stalled + 1
        return draws

    def cast(self, point):
        out = numpy.asarray(point).astype(float)
        return out if isinstance(point, numpy.ndarray) else out.tolist()

    def get_prior_string(self):
        s = super().get_prior_string()
        extras = []
        if self._low != -numpy.inf:
            extras.append(f"low={self._low}")
        if self._high != numpy.inf:
            extras.append(f"high={self._high}")
        if extras:
            s = s[:-1] + (", " if not s.endswith("(") else "") + ", ".join(extras) + ")"
        return s


class _Discrete(Dimension):
    def _compute_interval(self, alpha=1.0):
        low, high = super()._compute_interval(alpha)
        try:
            int_low = int(numpy.floor(low))
        except OverflowError:
            int_low = -numpy.inf
        try:
            int_high = int(numpy.floor(high))
        except OverflowError:
            int_high = numpy.inf
        if int_high < high:  # exclusive upper bound
            int_high += 1
        return (int_low, int_high)


class Integer(Real, _Discrete):
    """Integer dimension: prior draws are floored (``numpy.floor``), like the reference."""

    def __contains__(self, point):
        if not self.shape and isinstance(point, (int, float, numpy.number)) and \
                not isinstance(point, (bool, numpy.bool_)):
            return float(point) % 1 == 0 and super().__contains__(point)
        if not _is_numeric_array(point):
            return False
        p = numpy.asarray(point)
        if not numpy.all(numpy.equal(numpy.mod(p, 1), 0)):
            return False
        return super().__contains__(point)

    def sample(self, n_samples=1, seed=None):
        rng = check_random_state(seed)
        draws = numpy.floor(self._rvs(n_samples, rng).astype(float))
        draws = self._redraw(draws, rng,
                             lambda k: numpy.floor(self._rvs(k, rng).astype(float)))
        draws = draws.astype(int)
        return list(draws) if self.shape else draws.tolist()

    def cast(self, point):
        out = numpy.asarray(point).astype(int)
        return out if isinstance(point, numpy.ndarray) else out.tolist()

    @property
    def cardinality(self):
        low, high = self.interval()
        if not (numpy.isfinite(low) and numpy.isfinite(high)):
            return numpy.inf
        return int((high - low) ** max(1, int(numpy.prod(self.shape)) if self.shape else 1))


class Categorical(Dimension):
    """Categorical dimension over ``categories`` (a dict maps category -> probability)."""

    def __init__(self, name, categories, **kwargs):
        if isinstance(categories, dict):
            self.categories = tuple(categories.keys())
            self._probs = tuple(float(p) for p in categories.values())
        else:
            self.categories = tuple(categories)
            if not self.categories:
                raise ValueError("Categorical dimension needs at least one category")
            self._probs = tuple([1.0 / len(self.categories)] * len(self.categories))
        if not self.categories:
            raise ValueError("Categorical dimension needs at least one category")
        if abs(sum(self._probs) - 1.0) > 1e-6:
            raise ValueError("Categorical probabilities must sum to 1")
        prior = distributions.rv_discrete(values=(list(range(len(self.categories))), self._probs))
        super().__init__(name, prior, **kwargs)

    def sample(self, n_samples=1, seed=None):
        rng = check_random_state(seed)
        idx = rng.choice(len(self.categories), p=self._probs, size=(n_samples,) + self.shape)
        cats = numpy.empty(len(self.categories), dtype=object)
        cats[:] = list(self.categories)
        return list(cats[idx])

    def interval(self, alpha=1.0):
        raise RuntimeError("Categories have no ``interval`` (as they are not ordered).\n"
                           "Use ``self.categories`` instead.")

    def __contains__(self, point):
        if self.shape:
            arr = numpy.asarray(point, dtype=object)
            if arr.shape != self.shape:
                return False
            return all(_cat_in(x, self.categories) for x in arr.ravel())
        if isinstance(point, (list, tuple, numpy.ndarray)):
            return False
        return _cat_in(point, self.categories)

    @property
    def probabilities(self):
        return self._probs

    @property
    def cardinality(self):
        return len(self.categories) ** (int(numpy.prod(self.shape)) if self.shape else 1)

    def __repr__(self):
        if len(self.categories) > 5:
            cats = self.categories[:2] + self.categories[-2:]
            probs = self._probs[:2] + self._probs[-2:]
            pairs = list(zip(cats, probs))
            parts = [f"{c}: {p:.2f}" for c, p in pairs[:2]] + ["..."] + \
                    [f"{c}: {p:.2f}" for c, p in pairs[2:]]
        else:
            parts = [f"{c}: {p:.2f}" for c, p in zip(self.categories, self._probs)]
        return (f"Categorical(name={self.name}, prior={{{', '.join(parts)}}}, shape={self.shape}, "
                f"default value={self.default_value})")

    def get_prior_string(self):
        cats = [repr(c) for c in self.categories]
        if all(p == self._probs[0] for p in self._probs):
            prior = f"[{', '.join(cats)}]"
        else:
            prior = "{" + ", ".join(f"{c}: {p:.2f}" for c, p in zip(cats, self._probs)) + "}"
        args = [prior]
        if self._shape is not None:
            args.append(f"shape={self._shape}")
        if self.default_value is not self.NO_DEFAULT_VALUE:
            args.append(f"default_value={self.default_value!r}")
        return f"choices({', '.join(args)})"

    def cast(self, point):
        lookup = {str(c): c for c in self.categories}

        def get(v):
            if str(v) not in lookup:
                raise ValueError(f"Invalid category: {v}")
            return lookup[str(v)]

        if isinstance(point, numpy.ndarray):
            out = numpy.empty(point.shape, dtype=object)
            for i, v in numpy.ndenumerate(point):
                out[i] = get(v)
            return out
        if isinstance(point, (list, tuple)):
            return [self.cast(p) if isinstance(p, (list, tuple)) else get(p) for p in point]
        return get(point)


def _cat_in(x, categories) -> bool:
    try:
        return x in categories
    except (TypeError, ValueError):  # unhashable / array-valued comparison
        return any(x is c for c in categories)


class Fidelity(Dimension):
    """Placeholder for the resource dimension (epochs, steps, ...) of multi-fidelity algorithms.

    ``sample`` returns ``high``; algorithms such as ASHA choose the level themselves.
    """

    def __init__(self, name, low, high, base=2):  # pylint: disable=super-init-not-called
        if low <= 0:
            raise AttributeError("Minimum resources must be a positive number.")
        if low > high:
            raise AttributeError("Minimum resources must be smaller than maximum resources.")
        if base <= 1:
            raise AttributeError("Base should be greater than 1")
        self._name = None
        self.name = name
        self.low = int(low)
        self.high = int(high)
        self.base = int(base)
        self.prior = None
        self._prior_name = "None"
        self._args = ()
        self._kwargs = {}
        self._shape = None
        self._default_value = self.high

    @property
    def default_value(self):
        return self.high

    def get_prior_string(self):
        return f"fidelity({self.low}, {self.high}, {self.base})"

    def validate(self):
        raise NotImplementedError

    def sample(self, n_samples=1, seed=None):
        return [self.high] * n_samples

    def interval(self, alpha=1.0):
        return (self.low, self.high)

    def cast(self, point=0):
        return int(point)

    def __repr__(self):
        return (f"Fidelity(name={self.name}, low={self.low}, high={self.high}, base={self.base})")

    def __contains__(self, value):
        try:
            return self.low <= value <= self.high
        except TypeError:
            return False

    def _hashable(self):
        return (self.name, "fidelity", self.low, self.high, self.base)


class Space(dict):
    """Sorted mapping name -> :class:`Dimension`; points are tuples in sorted-name order."""

    contains = Dimension

    def register(self, dimension: Dimension) -> None:
        self[dimension.name] = dimension

    def sample(self, n_samples=1, seed=None) -> List[tuple]:
        rng = check_random_state(seed)
        cols = [dim.sample(n_samples, rng) for dim in self.values()]
        return list(zip(*cols))

    def interval(self, alpha=1.0):
        return [dim.categories if dim.type == "categorical" else dim.interval(alpha)
                for dim in self.values()]

    def __getitem__(self, key):
        if isinstance(key, str):
            return super().__getitem__(key)
        return self.values()[key]

    def __setitem__(self, key, value):
        if not isinstance(key, str):
            raise TypeError(f"Keys registered to {self.__class__.__name__} must be string types. "
                            f"Provided: {key}")
        if not isinstance(value, self.contains):
            raise TypeError(f"Values registered to {self.__class__.__name__} must be "
                            f"{self.contains.__name__} types. Provided: {value}")
        if key in self.keys():
            raise ValueError("There is already a Dimension registered with this name. "
                             f"Register it with another name. Provided: {key}")
        super().__setitem__(key, value)

    def __contains__(self, value):
        if isinstance(value, str):
            return super().__contains__(value)
        try:
            len(value)
        except TypeError as exc:
            raise TypeError("Can check only for dimension names or "
                            "for tuples with parameter values.") from exc
        if not self or len(value) != len(self):
            return False
        for component, dim in zip(value, self._sorted_values()):
            if component not in dim:
                return False
        return True

    def __repr__(self):
        return "Space([{}])".format(",\n       ".join(map(str, self.values())))

    def items(self):
        return [(k, dict.__getitem__(self, k)) for k in self._sorted_keys()]

    def values(self):
        return list(self._sorted_values())

    def _sorted_values(self):
        keys = self._sorted_keys()
        cache = getattr(self, "_values_cache", None)
        if cache is None or cache[0] is not keys:
            cache = (keys, tuple(dict.__getitem__(self, k) for k in keys))
            self._values_cache = cache
        return cache[1]

    def keys(self):
        return list(self._sorted_keys())

    def _sorted_keys(self):
        cache = getattr(self, "_keys_cache", None)
        if cache is None or cache[0] != len(self):
            cache = (len(self), tuple(sorted(dict.keys(self))))
            self._keys_cache = cache
        return cache[1]

    def __iter__(self):
        return iter(self._sorted_keys())

    def point_to_dict(self, point: Sequence) -> dict:
        return dict(zip(self.keys(), point))

    def dict_to_point(self, params: dict) -> tuple:
        return tuple(params[k] for k in self.keys())

    @property
    def configuration(self) -> dict:
        """name -> prior string (the ``priors`` metadata format)."""
        return {name: dim.get_prior_string() for name, dim in self.items()}

    @property
    def cardinality(self):
        c = 1
        for dim in self.values():
            c *= dim.cardinality
        return c
