"""Transformations from the user's space to the space an algorithm requires.

Same contract as the reference's ``src/orion/core/worker/transformer.py:21-481``:
``build_required_space(requirements, space)`` maps every dimension through a chain of
transformers so that an algorithm requiring ``'real'`` or ``'integer'`` only ever sees such
dimensions, and ``TransformedSpace.transform/reverse`` convert whole points.

* real -> integer: ``Quantize`` (floor);  integer -> real: ``Reverse(Quantize)``
* categorical -> integer: ``Enumerate``;  categorical -> real: ``Enumerate`` + ``OneHotEncode``
  (two categories collapse to one scalar in [0, 1], one category to a constant)
* fidelity dimensions pass through unchanged for every requirement (algorithms never optimise
  them; the reference raises here, which breaks multi-fidelity algorithms with requirements).
"""
from __future__ import annotations

from typing import List, Optional

import numpy

from .dims import Dimension, Space


class Transformer:
    """An injective map and its inverse between a domain type and a target type."""

    domain_type: Optional[str] = None
    target_type: Optional[str] = None

    def transform(self, point):
        raise NotImplementedError

    def reverse(self, transformed_point):
        raise NotImplementedError

    def infer_target_shape(self, shape):
        return shape

    def repr_format(self, what):
        return f"{self.__class__.__name__}({what})"

    def _hashable(self):
        return (self.__class__.__name__, self.domain_type, self.target_type)

    def __eq__(self, other):
        return isinstance(other, Transformer) and self._hashable() == other._hashable()

    def __hash__(self):
        return hash(self._hashable())


class Identity(Transformer):
    def __init__(self, domain_type=None):
        self._domain_type = domain_type

    @property
    def domain_type(self):
        return self._domain_type

    @property
    def target_type(self):
        return self._domain_type

    def transform(self, point):
        return point

    def reverse(self, transformed_point):
        return transformed_point

    def repr_format(self, what):
        return what


class Compose(Transformer):
    """Apply ``transformers`` left to right (reverse: right to left)."""

    def __init__(self, transformers: List[Transformer], base_domain_type=None):
        chain = Identity(base_domain_type)
        for t in transformers:
            chain = _Pair(t, chain)
        self._chain = chain
        self.transformers = list(transformers)
        self._base = base_domain_type

    def transform(self, point):
        return self._chain.transform(point)

    def reverse(self, transformed_point):
        return self._chain.reverse(transformed_point)

    def infer_target_shape(self, shape):
        return self._chain.infer_target_shape(shape)

    def repr_format(self, what):
        return self._chain.repr_format(what)

    @property
    def domain_type(self):
        return self._base

    @property
    def target_type(self):
        return self._chain.target_type

    def _hashable(self):
        return ("Compose", self._base) + tuple(t._hashable() for t in self.transformers)


class _Pair(Transformer):
    """outer(inner(x))."""

    def __init__(self, outer: Transformer, inner: Transformer):
        self.outer, self.inner = outer, inner

    def transform(self, point):
        return self.outer.transform(self.inner.transform(point))

    def reverse(self, transformed_point):
        return self.inner.reverse(self.outer.reverse(transformed_point))

    def infer_target_shape(self, shape):
        return self.outer.infer_target_shape(self.inner.infer_target_shape(shape))

    def repr_format(self, what):
        return self.outer.repr_format(self.inner.repr_format(what))

    @property
    def domain_type(self):
        return self.inner.domain_type

    @property
    def target_type(self):
        t = self.outer.target_type
        return t if t is not None else self.inner.target_type


class Reverse(Transformer):
    """Swap a transformer's forward and inverse maps."""

    def __init__(self, transformer: Transformer):
        self.transformer = transformer

    @property
    def domain_type(self):
        return self.transformer.target_type

    @property
    def target_type(self):
        return self.transformer.domain_type

    def transform(self, point):
        return self.transformer.reverse(point)

    def reverse(self, transformed_point):
        return self.transformer.transform(transformed_point)

    def repr_format(self, what):
        return f"ReverseTransform({self.transformer.repr_format(what)})"

    def _hashable(self):
        return ("Reverse",) + self.transformer._hashable()


class Quantize(Transformer):
    """real -> integer by ``floor`` (not injective; reverse casts back to float)."""

    domain_type = "real"
    target_type = "integer"

    def transform(self, point):
        return numpy.floor(numpy.asarray(point)).astype(int)

    def reverse(self, transformed_point):
        return numpy.asarray(transformed_point).astype(float)


class Enumerate(Transformer):
    """categorical -> integer index of the category."""

    domain_type = "categorical"
    target_type = "integer"

    def __init__(self, categories):
        self.categories = tuple(categories)
        self._index = {self._key(c): i for i, c in enumerate(self.categories)}

    @staticmethod
    def _key(c):
        try:
            hash(c)
            return c
        except TypeError:
            return repr(c)

    def transform(self, point):
        arr = numpy.asarray(point, dtype=object)
        out = numpy.empty(arr.shape, dtype=int)
        for idx, v in numpy.ndenumerate(arr):
            out[idx] = self._index[self._key(v)]
        return out if out.shape else numpy.asarray(int(out))

    def reverse(self, transformed_point):
        arr = numpy.asarray(transformed_point)
        out = numpy.empty(arr.shape, dtype=object)
        for idx, v in numpy.ndenumerate(arr):
            out[idx] = self.categories[int(v)]
        return out if out.shape else out[()]

    def _hashable(self):
        return super()._hashable() + (tuple(repr(c) for c in self.categories),)


class OneHotEncode(Transformer):
    """integer in [0, bound) -> one-hot real vector (bound <= 2: a single real in [0, 1])."""

    domain_type = "integer"
    target_type = "real"

    def __init__(self, bound: int):
        self.num_cats = int(bound)

    def transform(self, point):
        p = numpy.asarray(point)
        if not (numpy.all(p < self.num_cats) and numpy.all(p >= 0) and numpy.all(p % 1 == 0)):
            raise AssertionError("point outside the encodable range")
        if self.num_cats <= 2:
            return numpy.asarray(p, dtype=float)
        hot = numpy.zeros(self.infer_target_shape(p.shape))
        hot.reshape(-1, self.num_cats)[numpy.arange(p.size), p.reshape(-1).astype(int)] = 1.0
        return hot

    def reverse(self, transformed_point):
        p = numpy.asarray(transformed_point)
        if self.num_cats == 2:
            return (p > 0.5).astype(int)
        if self.num_cats == 1:
            return numpy.zeros_like(p, dtype=int)
        if p.shape[-1] != self.num_cats:
            raise AssertionError("wrong one-hot width")
        return p.argmax(axis=-1)

    def infer_target_shape(self, shape):
        return tuple(shape) + (self.num_cats,) if self.num_cats > 2 else tuple(shape)

    def _hashable(self):
        return super()._hashable() + (self.num_cats,)


class TransformedDimension:
    """Duck-typed :class:`Dimension` seen through a transformer."""

    NO_DEFAULT_VALUE = Dimension.NO_DEFAULT_VALUE

    def __init__(self, transformer: Transformer, original_dimension: Dimension):
        self.original_dimension = original_dimension
        self.transformer = transformer

    def transform(self, point):
        return self.transformer.transform(point)

    def reverse(self, transformed_point):
        return self.transformer.reverse(transformed_point)

    def sample(self, n_samples=1, seed=None):
        return [self.transform(s) for s in self.original_dimension.sample(n_samples, seed)]

    def interval(self, alpha=1.0):
        try:
            low, high = self.original_dimension.interval(alpha)
        except RuntimeError as exc:
            if "Categories" in str(exc):
                return (-0.1, 1.1)
            raise
        if self.original_dimension.type == "fidelity":
            return (low, high)
        return self.transform(low), self.transform(high)

    def __contains__(self, point):
        try:
            orig = self.reverse(point)
        except (AssertionError, IndexError, KeyError, ValueError):
            return False
        if isinstance(orig, numpy.ndarray) and orig.shape == () and \
                self.original_dimension.type != "categorical":
            orig = orig.item()
        return orig in self.original_dimension

    def __repr__(self):
        return self.transformer.repr_format(repr(self.original_dimension))

    def __eq__(self, other):
        return (hasattr(other, "transformer") and hasattr(other, "original_dimension")
                and self.transformer == other.transformer
                and self.original_dimension == other.original_dimension)

    def __hash__(self):
        return hash((self.transformer._hashable(), self.original_dimension))

    def validate(self):
        self.original_dimension.validate()

    def get_prior_string(self):
        return self.transformer.repr_format(self.original_dimension.get_prior_string())

    def get_string(self):
        return f"{self.name}~{self.get_prior_string()}"

    @property
    def name(self):
        return self.original_dimension.name

    @property
    def type(self):
        t = self.transformer.target_type
        return t if t is not None else self.original_dimension.type

    @property
    def shape(self):
        return self.transformer.infer_target_shape(self.original_dimension.shape)

    @property
    def default_value(self):
        d = self.original_dimension.default_value
        return self.transform(d) if d is not None else None

    @property
    def prior_name(self):
        return self.original_dimension.prior_name

    def cast(self, point):
        return self.transform(self.original_dimension.cast(point))

    # fidelity pass-through attributes
    def __getattr__(self, item):
        if item in ("low", "high", "base", "categories"):
            return getattr(self.original_dimension, item)
        raise AttributeError(item)


class TransformedSpace(Space):
    contains = TransformedDimension

    def _is_identity(self) -> bool:
        """True when no dimension is transformed (e.g. ASHA / random / PBT on any space): points
        then pass through unchanged and membership is the original dimensions' -- the device
        sweep moves thousands of points per sync through here."""
        cache = getattr(self, "_identity_cache", None)
        if cache is None or cache[0] != len(self):
            ident = all(isinstance(d.transformer, Compose) and not d.transformer.transformers
                        for d in self.values())
            cache = (len(self), ident)
            self._identity_cache = cache
        return cache[1]

    def transform(self, point):
        if self._is_identity():
            return tuple(point)
        return tuple(dim.transform(point[i]) for i, dim in enumerate(self.values()))

    def reverse(self, transformed_point):
        if self._is_identity():
            return tuple(transformed_point)
        return tuple(dim.reverse(transformed_point[i]) for i, dim in enumerate(self.values()))

    def __contains__(self, value):
        if isinstance(value, str) or not self._is_identity():
            return super().__contains__(value)
        try:
            n = len(value)
        except TypeError as exc:
            raise TypeError("Can check only for dimension names or "
                            "for tuples with parameter values.") from exc
        if not self or n != len(self):
            return False
        return all(v in d.original_dimension for v, d in zip(value, self._sorted_values()))


def build_required_space(requirements, original_space: Space) -> TransformedSpace:
    """Transformed copy of ``original_space`` satisfying ``requirements`` (None/'real'/'integer')."""
    requirements = requirements if isinstance(requirements, list) else [requirements]
    space = TransformedSpace()
    for dim in original_space.values():
        transformers: List[Transformer] = []
        type_ = dim.type
        base = type_
        for req in requirements:
            if type_ == "fidelity":
                pass
            elif type_ == "real" and req in ("real", None):
                pass
            elif type_ == "real" and req == "integer":
                transformers.append(Quantize())
            elif type_ == "integer" and req in ("integer", None):
                pass
            elif type_ == "integer" and req == "real":
                transformers.append(Reverse(Quantize()))
            elif type_ == "categorical" and req == "real":
                transformers.extend([Enumerate(dim.categories), OneHotEncode(len(dim.categories))])
            elif type_ == "categorical" and req == "integer":
                transformers.append(Enumerate(dim.categories))
            elif type_ == "categorical" and req is None:
                pass
            else:
                raise TypeError(f"Unsupported dimension type ('{type_}') or requirement ('{req}')")
            if transformers and transformers[-1].target_type is not None:
                type_ = transformers[-1].target_type
        space.register(TransformedDimension(Compose(transformers, base), dim))
    return space
