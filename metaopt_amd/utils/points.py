"""Flat vectors <-> shaped space points (reference: ``src/orion/core/utils/points.py:13-74``)."""
from __future__ import annotations

import numpy


def flatten_dims(point, space):
    """Flatten every (possibly shaped) component of ``point`` into one flat list."""
    flat = []
    for subpoint, dim in zip(point, space.values()):
        if getattr(dim, "shape", ()):
            flat.extend(numpy.asarray(subpoint).reshape(-1).tolist())
        else:
            flat.append(subpoint)
    return flat


def regroup_dims(point, space):
    """Inverse of :func:`flatten_dims`."""
    out, i = [], 0
    for dim in space.values():
        shape = getattr(dim, "shape", ())
        if shape:
            n = int(numpy.prod(shape))
            out.append(numpy.asarray(point[i:i + n]).reshape(shape))
            i += n
        else:
            out.append(point[i])
            i += 1
    if i != len(point):
        raise ValueError(f"point of length {len(point)} does not match space ({i} values)")
    return tuple(out)


def flatten_points(points, space):
    return [flatten_dims(p, space) for p in points]
