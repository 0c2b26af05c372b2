"""Batched device copies (``mopt_multi_copy``) used by the sweep's checkpoint pool.

``multi_copy(items)`` moves every ``(src, dst, dst16)`` triple in ONE kernel launch on the GPU,
or with plain tensor copies on the CPU reference backend.  ``src`` is an f32 or bf16 view,
``dst`` an f32 view or None, ``dst16`` an optional bf16 view that receives the rounded copy (a bf16
momentum buffer goes into the f32 checkpoint pool widened, and comes back through ``dst16``).  Replaces the one-framework-copy-per-tensor checkpoint and
resume path that left the GPU idle for ~0.3 ms per copy at every sync.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Tuple

import numpy as np
import torch

from . import _lib

DESC_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("dst16", "<u8"), ("n", "<i8"),
                       ("src16", "<u8"), ("src_lo", "<u8"), ("dst_lo", "<u8"), ("pad", "<i8")])
assert DESC_DTYPE.itemsize == 64


class Split:
    """A split f32 master (``hi`` bf16 working copy + ``lo`` int16 residual, see
    ``csrc/common.h``) as a multi_copy source or destination."""

    __slots__ = ("hi", "lo")

    def __init__(self, hi: torch.Tensor, lo: torch.Tensor):
        self.hi, self.lo = hi, lo

    def numel(self):
        return self.hi.numel()
CHUNK_DTYPE = np.dtype([("desc", "<i4"), ("pad", "<i4"), ("start", "<i8")])
CHUNK = 4096

_lib.register_signatures({
    "mopt_multi_copy": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
                        ctypes.c_int),
})


def multi_copy(items: Iterable[Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]]):
    items = list(items)
    if not items:
        return
    first = items[0][0]
    dev = (first.hi if isinstance(first, Split) else first).device
    if dev.type != "cuda":
        from .reference import join_f32, split_f32
        for src, dst, dst16 in items:
            if isinstance(src, Split):
                src = join_f32(src.hi, src.lo)
            if dst is not None:
                dst.copy_(src)
            if isinstance(dst16, Split):
                hi, lo = split_f32(src.float())
                dst16.hi.copy_(hi)
                dst16.lo.copy_(lo)
            elif dst16 is not None:
                dst16.copy_(src.to(dst16.dtype))
        return
    descs = np.zeros(len(items), dtype=DESC_DTYPE)
    counts = []
    for i, (src, dst, dst16) in enumerate(items):
        n = src.numel()
        if (dst is not None and dst.numel() != n) or (dst16 is not None and dst16.numel() != n):
            raise ValueError("multi_copy: size mismatch")
        if dst is None and dst16 is None:
            raise ValueError("multi_copy: no destination")
        views = [v for v in (src, dst, dst16) if v is not None]
        flat = [t for v in views for t in ((v.hi, v.lo) if isinstance(v, Split) else (v,))]
        if n % 4 or not all(t.is_contiguous() for t in flat):
            raise ValueError("multi_copy: views must be contiguous with a multiple of 4 elements")
        if isinstance(src, Split):
            s32, s16, slo = 0, src.hi.data_ptr(), src.lo.data_ptr()
        elif src.dtype == torch.bfloat16:
            s32, s16, slo = 0, src.data_ptr(), 0
        elif src.dtype == torch.float32:
            s32, s16, slo = src.data_ptr(), 0, 0
        else:
            raise TypeError("multi_copy: source must be f32, bf16 or a split master")
        if dst is not None and dst.dtype != torch.float32:
            raise TypeError("multi_copy: dst must be f32")
        if isinstance(dst16, Split):
            d16, dlo = dst16.hi.data_ptr(), dst16.lo.data_ptr()
        elif dst16 is not None:
            if dst16.dtype != torch.bfloat16:
                raise TypeError("multi_copy: dst16 must be bf16")
            d16, dlo = dst16.data_ptr(), 0
        else:
            d16, dlo = 0, 0
        descs[i] = (s32, 0 if dst is None else dst.data_ptr(), d16, n, s16, slo, dlo, 0)
        counts.append((n + CHUNK - 1) // CHUNK)
    launch_descs(descs, dev)


def launch_descs(descs: np.ndarray, dev) -> None:
    """One ``mopt_multi_copy`` launch over a prebuilt DESC_DTYPE array (raw device pointers;
    the callers build it with numpy -- no per-item tensor views)."""
    if not len(descs):
        return
    counts = (descs["n"].astype(np.int64) + CHUNK - 1) // CHUNK
    chunks = np.zeros(int(counts.sum()), dtype=CHUNK_DTYPE)
    chunks["desc"] = np.repeat(np.arange(len(descs), dtype=np.int32), counts)
    first = np.concatenate([[0], np.cumsum(counts)[:-1]])
    chunks["start"] = (np.arange(len(chunks)) - np.repeat(first, counts)) * CHUNK
    d = _lib.upload_bytes(descs, dev)
    c = _lib.upload_bytes(chunks, dev)
    lib = _lib.get_lib()
    _lib.check(lib.mopt_multi_copy(d.data_ptr(), c.data_ptr(), len(chunks),
                                   _lib.stream_ptr(dev)), "multi_copy")
