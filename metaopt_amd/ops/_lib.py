"""ctypes binding of ``libmopt_kernels.so`` (the gfx950 HIP kernels).

The library is loaded after ``torch`` so that its ``libamdhip64.so.7`` dependency resolves to the
HIP runtime torch already mapped (same SONAME): kernels then launch on torch's streams and are
captured by torch's HIP graphs like any other work.

``get_lib()`` raises loudly when the library is missing or fails to load while a GPU is present:
GPU code paths never fall back silently to the PyTorch reference.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import torch  # noqa: F401  (must be imported before the HIP library is dlopen'ed)

from . import build as _build

_LOCK = threading.Lock()
_LIB = None
ABI_VERSION = 15

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_uint = ctypes.c_uint
c_float = ctypes.c_float

_SIGNATURES = {
    "mopt_abi_version": ([], c_int),
    "mopt_mlp_fwd": ([c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                      c_void_p, c_uint, c_int, c_int, c_int, c_void_p], c_int),
    "mopt_mlp_fwd_ce": ([c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_void_p], c_int),
    "mopt_mlp_init": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
                      c_int),
    "mopt_mlp_bwd": ([c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                      c_void_p, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "mopt_mlp_step": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "mopt_mlp_w_layout": ([], c_int),
    "mopt_mlp_steps": ([c_void_p, c_void_p, c_void_p, c_int, c_void_p], c_int),
    "mopt_mlp_bwd0_fwd": ([c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "mopt_mlp_steps_range": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
                             c_int),
}

_OPTIONAL_SIGNATURES: dict = {}


def register_signatures(sigs: dict) -> None:
    """Other op modules declare the C symbols they use (bound lazily on first load)."""
    _OPTIONAL_SIGNATURES.update(sigs)
    if _LIB is not None:
        _bind(_LIB, sigs)


def _bind(lib, sigs):
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


class KernelLibraryError(RuntimeError):
    pass


def get_lib(build_if_missing: bool = True):
    """Return the loaded kernel library (building it in-tree first if needed)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        override = os.environ.get("MOPT_KERNEL_LIB")   # A/B experiments with variant builds
        if CHECKED and not override:
            return _load_checked()
        path = _build.lib_path() if not override else __import__("pathlib").Path(override)
        if not override and build_if_missing and (os.environ.get("MOPT_REBUILD") or
                                                  not path.exists()):
            try:
                _build.build()
            except Exception as exc:  # pragma: no cover - exercised on hosts without hipcc
                raise KernelLibraryError(f"cannot build {path}: {exc}") from exc
        if not path.exists():
            raise KernelLibraryError(f"HIP kernel library not found at {path}; run "
                                     "`python -m metaopt_amd.ops.build`")
        if not override and _build.built_digest() != _build.source_digest():
            if build_if_missing:
                try:
                    _build.build()
                except Exception as exc:  # pragma: no cover - hosts without hipcc
                    raise KernelLibraryError(
                        f"{path} was built from other sources and cannot be rebuilt: {exc}"
                    ) from exc
            if _build.built_digest() != _build.source_digest():
                raise KernelLibraryError(f"{path} was built from other kernel sources than "
                                         "the ones in this tree; rebuild it")
        try:
            lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        except OSError as exc:
            raise KernelLibraryError(f"failed to load {path}: {exc}") from exc
        _bind(lib, _SIGNATURES)
        _bind(lib, _OPTIONAL_SIGNATURES)
        ver = lib.mopt_abi_version()
        if ver != ABI_VERSION:
            raise KernelLibraryError(f"{path} has ABI {ver}, expected {ABI_VERSION}; rebuild it")
        _LIB = lib
        return lib


def _load_checked():
    """The bounds-checked variant (MOPT_KERNEL_CHECKED=1), built in-tree when missing/stale."""
    global _LIB
    path = _build.variant_path(_build.CHECKED)
    digest = _build.source_digest(_build.CHECKED_FLAGS)
    if not path.exists() or _build.variant_digest(_build.CHECKED) != digest:
        try:
            _build.build_variant(_build.CHECKED, _build.CHECKED_FLAGS, force=False)
        except Exception as exc:  # pragma: no cover - hosts without hipcc
            raise KernelLibraryError(f"cannot build the checked library {path}: {exc}") from exc
    try:
        lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    except OSError as exc:
        raise KernelLibraryError(f"failed to load {path}: {exc}") from exc
    _bind(lib, _SIGNATURES)
    _bind(lib, _OPTIONAL_SIGNATURES)
    if lib.mopt_abi_version() != ABI_VERSION or lib.mopt_checked_build() != 1:
        raise KernelLibraryError(f"{path} is not the checked build of ABI {ABI_VERSION}")
    _LIB = lib
    return lib


# Bounds-checked debug build: MOPT_KERNEL_CHECKED=1 loads lib/variants/checked/ (compiled with
# -DMOPT_BOUNDS_CHECK: the kernels verify token ids, labels and gather indices on the device)
# and check() synchronises after every launch, reads the per-module violation counters and
# raises naming the launch.  Implies the synchronous launch checking below.
CHECKED = os.environ.get("MOPT_KERNEL_CHECKED", "0") not in ("", "0")
_CHECKED_MODULES = ("lm_ops", "pop_mlp", "resnet_head")


class BoundsViolation(RuntimeError):
    pass


def violations() -> int:
    """Device-side index violations since the last call (0 outside the checked build)."""
    lib = get_lib()
    total = 0
    for mod in _CHECKED_MODULES:
        fn = getattr(lib, "mopt_violations_" + mod)
        fn.restype = c_uint
        total += fn()
    return total


# Debug mode (SURVEY.md §5 "race detection / sanitizers": the HIP-side analogue of
# HIP_LAUNCH_BLOCKING): MOPT_SYNC_CHECK=1 synchronises the device after every kernel launch
# that is not being captured into a graph, so an asynchronous fault (out-of-bounds access,
# illegal instruction) is reported at the launch that caused it, naming that kernel.
SYNC_CHECK = CHECKED or os.environ.get("MOPT_SYNC_CHECK", "0") not in ("", "0")


def check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"HIP launch of {what} failed with hipError_t {err}")
    if SYNC_CHECK and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.synchronize()
        except RuntimeError as exc:
            raise RuntimeError(f"[MOPT_SYNC_CHECK] device fault after launching {what}: "
                               f"{exc}") from exc
        if CHECKED:
            n = violations()
            if n:
                raise BoundsViolation(f"[MOPT_KERNEL_CHECKED] {what}: {n} out-of-range "
                                      "device index access(es) skipped (see the "
                                      "'[mopt bounds]' line on stdout)")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def upload(data, device, dtype=None) -> torch.Tensor:
    """Host -> device copy that does NOT stall the host on the queued GPU work.

    A copy from pageable host memory makes the runtime wait for the stream to drain first, which
    during a sweep means waiting for every kernel already queued (tens of ms).  The bytes are
    staged in pinned memory from torch's caching host allocator (which keeps the block alive
    until the asynchronous copy has run) and copied with ``non_blocking=True``.
    """
    t = data if isinstance(data, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(data))
    if dtype is not None:
        t = t.to(dtype)
    device = torch.device(device)
    if device.type != "cuda":
        return t.to(device)
    staged = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    staged.copy_(t)
    return staged.to(device, non_blocking=True)


def upload_bytes(arr, device) -> torch.Tensor:
    """``upload`` of a numpy structured array as raw bytes."""
    return upload(np.ascontiguousarray(arr).view(np.uint8), device)


def upload_bytes_into(dst: torch.Tensor, arr) -> None:
    """``upload_bytes`` straight into the existing device buffer ``dst`` (one host -> device
    copy, no device-side copy of a fresh tensor)."""
    t = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8))
    if dst.device.type != "cuda":
        dst.copy_(t)
        return
    staged = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    staged.copy_(t)
    dst.copy_(staged, non_blocking=True)


def available() -> bool:
    """True when a GPU is visible and the kernel library loads."""
    if not torch.cuda.is_available():
        return False
    try:
        get_lib()
        return True
    except KernelLibraryError:
        return False
