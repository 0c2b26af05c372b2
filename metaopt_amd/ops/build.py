"""In-tree build of the gfx950 HIP kernels into one shared library.

The kernels are plain HIP C++ (no hipify, no CUDA shims) compiled by ``hipcc --offload-arch=gfx950``
into ``metaopt_amd/ops/lib/libmopt_kernels.so``.  The library exposes a C ABI that
:mod:`metaopt_amd.ops._lib` binds with ctypes, so the build needs neither torch headers nor a JIT
cache: the ``.so`` lives in the source tree and travels with the repository snapshot to the GPU box.

Each ``csrc/*.hip`` file is compiled to its own object (incremental: only stale objects rebuild) and
the objects are linked once.  ``python -m metaopt_amd.ops.build [--force]`` rebuilds by hand.

Provenance: the link also writes ``libmopt_kernels.so.sha256``, the digest of every source,
header, flag and the target arch the library was built from, paired with the sha256 of the
linked binary itself (a stamp is void next to any other binary).  ``build()`` recompiles everything
when the digest of the current tree differs (modification times do not survive a copy of the
tree), and the loader (:mod:`._lib`) refuses a library whose digest does not match the sources
next to it -- a stale ``.so`` shipped with a snapshot fails loudly instead of running old code.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OUT_DIR = HERE / "lib"
LIB_NAME = "libmopt_kernels.so"
ARCH = os.environ.get("MOPT_OFFLOAD_ARCH", "gfx950")

COMMON_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]


def hipcc_path() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the HIP kernels cannot be built")


def lib_path() -> Path:
    return OUT_DIR / LIB_NAME


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _headers():
    return sorted(CSRC.glob("*.h"))


def digest_path() -> Path:
    return OUT_DIR / (LIB_NAME + ".sha256")


def source_digest(extra_flags=None) -> str:
    """sha256 of the kernel sources, headers, compiler flags and target arch."""
    h = hashlib.sha256()
    h.update(repr((ARCH, COMMON_FLAGS, list(extra_flags or []))).encode())
    for f in sorted(_sources() + _headers()):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


def _file_sha256(path: Path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def _write_stamp(lib: Path, stamp: Path, digest: str) -> None:
    """Record the source digest together with the hash of the library it describes."""
    stamp.write_text(f"{digest} {_file_sha256(lib)}\n")


def _read_stamp(lib: Path, stamp: Path) -> str:
    """The source digest ``lib`` was built from -- but only when the stamp names this very
    binary (its sha256): a stamp left next to another library (a checkout that changed the
    sources, a copied file) vouches for nothing and reads as ""."""
    if not stamp.exists() or not lib.exists():
        return ""
    parts = stamp.read_text().split()
    if len(parts) != 2 or parts[1] != _file_sha256(lib):
        return ""
    return parts[0]


def built_digest() -> str:
    return _read_stamp(lib_path(), digest_path())


def _needs(obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path, hipcc: str, extra) -> None:
    cmd = [hipcc, *COMMON_FLAGS, *extra, "-c", str(src), "-o", str(obj)]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{proc.stderr}")


def build(force: bool = False, verbose: bool = False, extra_flags=None) -> Path:
    """Compile every ``csrc/*.hip`` for gfx950 and link ``libmopt_kernels.so``; returns its path."""
    hipcc = hipcc_path()
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    digest = source_digest(extra_flags)
    if not force and (built_digest() != digest or not lib_path().exists()):
        force = True                  # other sources/flags than the library's: rebuild all
    obj_dir = OUT_DIR / "obj"
    obj_dir.mkdir(exist_ok=True)
    extra = list(extra_flags or [])
    headers = _headers()
    jobs = []
    objs = []
    for src in _sources():
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _needs(obj, [src, *headers, Path(__file__)]):
            jobs.append((src, obj))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "8"))))
    if jobs:
        with cf.ThreadPoolExecutor(workers) as ex:
            futs = [ex.submit(_compile, s, o, hipcc, extra) for s, o in jobs]
            for f in futs:
                f.result()
        if verbose:
            print(f"[mopt build] compiled {[s.name for s, _ in jobs]}")
    lib = lib_path()
    if force or jobs or _needs(lib, objs):
        tmp = lib.with_suffix(".so.tmp")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
        proc = subprocess.run(cmd, capture_output=True, text=True)
        if proc.returncode != 0:
            raise RuntimeError(f"link failed:\n{proc.stderr}")
        os.replace(tmp, lib)
        _write_stamp(lib, digest_path(), digest)
        if verbose:
            print(f"[mopt build] linked {lib}")
    return lib


# The bounds-checked debug build (SURVEY.md §5 "race detection / sanitizers"): every kernel
# verifies its data-dependent indices on the device (csrc/common.h, MOPT_IN_RANGE) and the host
# raises on a violation after each launch.  Loaded instead of the default library with
# MOPT_KERNEL_CHECKED=1 (metaopt_amd/ops/_lib.py).
CHECKED = "checked"
CHECKED_FLAGS = ["-DMOPT_BOUNDS_CHECK"]


def variant_path(name: str) -> Path:
    return OUT_DIR / "variants" / name / LIB_NAME


def variant_digest(name: str) -> str:
    lib = variant_path(name)
    return _read_stamp(lib, lib.with_suffix(".so.sha256"))


def build_variant(name: str, extra_flags, verbose: bool = False, force: bool = True) -> Path:
    """Build the library with ``extra_flags`` into ``lib/variants/<name>/`` (the checked debug
    build; A/B experiments: load it with ``MOPT_KERNEL_LIB``; the default library is
    untouched).  With ``force=False`` an up-to-date variant (same source digest) is kept."""
    digest = source_digest(extra_flags)
    if not force and variant_path(name).exists() and variant_digest(name) == digest:
        return variant_path(name)
    hipcc = hipcc_path()
    out = OUT_DIR / "variants" / name
    (out / "obj").mkdir(parents=True, exist_ok=True)
    objs = [out / "obj" / (src.stem + ".o") for src in _sources()]
    with cf.ThreadPoolExecutor(max(1, min(len(objs), int(os.environ.get("MAX_JOBS", "8"))))) as ex:
        for f in [ex.submit(_compile, src, obj, hipcc, list(extra_flags))
                  for src, obj in zip(_sources(), objs)]:
            f.result()
    lib = out / LIB_NAME
    proc = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
                           "-o", str(lib)], capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"link failed:\n{proc.stderr}")
    _write_stamp(lib, lib.with_suffix(".so.sha256"), digest)
    if verbose:
        print(f"[mopt build] variant {name}: {lib}")
    return lib


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", default=None, help="name of an A/B variant build")
    ap.add_argument("--checked", action="store_true",
                    help="also build the bounds-checked debug variant")
    ap.add_argument("-D", dest="defines", action="append", default=[],
                    help="preprocessor define of the variant (repeatable)")
    args = ap.parse_args(argv)
    if args.variant:
        print(build_variant(args.variant, [f"-D{d}" for d in args.defines], verbose=True))
        return 0
    path = build(force=args.force, verbose=True)
    print(path)
    if args.checked:
        print(build_variant(CHECKED, CHECKED_FLAGS, verbose=True, force=args.force))
    return 0


if __name__ == "__main__":
    sys.exit(main())
