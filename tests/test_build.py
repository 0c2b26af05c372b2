"""Provenance of the in-tree kernel library (ops/build.py): the digest of the sources it was
built from travels with it, and a library built from other sources is refused or rebuilt."""
import pytest

from metaopt_amd.ops import _lib, build


def test_digest_covers_sources_and_flags():
    d = build.source_digest()
    assert len(d) == 64 and d == build.source_digest()
    assert build.source_digest(["-DMOPT_X"]) != d


def test_stale_library_is_refused(monkeypatch):
    if not build.lib_path().exists():
        pytest.skip("kernel library not built")
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(build, "source_digest", lambda extra=None: "0" * 64)
    with pytest.raises(_lib.KernelLibraryError, match="other kernel sources"):
        _lib.get_lib(build_if_missing=False)


def test_built_library_matches_tree():
    if not build.lib_path().exists():
        pytest.skip("kernel library not built")
    assert build.built_digest() == build.source_digest()


def test_checked_variant_is_the_bounds_checked_build():
    """The debug variant (MOPT_KERNEL_CHECKED=1) is built from this tree with
    -DMOPT_BOUNDS_CHECK and says so; the default library says it is not."""
    import ctypes
    path = build.variant_path(build.CHECKED)
    if not path.exists():
        pytest.skip("checked variant not built")
    assert build.variant_digest(build.CHECKED) == build.source_digest(build.CHECKED_FLAGS)
    chk = ctypes.CDLL(str(path))
    assert chk.mopt_checked_build() == 1
    for mod in _lib._CHECKED_MODULES:
        assert hasattr(chk, "mopt_violations_" + mod)
    if build.lib_path().exists():
        assert ctypes.CDLL(str(build.lib_path())).mopt_checked_build() == 0
