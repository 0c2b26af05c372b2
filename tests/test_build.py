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
