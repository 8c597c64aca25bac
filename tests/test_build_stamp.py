"""The in-tree build's staleness check is by content (a sha256 stamp over the native sources written by build()):
snapshots and copies that only change mtimes must not trigger a rebuild on a GPU box that has no build tree."""
import os

from stencil2_amd import _build


def test_stamp_matches_sources():
    assert os.path.exists(_build.STAMP)
    with open(_build.STAMP) as f:
        assert f.read().strip() == _build._source_hash()
    assert not _build.is_stale()


def test_mtime_only_change_is_not_stale():
    src = sorted(_build._sources())[0]
    st = os.stat(src)
    try:
        os.utime(src, (st.st_atime, st.st_mtime + 3600))
        assert not _build.is_stale()
    finally:
        os.utime(src, (st.st_atime, st.st_mtime))


def _no_tree(monkeypatch, tmp_path):
    monkeypatch.setattr(_build, "BUILD", str(tmp_path))
    monkeypatch.setattr(_build, "is_stale", lambda: True)

    def no_build(*a, **k):
        raise AssertionError("build() called without a build tree")

    monkeypatch.setattr(_build, "build", no_build)


def test_no_build_tree_refuses_stale_artifacts(monkeypatch, tmp_path):
    """a snapshot whose sources differ from the stamp and that has no configured build tree (a GPU box) must neither
    rebuild half-way nor silently load native code built from other sources"""
    import pytest
    _no_tree(monkeypatch, tmp_path)
    monkeypatch.delenv("STENCIL_ALLOW_STALE", raising=False)
    with pytest.raises(RuntimeError, match="differ from the build stamp"):
        _build.ensure_built()


def test_no_build_tree_stale_opt_in(monkeypatch, tmp_path):
    _no_tree(monkeypatch, tmp_path)
    monkeypatch.setenv("STENCIL_ALLOW_STALE", "1")
    _build.ensure_built()  # loads the shipped artifacts, with a warning


def test_cmake_helpers_are_hashed():
    assert any(f.endswith("git_sha.cmake") for f in _build._sources())
