"""Build provenance: libmjx355.so carries the hash of the sources it was built from
(mjx_amd/_srchash.py, stamped by csrc/Makefile into mjl_version()), and the loader refuses a library
whose stamp differs from the tree's sources, so a stale binary cannot pass the GPU suite or feed the
bench. CPU only: the library is loaded, nothing is launched."""
import os
import shutil
import subprocess

import pytest

from mjx_amd import _lib, _srchash

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_loaded_library_is_stamped_with_the_tree_hash():
    info = _lib.build_info()
    assert info["lib_src_hash"] == info["tree_src_hash"] == _lib.source_hash()
    assert len(info["lib_src_hash"]) == 16 and "gfx950" in info["version"]


def test_makefile_stamps_the_hash():
    out = subprocess.run(["make", "-n", "-B", "-C", _lib.CSRC], check=True, capture_output=True, text=True).stdout
    assert f'-DMJL_SRC_HASH=\\"{_lib.source_hash()}\\"' in out


def test_edited_source_makes_the_library_stale(tmp_path, monkeypatch):
    """A one-comment edit to a .hip source changes the hash, and the loader then refuses the library
    (an explicit MJX355_LIB keeps the A/B opt-out)."""
    src = tmp_path / "csrc"
    shutil.copytree(_lib.CSRC, src)
    assert _srchash.source_hash(str(src)) == _lib.source_hash()
    with open(src / "step_kernels.hip", "a") as f:
        f.write("\n// an edit after the build\n")
    assert _srchash.source_hash(str(src)) != _lib.source_hash()
    monkeypatch.setattr(_lib, "CSRC", str(src))
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.delenv("MJX355_LIB", raising=False)
    with pytest.raises(_lib.MjlError, match="stale native library"):
        _lib.lib()
    monkeypatch.setenv("MJX355_LIB", _lib.LIB_PATH)  # explicit override: loaded, no check
    assert _lib.lib() is not None
    assert _lib.build_info()["override"]


def test_stamp_parsing():
    assert _lib.stamped_hash("mjx355 0.2 (gfx950) src=0123456789abcdef") == "0123456789abcdef"
    assert _lib.stamped_hash("mjx355 0.1 (gfx950)") == ""
