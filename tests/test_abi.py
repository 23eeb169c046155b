"""The C-ABI library builds for gfx950, loads, and exports every symbol that
include/vdb.h declares.  No compute calls (runs without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "vdb.h")).read()
    return sorted(set(re.findall(r"\b(vdb_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    from service import _vdb
    assert sorted(_vdb.EXPORTED_SYMBOLS) == _header_symbols()


def test_library_exports_every_header_symbol():
    from service import _vdb
    lib = _vdb.load_library()
    for name in _header_symbols():
        assert hasattr(lib, name), name
    assert lib.vdb_version() >= 1


def test_library_is_gfx950_code_object():
    from service import _vdb
    data = open(_vdb.library_path(), "rb").read()
    assert b"gfx950" in data


def test_no_device_raises_loudly_without_gpu():
    from service import _vdb
    if _vdb.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_vdb.VDBError, match="no HIP device"):
        _vdb.NativeIndex(16, "cosine")


def test_unsupported_metric_is_rejected_before_device():
    from service import _vdb
    with pytest.raises(ValueError):
        _vdb.NativeIndex(16, "dot_product")
