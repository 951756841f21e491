"""C ABI: libfloam_amd.so loads on a CPU-only host, exports every entry point include/floam_c.h declares, and the
product path fails loudly (no CPU fallback) when no gfx950 device is present."""
import os
import re

import pytest

from floam_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "floam_c.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(floam_[a-z0-9_]+)\s*\(", hdr)))


def test_header_lists_entry_points():
    names = _declared()
    assert "floam_lp_feature_extraction" in names and "floam_odom_update_selector" in names
    assert set(names) == set(_ffi.EXPORTS), set(names) ^ set(_ffi.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _ffi.load()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing


def test_version_string():
    v = _ffi.load().floam_version().decode()
    assert "gfx950" in v


def test_error_reporting_without_device_is_loud():
    """On this CPU-only container every device call must raise, never silently fall back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from floam_amd import DeviceCloud, FloamError
    with pytest.raises(FloamError) as ei:
        DeviceCloud()
    assert ei.value.status == _ffi.ERR_DEVICE
    assert "device" in str(ei.value).lower()


def test_null_arguments_are_rejected():
    import ctypes as C
    L = _ffi.load()
    assert L.floam_cloud_create(0, 0, None) == _ffi.ERR_INVALID_ARGUMENT
    assert L.floam_lp_create(None, 0, C.byref(C.c_void_p())) == _ffi.ERR_INVALID_ARGUMENT
    assert L.floam_odom_get_pose(None, None, None) == _ffi.ERR_INVALID_ARGUMENT
    assert b"null" in L.floam_last_error()
