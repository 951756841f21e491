"""C ABI: libfloam_amd.so loads on a CPU-only host, exports every entry point include/floam_c.h declares, and the
product path fails loudly (no CPU fallback) when no gfx950 device is present."""
import os
import re

import numpy as np
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


def test_abi_version_matches_header():
    """floam_odom_keyframe_update's parameter list changed; the header carries FLOAM_ABI_VERSION and the
    library reports the one it was built with, which the loader checks."""
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "floam_c.h")).read()
    v = int(re.search(r"#define FLOAM_ABI_VERSION (\d+)", hdr).group(1))
    assert _ffi.load().floam_abi_version() == v == _ffi.ABI_VERSION


def test_pose_qt_any_rotation():
    """the 4x4 -> quaternion conversion of the keyframe wrapper needs no scipy and is exact near 180 deg."""
    from floam_amd.odom_estimation import _pose_qt
    rng = np.random.default_rng(3)
    for ang in [0.0, 1e-3, 1.0, np.pi - 1e-9, np.pi]:
        for _ in range(20):
            ax = rng.normal(size=3)
            ax /= np.linalg.norm(ax)
            K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
            R = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
            T = np.eye(4)
            T[:3, :3] = R
            q, _ = _pose_qt(T)
            x, y, z, w = q
            R2 = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                           [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                           [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
            assert abs(np.linalg.norm(q) - 1.0) < 1e-12
            np.testing.assert_allclose(R2, R, atol=1e-12)


def _env_names(path):
    data = open(path, "rb").read()
    return sorted(set(m.decode() for m in re.findall(rb"FLOAM_[A-Z0-9_]+", data)))


def test_product_library_reads_only_documented_variables():
    """A/B switches, stamps and test hooks live in the diagnostic build only
    (FLOAM_DIAG_ENV, floam_amd/csrc/floam_common.hpp); the product library names exactly the two documented variables
    (FLOAM_GRAPH opts into hipGraph capture, FLOAM_MAP_MERGE=0 re-voxelises the whole map)."""
    names = [n for n in _env_names(_ffi.PRODUCT_LIB_PATH) if not n.startswith(("FLOAM_OK", "FLOAM_ERR", "FLOAM_WARN"))]
    assert names == ["FLOAM_GRAPH", "FLOAM_MAP_MERGE"], names


def test_diagnostic_library_exports_every_declared_symbol():
    """The diagnostic build (tests/diag.py loads it for the hook tests) is the same ABI."""
    import ctypes as C
    assert os.path.exists(_ffi.DIAG_LIB_PATH), "libfloam_amd_diag.so not built"
    L = C.CDLL(_ffi.DIAG_LIB_PATH)
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    assert L.floam_abi_version() == _ffi.ABI_VERSION
    assert "FLOAM_LM_FAIL_TEST" in _env_names(_ffi.DIAG_LIB_PATH)
