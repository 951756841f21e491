"""LaserMappingClass — host mirror of include/laserMappingClass.h:38-66 over the C ABI.

Same method names and argument meaning: ``init(map_resolution)``, ``updateCurrentPointsToMap(pc_in, pose)``,
``getMap()``.  The pose is (q_xyzw, t) — what the mapping node reads from /odom (src/laserMappingNode.cpp:108-110) —
or a 4x4 isometry.  Clouds are ``DeviceCloud``s of PointXYZI records.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi
from .cloud import DeviceCloud

_dp = C.POINTER(C.c_double)


def _pose(pose, t=None):
    if t is not None:
        return np.ascontiguousarray(pose, dtype=np.float64), np.ascontiguousarray(t, dtype=np.float64)
    T = np.asarray(pose, dtype=np.float64)
    from .formats import _quat_from_matrix
    return _quat_from_matrix(T[:3, :3]), np.ascontiguousarray(T[:3, 3])


class LaserMappingClass:
    def __init__(self, device: int = 0):
        self._L = _ffi.load()
        self.device = device
        self._h = None

    def init(self, map_resolution: float) -> None:
        """LaserMappingClass::init (src/laserMappingClass.cpp:7-32)."""
        self.close()
        h = C.c_void_p()
        _ffi.check(self._L.floam_mapping_create(float(map_resolution), self.device, C.byref(h)))
        self._h = h

    def updateCurrentPointsToMap(self, pc_in: DeviceCloud, pose_current, t=None) -> None:
        """updateCurrentPointsToMap (src/laserMappingClass.cpp:148-186); pose as (q_xyzw, t) or a 4x4 matrix."""
        q, tt = _pose(pose_current, t)
        _ffi.check(self._L.floam_mapping_update(self._h, pc_in.handle, q.ctypes.data_as(_dp), tt.ctypes.data_as(_dp)))

    def getMap(self) -> DeviceCloud:
        """getMap (src/laserMappingClass.cpp:188-200): a new cloud with every cell's points in cell order."""
        out = DeviceCloud(device=self.device)
        _ffi.check(self._L.floam_mapping_get_map(self._h, out.handle))
        return out

    def size(self) -> int:
        n = C.c_size_t()
        _ffi.check(self._L.floam_mapping_size(self._h, C.byref(n)))
        return n.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.floam_mapping_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
