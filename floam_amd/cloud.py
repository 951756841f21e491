"""DeviceCloud: a device-resident (HBM) point cloud, the stand-in for pcl::PointCloud<PointXYZIRT|PointXYZI>::Ptr."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi
from .synth import POINT_DTYPE


class DeviceCloud:
    """32-B point records (vel_point::PointXYZIRT layout) on GPU ``device``."""

    def __init__(self, points: np.ndarray | None = None, device: int = 0, capacity: int = 0):
        self._L = _ffi.load()
        self.device = device
        h = C.c_void_p()
        _ffi.check(self._L.floam_cloud_create(device, capacity, C.byref(h)))
        self._h = h
        if points is not None:
            self.upload(points)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def upload(self, points: np.ndarray) -> None:
        a = np.ascontiguousarray(points)
        if a.dtype.itemsize != 32:
            raise ValueError("points must be 32-byte PointXYZIRT records (floam_amd.POINT_DTYPE)")
        _ffi.check(self._L.floam_cloud_upload(self._h, a.ctypes.data_as(C.c_void_p), a.shape[0], 32))

    def __len__(self) -> int:
        n = C.c_size_t()
        _ffi.check(self._L.floam_cloud_size(self._h, C.byref(n)))
        return n.value

    def download(self) -> np.ndarray:
        n = len(self)
        out = np.zeros(n, POINT_DTYPE)
        got = C.c_size_t()
        _ffi.check(self._L.floam_cloud_download(self._h, out.ctypes.data_as(C.c_void_p), n, C.byref(got)))
        return out

    def clear(self) -> None:
        _ffi.check(self._L.floam_cloud_clear(self._h))

    def copy_from(self, other: "DeviceCloud") -> None:
        _ffi.check(self._L.floam_cloud_copy(self._h, other._h))

    def voxel_grid(self, leaf: float, out: "DeviceCloud | None" = None) -> "DeviceCloud":
        """pcl::VoxelGrid with a cubic leaf (PCL 1.8.1 semantics) into ``out`` (a new cloud by default)."""
        out = out if out is not None else DeviceCloud(device=self.device)
        _ffi.check(self._L.floam_voxel_grid(self._h, C.c_float(leaf), out._h))
        return out

    def device_ptr(self) -> int:
        return self._L.floam_cloud_device_ptr(self._h) or 0

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h:
            self._L.floam_cloud_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
