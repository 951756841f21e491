"""LaserProcessingClass — host mirror of include/laserProcessingClass.h:37-50 over the C ABI.

Same method names, argument meaning and append semantics as the reference; clouds are ``DeviceCloud``s
(device-resident 32-B PointXYZIRT records) instead of ``pcl::PointCloud<PointXYZIRT>::Ptr``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
from dataclasses import dataclass

from . import _ffi
from .cloud import DeviceCloud


@dataclass
class LidarParams:
    """lidar::Lidar (include/lidar.h:53-85): the fields the path reads."""
    num_lines: int = 64
    scan_period: float = 0.1
    vertical_angle: float = 2.0
    max_distance: float = 60.0
    min_distance: float = 2.0

    # setters of lidar::Lidar (src/lidar.cpp)
    def setLines(self, n):
        self.num_lines = int(n)

    def setScanPeriod(self, p):
        self.scan_period = float(p)

    def setVerticalAngle(self, a):
        self.vertical_angle = float(a)

    def setMaxDistance(self, d):
        self.max_distance = float(d)

    def setMinDistance(self, d):
        self.min_distance = float(d)

    def to_c(self) -> _ffi.LidarParams:
        return _ffi.LidarParams(self.num_lines, self.scan_period, self.vertical_angle, self.max_distance,
                                self.min_distance)


class LaserProcessingClass:
    def __init__(self, device: int = 0, asynchronous: bool = False):
        """asynchronous=True: featureExtraction does not synchronise (floam_lp_set_async); output sizes stay on the
        device and input-validation errors surface at the next odometry update that consumes the clouds (or at
        wait()).  Default False: the reference's synchronous behaviour."""
        self._L = _ffi.load()
        self.device = device
        self.asynchronous = asynchronous
        self._h = None

    def init(self, lidar_param: LidarParams) -> None:
        """LaserProcessingClass::init (src/laserProcessingClass.cpp:6-10)."""
        self.close()
        h = C.c_void_p()
        p = lidar_param.to_c()
        _ffi.check(self._L.floam_lp_create(C.byref(p), self.device, C.byref(h)))
        self._h = h
        self._lines = int(lidar_param.num_lines)
        if self.asynchronous:
            _ffi.check(self._L.floam_lp_set_async(self._h, 1))

    def wait(self) -> None:
        """Synchronise and raise the validation error of the last asynchronous featureExtraction, if any."""
        if self._h is not None:
            _ffi.check(self._L.floam_lp_wait(self._h))

    def featureExtraction(self, pc_in: DeviceCloud, pc_out_edge: DeviceCloud, pc_out_surf: DeviceCloud) -> None:
        """LaserProcessingClass::featureExtraction (src/laserProcessingClass.cpp:72-118): appends edge / surf
        features of pc_in to pc_out_edge / pc_out_surf (never clears them, like the reference)."""
        if self._h is None:
            raise _ffi.FloamError(_ffi.ERR_INVALID_ARGUMENT, "LaserProcessingClass.init() not called")
        _ffi.check(self._L.floam_lp_feature_extraction(self._h, pc_in.handle, pc_out_edge.handle, pc_out_surf.handle))

    def featureExtractionHost(self, points):
        """featureExtraction on a host cloud (POINT_DTYPE array, what the processing node holds): returns the
        (edge, surf) feature arrays — floam_lp_feature_extraction_host, the drop-in adapter's one-call path."""
        from .synth import POINT_DTYPE
        if self._h is None:
            raise _ffi.FloamError(_ffi.ERR_INVALID_ARGUMENT, "LaserProcessingClass.init() not called")
        a = np.ascontiguousarray(points, dtype=POINT_DTYPE)
        n = a.shape[0]
        edge = np.zeros(max(1, min(n, self._lines * 120)), POINT_DTYPE)
        surf = np.zeros(max(1, n), POINT_DTYPE)
        ne, ns = C.c_size_t(), C.c_size_t()
        _ffi.check(self._L.floam_lp_feature_extraction_host(
            self._h, a.ctypes.data_as(C.c_void_p), n, 32, edge.ctypes.data_as(C.c_void_p), edge.shape[0],
            C.byref(ne), surf.ctypes.data_as(C.c_void_p), surf.shape[0], C.byref(ns)))
        return edge[: ne.value].copy(), surf[: ns.value].copy()

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.floam_lp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
