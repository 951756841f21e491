"""IMU pre-processing of the laser-processing node — host mirror of dmapping (include/dataHandler.h,
src/dataHandler.cpp) and of the node's CenterTime / IMU alignment (src/laserProcessingNode.cpp:65-120) over the C ABI.

Same names and argument meaning as the reference: ``ImuHandler.AddMsg / Get / TimeContained / size``,
``CenterTime(cloud, stamp)``, ``Compensate(input, compensated, handler, extrinsics) -> bool`` and
``euler2Quaternion``.  Quaternions are (x, y, z, w) numpy arrays (Eigen::Quaterniond coefficient order); stamps are
seconds, cloud stamps PCL microsecond stamps (the reference keeps them in ``cloud->header.stamp``).
``preprocess`` is the node's whole sequence (CenterTime, Compensate, ImuNowT alignment) fused into one device pass.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi
from .cloud import DeviceCloud

_dp = C.POINTER(C.c_double)


def _d(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def euler2Quaternion(roll: float, pitch: float, yaw: float) -> np.ndarray:
    """euler2Quaternion (src/lidar.cpp:8-16), degrees -> (x, y, z, w)."""
    q = np.zeros(4)
    _ffi.check(_ffi.load().floam_euler_to_quaternion(float(roll), float(pitch), float(yaw), q.ctypes.data_as(_dp)))
    return q


class ImuHandler:
    """dmapping::ImuHandler (include/dataHandler.h:31-66) on GPU ``device`` (orientation stream in HBM)."""

    def __init__(self, device: int = 0):
        self._L = _ffi.load()
        self.device = device
        h = C.c_void_p()
        _ffi.check(self._L.floam_imu_create(device, C.byref(h)))
        self._h = h

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def AddMsg(self, stamp: float, orientation_xyzw) -> bool:
        """ImuHandler::AddMsg (src/dataHandler.cpp:23-38): dropped unless stamp > last + 1e-5 s."""
        q = _d(orientation_xyzw)
        added = C.c_int()
        _ffi.check(self._L.floam_imu_add_msg(self._h, float(stamp), q.ctypes.data_as(_dp), C.byref(added)))
        return bool(added.value)

    def add_msgs(self, stamps, orientations_xyzw) -> int:
        """AddMsg over a batch of messages (in order); returns how many were appended."""
        s, q = _d(stamps), _d(orientations_xyzw).reshape(-1, 4)
        if s.shape[0] != q.shape[0]:
            raise ValueError("stamps and orientations differ in length")
        added = C.c_size_t()
        _ffi.check(self._L.floam_imu_add_msgs(self._h, s.ctypes.data_as(_dp), q.ctypes.data_as(_dp), s.shape[0],
                                              C.byref(added)))
        return added.value

    def Get(self, stamp: float):
        """ImuHandler::Get (src/dataHandler.cpp:48-75): (orientation_xyzw, found); zero orientation if not found."""
        q = np.zeros(4)
        found = C.c_int()
        _ffi.check(self._L.floam_imu_get(self._h, float(stamp), q.ctypes.data_as(_dp), C.byref(found)))
        return q, bool(found.value)

    def TimeContained(self, stamp: float) -> bool:
        """ImuHandler::TimeContained (src/dataHandler.cpp:76-81)."""
        c = C.c_int()
        _ffi.check(self._L.floam_imu_time_contained(self._h, float(stamp), C.byref(c)))
        return bool(c.value)

    def size(self) -> int:
        n = C.c_size_t()
        _ffi.check(self._L.floam_imu_size(self._h, C.byref(n)))
        return n.value

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h:
            self._L.floam_imu_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def CenterTime(cloud: DeviceCloud, stamp_us: int) -> int:
    """CenterTime (src/laserProcessingNode.cpp:65-78): re-references the point times to the scan centre in place
    and returns the centred PCL stamp (microseconds)."""
    st = C.c_uint64(int(stamp_us))
    _ffi.check(_ffi.load().floam_center_time(cloud.handle, C.byref(st)))
    return int(st.value)


def Compensate(input: DeviceCloud, compensated: DeviceCloud, handler: ImuHandler, extrinsics_xyzw,
               stamp_us: int) -> bool:
    """dmapping::Compensate (src/dataHandler.cpp:93-122).  The reference reads the stamp from input->header;
    here it is passed explicitly.  False ("no imu data") when the scan's ends are outside the IMU stream."""
    e = _d(extrinsics_xyzw)
    rc = _ffi.check(_ffi.load().floam_imu_compensate(handler.handle, input.handle, C.c_uint64(int(stamp_us)),
                                                      e.ctypes.data_as(_dp), compensated.handle))
    return rc != _ffi.WARN_NO_IMU_DATA


def preprocess(cloud: DeviceCloud, stamp_us: int, handler: ImuHandler, extrinsics_xyzw, aligned: DeviceCloud):
    """The laser-processing node's sequence before featureExtraction (src/laserProcessingNode.cpp:92-113):
    CenterTime(cloud) in place, Compensate, IMU alignment by Affine3d(q(Get(stamp)) * extrinsics) into ``aligned``.
    Returns (ok, centred stamp); ok False is the node's "cannot compensate - no IMU data" skip."""
    e = _d(extrinsics_xyzw)
    st = C.c_uint64(int(stamp_us))
    rc = _ffi.check(_ffi.load().floam_imu_preprocess(handler.handle, cloud.handle, C.byref(st),
                                                      e.ctypes.data_as(_dp), aligned.handle))
    return rc != _ffi.WARN_NO_IMU_DATA, int(st.value)
