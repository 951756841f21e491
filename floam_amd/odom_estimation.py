"""OdomEstimationClass — host mirror of include/odomEstimationClass.h:52-126 over the C ABI.

Method names, argument meaning and update semantics follow the reference (src/odomEstimationClass.cpp); the
public members ``odom``, ``laserCloudCornerMap`` and ``laserCloudSurfMap`` are properties that read the device
state.  Clouds are ``DeviceCloud``s.  Non-fatal warnings (the reference's printf diagnostics) are kept in
``last_status``.
"""
from __future__ import annotations

import ctypes as C
from enum import IntEnum

import numpy as np

from . import _ffi
from .cloud import DeviceCloud
from .laser_processing import LidarParams


class UpdateType(IntEnum):   # include/odomEstimationClass.h:56
    VANILLA = 0
    INITIAL_ITERATION = 1
    REFINEMENT_AND_UPDATE = 2


def quat_to_matrix(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class OdomEstimationClass:
    VANILLA = UpdateType.VANILLA
    INITIAL_ITERATION = UpdateType.INITIAL_ITERATION
    REFINEMENT_AND_UPDATE = UpdateType.REFINEMENT_AND_UPDATE

    def __init__(self, device: int = 0):
        self._L = _ffi.load()
        self.device = device
        self._h = None
        self.last_status = _ffi.OK

    def init(self, lidar_param: LidarParams, map_resolution: float, loss_function: str) -> None:
        """OdomEstimationClass::init (src/odomEstimationClass.cpp:7-26)."""
        self.close()
        h = C.c_void_p()
        p = lidar_param.to_c()
        _ffi.check(self._L.floam_odom_create(C.byref(p), float(map_resolution), loss_function.encode(), self.device,
                                             C.byref(h)))
        self._h = h
        self.lidar_param = lidar_param

    def _need(self):
        if self._h is None:
            raise _ffi.FloamError(_ffi.ERR_INVALID_ARGUMENT, "OdomEstimationClass.init() not called")
        return self._h

    def initMapWithPoints(self, edge_in: DeviceCloud, surf_in: DeviceCloud) -> None:
        """src/odomEstimationClass.cpp:28-32"""
        _ffi.check(self._L.floam_odom_init_map(self._need(), edge_in.handle, surf_in.handle))

    def UpdatePointsToMapSelector(self, edge_in: DeviceCloud, surf_in: DeviceCloud, deskew: bool) -> int:
        """src/odomEstimationClass.cpp:34-50 (deskew velocity-compensates the clouds in place, Q5)."""
        self.last_status = _ffi.check(self._L.floam_odom_update_selector(self._need(), edge_in.handle,
                                                                          surf_in.handle, int(bool(deskew))))
        return self.last_status

    def UpdatePointsToMapSelectorHost(self, edge_in, surf_in, deskew: bool) -> int:
        """UpdatePointsToMapSelector on host clouds (POINT_DTYPE arrays, deskewed IN PLACE like the reference, Q5):
        floam_odom_update_selector_host, the drop-in adapter's one-call path (synchronous)."""
        from .synth import POINT_DTYPE
        for a in (edge_in, surf_in):
            if not (isinstance(a, np.ndarray) and a.dtype == POINT_DTYPE and a.flags["C_CONTIGUOUS"]):
                raise _ffi.FloamError(_ffi.ERR_INVALID_ARGUMENT, "host clouds must be contiguous POINT_DTYPE arrays")
        self.last_status = _ffi.check(self._L.floam_odom_update_selector_host(
            self._need(), edge_in.ctypes.data_as(C.c_void_p), edge_in.shape[0], surf_in.ctypes.data_as(C.c_void_p),
            surf_in.shape[0], 32, int(bool(deskew))))
        return self.last_status

    def updatePointsToMap(self, edge_in: DeviceCloud, surf_in: DeviceCloud,
                          update_type: UpdateType = UpdateType.VANILLA) -> int:
        """src/odomEstimationClass.cpp:52-124"""
        self.last_status = _ffi.check(self._L.floam_odom_update(self._need(), edge_in.handle, surf_in.handle,
                                                                 int(update_type)))
        return self.last_status

    def set_async(self, depth: int) -> int:
        """Streaming mode (floam_odom_set_async): with depth > 0 the update calls only issue device work, up to
        `depth` updates stay in flight, and wait() collects their poses and warnings."""
        return _ffi.check(self._L.floam_odom_set_async(self._need(), int(depth)))

    def wait(self, max_pending: int = 0) -> list:
        """Collect in-flight updates until at most max_pending remain; returns the (q_xyzw, t) pose of every update
        collected since the previous wait(), in issue order."""
        cap = 64
        buf = np.zeros((cap, 7))
        n = C.c_size_t()
        self.last_status = _ffi.check(self._L.floam_odom_wait(self._need(), int(max_pending),
                                                              buf.ctypes.data_as(C.POINTER(C.c_double)), cap,
                                                              C.byref(n)))
        return [(buf[i, :4].copy(), buf[i, 4:].copy()) for i in range(min(n.value, cap))]

    def getMap(self, laserCloudMap: DeviceCloud) -> None:
        """src/odomEstimationClass.cpp:296-300 (appends surf map, then corner map)."""
        _ffi.check(self._L.floam_odom_get_map(self._need(), laserCloudMap.handle))

    def GetVelocity(self) -> np.ndarray:
        """include/odomEstimationClass.h:78"""
        v = np.zeros(3)
        _ffi.check(self._L.floam_odom_get_velocity(self._need(), v.ctypes.data_as(C.POINTER(C.c_double))))
        return v

    def pose(self):
        """(q_xyzw, t) of the public member `odom`."""
        q, t = np.zeros(4), np.zeros(3)
        _ffi.check(self._L.floam_odom_get_pose(self._need(), q.ctypes.data_as(C.POINTER(C.c_double)),
                                               t.ctypes.data_as(C.POINTER(C.c_double))))
        return q, t

    def last_pose(self):
        q, t = np.zeros(4), np.zeros(3)
        _ffi.check(self._L.floam_odom_get_last_pose(self._need(), q.ctypes.data_as(C.POINTER(C.c_double)),
                                                    t.ctypes.data_as(C.POINTER(C.c_double))))
        return q, t

    @property
    def odom(self) -> np.ndarray:
        """Eigen::Isometry3d odom as a 4x4 matrix."""
        q, t = self.pose()
        T = np.eye(4)
        T[:3, :3] = quat_to_matrix(q)
        T[:3, 3] = t
        return T

    def map_sizes(self):
        a, b = C.c_size_t(), C.c_size_t()
        _ffi.check(self._L.floam_odom_get_map_sizes(self._need(), C.byref(a), C.byref(b)))
        return a.value, b.value

    def _maps(self):
        from .synth import POINT_DTYPE
        ne, ns = self.map_sizes()
        e = np.zeros(ne, POINT_DTYPE)
        s = np.zeros(ns, POINT_DTYPE)
        _ffi.check(self._L.floam_odom_download_maps(self._need(), e.ctypes.data_as(C.c_void_p), ne,
                                                    s.ctypes.data_as(C.c_void_p), ns))
        return e, s

    @property
    def laserCloudCornerMap(self) -> np.ndarray:
        return self._maps()[0]

    @property
    def laserCloudSurfMap(self) -> np.ndarray:
        return self._maps()[1]

    def stats(self) -> dict:
        s = _ffi.OdomStats()
        _ffi.check(self._L.floam_odom_get_stats(self._need(), C.byref(s)))
        return {k: getattr(s, k) for k, _ in _ffi.OdomStats._fields_}

    def KeyFrameUpdate(self, surf_cloud: DeviceCloud | None, edge_cloud: DeviceCloud | None, pose) -> bool:
        """include/odomEstimationClass.h:80 (src/odomEstimationClass.cpp:320-343): KeyFrameUpdate(surf_cloud,
        edge_cloud, pose) -> is `pose` a new keyframe; a keyframe joins the 3-deep history with copies of the clouds.
        `pose` is (q_xyzw, t) or a 4x4 matrix."""
        q, tt = _pose_qt(pose)
        flag = C.c_int()
        _ffi.check(self._L.floam_odom_keyframe_update(
            self._need(), surf_cloud.handle if surf_cloud is not None else None,
            edge_cloud.handle if edge_cloud is not None else None, q.ctypes.data_as(C.POINTER(C.c_double)),
            tt.ctypes.data_as(C.POINTER(C.c_double)), C.byref(flag)))
        return bool(flag.value)

    def keyframes(self) -> list:
        """The keyframe history keyframes_ (private in the reference, include/odomEstimationClass.h:117), oldest
        first: (q_xyzw, t, surf points, edge points); entries of the updates themselves have empty clouds."""
        n = C.c_size_t()
        _ffi.check(self._L.floam_odom_get_keyframe(self._need(), 0, None, None, None, None, C.byref(n)))
        out = []
        for i in range(n.value):
            q, t = np.zeros(4), np.zeros(3)
            s, e = DeviceCloud(device=self.device), DeviceCloud(device=self.device)
            _ffi.check(self._L.floam_odom_get_keyframe(self._need(), i, q.ctypes.data_as(C.POINTER(C.c_double)),
                                                       t.ctypes.data_as(C.POINTER(C.c_double)), s.handle, e.handle,
                                                       None))
            out.append((q, t, s.download(), e.download()))
        return out

    def set_precision(self, fp32, geometry: bool = False) -> None:
        """Residual / Jacobian precision (the C5 sweep, BASELINE.json configs[4]): fp32=False is the reference's fp64;
        fp32=True evaluates residuals, Jacobians and per-thread sums in float (fits and LM control in double);
        geometry=True also runs the line / plane fits in float."""
        level = _ffi.PRECISION_FP64
        if fp32:
            level = _ffi.PRECISION_FP32_GEOMETRY if geometry else _ffi.PRECISION_FP32
        _ffi.check(self._L.floam_odom_set_precision(self._need(), level))

    def set_trace(self, capacity: int) -> None:
        """Stage inspection: record every solve (up to `capacity`) and keep the last correspondence pass."""
        _ffi.check(self._L.floam_odom_set_trace(self._need(), int(capacity)))
        self._trace_cap = int(capacity)

    def traces(self) -> list:
        """The recorded solves since the last call (oracle.Odometry.traces() layout), then cleared."""
        cap = 4096
        buf = np.zeros((cap, _ffi.TRACE_WORDS))
        n = C.c_size_t()
        _ffi.check(self._L.floam_odom_get_traces(self._need(), buf.ctypes.data_as(C.POINTER(C.c_double)), cap,
                                                 C.byref(n)))
        if n.value > min(cap, getattr(self, "_trace_cap", cap)):
            raise _ffi.FloamError(_ffi.ERR_INVALID_ARGUMENT, f"{n.value} solves since the last call: trace truncated")
        out = []
        for b in buf[: min(n.value, cap)]:
            out.append(dict(n_edge_queries=int(b[0]), n_surf_queries=int(b[1]), n_edge_corr=int(b[2]),
                            n_surf_corr=int(b[3]), iterations=int(b[4]), successful=int(b[5]),
                            initial_cost=b[6], final_cost=b[7], x_in=b[8:15].copy(), x_out=b[15:22].copy(),
                            H0=b[22:43].copy(), g0=b[43:49].copy()))
        return out

    def find_correspondences(self, edge_in: DeviceCloud, surf_in: DeviceCloud, q_xyzw, t) -> None:
        """One correspondence pass at the pose (q, t) without a solve (stage inspection; needs set_trace)."""
        q = np.ascontiguousarray(q_xyzw, dtype=np.float64)
        tt = np.ascontiguousarray(t, dtype=np.float64)
        _ffi.check(self._L.floam_odom_find_correspondences(self._need(), edge_in.handle, surf_in.handle,
                                                           q.ctypes.data_as(C.POINTER(C.c_double)),
                                                           tt.ctypes.data_as(C.POINTER(C.c_double))))

    def correspondences(self, which: int) -> dict:
        """The last correspondence pass of set `which` (0 edge, 1 surf): queries, flags, neighbour indices and
        squared distances (n x 5), factor records (n x 9 edge / n x 7 surf)."""
        from .synth import POINT_DTYPE
        n = C.c_size_t()
        _ffi.check(self._L.floam_odom_get_correspondences(self._need(), int(which), None, None, None, None, None, 0,
                                                          C.byref(n)))
        k = n.value
        F = 9 if which == 0 else 7
        q = np.zeros(max(k, 1), POINT_DTYPE)
        fl = np.zeros(max(k, 1), np.uint8)
        idx = np.zeros((max(k, 1), 5), np.int32)
        sqd = np.zeros((max(k, 1), 5), np.float32)
        rec = np.zeros((max(k, 1), F))
        _ffi.check(self._L.floam_odom_get_correspondences(
            self._need(), int(which), q.ctypes.data_as(C.c_void_p), fl.ctypes.data_as(C.c_void_p),
            idx.ctypes.data_as(C.POINTER(C.c_int)), sqd.ctypes.data_as(C.POINTER(C.c_float)),
            rec.ctypes.data_as(C.POINTER(C.c_double)), k, C.byref(n)))
        return dict(queries=q[:k], flags=fl[:k], idx=idx[:k], sqd=sqd[:k], records=rec[:k])

    def set_shard(self, rank: int, world: int, unique_id: bytes | None) -> None:
        """Shard the correspondence queries over `world` ranks (one RCCL all-reduce per LM evaluation)."""
        buf = None
        if unique_id is not None:
            buf = C.create_string_buffer(bytes(unique_id), 128)
        _ffi.check(self._L.floam_odom_set_shard(self._need(), rank, world, buf))

    def set_shard_callback(self, rank: int, world: int, allreduce) -> None:
        """Shard with a host all-reduce: ``allreduce(values: np.ndarray[float64])`` sums in place over ranks
        (e.g. torch.distributed with gloo).  Validation mode for hosts where RCCL cannot run."""
        def _cb(ptr, n, _user):
            try:
                arr = np.ctypeslib.as_array(ptr, shape=(n,))
                allreduce(arr)
                return 0
            except Exception:   # reported as FLOAM_ERR_COMM by the library
                return 1
        self._ar_cb = _ffi.ALLREDUCE_FN(_cb)   # keep alive
        _ffi.check(self._L.floam_odom_set_shard_callback(self._need(), rank, world, self._ar_cb, None))

    def shard_exchange(self):
        """This rank's peer-sharding exchange buffer: (64-byte IPC handle for other processes, device pointer)."""
        h = C.create_string_buffer(64)
        ptr = C.c_void_p()
        _ffi.check(self._L.floam_odom_shard_exchange(self._need(), h, C.byref(ptr)))
        return h.raw, ptr.value

    def set_shard_peers(self, rank: int, world: int, handles=None, ptrs=None) -> None:
        """Peer sharding (one resident LM launch per solve; the ranks' sums exchanged through peer-mapped buffers):
        ``handles`` = every rank's 64-byte IPC handle (rank order; other processes) or ``ptrs`` = every rank's
        device pointer (handles in this process)."""
        hb = pp = None
        if handles is not None:
            assert len(handles) == world and all(len(h) == 64 for h in handles)
            hb = C.create_string_buffer(b"".join(bytes(h) for h in handles), 64 * world)
        if ptrs is not None:
            assert len(ptrs) == world
            pp = (C.c_void_p * world)(*ptrs)
        _ffi.check(self._L.floam_odom_set_shard_peers(self._need(), rank, world, hb, pp))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.floam_odom_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _pose_qt(pose):
    """(q_xyzw, t) from a (q, t) pair or a 4x4 isometry (numpy only: the branch on the largest of the trace and the
    diagonal keeps the division away from zero for any rotation, then the quaternion is normalised)."""
    if isinstance(pose, np.ndarray) and pose.shape == (4, 4):
        R = np.asarray(pose[:3, :3], dtype=np.float64)
        tr = R[0, 0] + R[1, 1] + R[2, 2]
        k = int(np.argmax([tr, R[0, 0], R[1, 1], R[2, 2]]))
        if k == 0:
            s = 2.0 * np.sqrt(1.0 + tr)
            q = [(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, s / 4.0]
        elif k == 1:
            s = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
            q = [s / 4.0, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s, (R[2, 1] - R[1, 2]) / s]
        elif k == 2:
            s = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
            q = [(R[0, 1] + R[1, 0]) / s, s / 4.0, (R[1, 2] + R[2, 1]) / s, (R[0, 2] - R[2, 0]) / s]
        else:
            s = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
            q = [(R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, s / 4.0, (R[1, 0] - R[0, 1]) / s]
        q = np.asarray(q, dtype=np.float64)
        q /= np.linalg.norm(q)
        return np.ascontiguousarray(q), np.ascontiguousarray(pose[:3, 3], dtype=np.float64)
    q, t = pose
    return np.ascontiguousarray(q, dtype=np.float64), np.ascontiguousarray(t, dtype=np.float64)


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    _ffi.check(_ffi.load().floam_comm_unique_id(buf))
    return buf.raw


def reset_process_state() -> None:
    """Reset KeyFrameUpdate's process-static `first` flag (src/odomEstimationClass.cpp:323, quirk Q6)."""
    _ffi.load().floam_reset_process_state()
