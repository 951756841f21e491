"""CPU ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg).

ctypes bindings over oracle/liboracle.so, the single-threaded C++ restatement of the FLOAM hot path
(see oracle/oracle.hpp for the reference file:line map).  PARITY UNPINNED: the reference has no tests or
fixtures and cannot be built here; the oracle is pinned by numpy/scipy cross-checks, known-answer tests and
its own committed golden vectors (tests/golden/).

Never imported by the product package ``floam_amd``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

c_double_p = C.POINTER(C.c_double)
c_float_p = C.POINTER(C.c_float)
c_int_p = C.POINTER(C.c_int)
c_size_p = C.POINTER(C.c_size_t)


def build(force: bool = False) -> str:
    so = os.path.join(_HERE, "liboracle.so")
    if force or not os.path.exists(so):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return so


def lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(so):
            build()
        L = C.CDLL(so)
        L.oracle_feature_extraction.argtypes = [C.c_int, C.c_double, C.c_double, C.c_void_p, C.c_size_t, C.c_int,
                                                C.c_void_p, c_size_p, C.c_void_p, c_size_p, c_size_p]
        L.oracle_feature_extraction.restype = C.c_int
        L.oracle_voxel_grid.argtypes = [C.c_void_p, C.c_size_t, C.c_float, C.c_int, C.c_void_p, c_size_p]
        L.oracle_voxel_grid.restype = C.c_int
        L.oracle_crop_box.argtypes = [C.c_void_p, C.c_size_t, c_float_p, c_float_p, C.c_void_p, c_size_p]
        L.oracle_crop_box.restype = C.c_int
        L.oracle_knn.argtypes = [C.c_void_p, C.c_size_t, c_float_p, C.c_size_t, C.c_int, c_int_p, c_float_p]
        L.oracle_eig_sym3.argtypes = [c_double_p, c_double_p, c_double_p]
        L.oracle_plane_solve.argtypes = [c_double_p, c_double_p]
        L.oracle_odom_create.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, C.c_char_p,
                                         C.c_int]
        L.oracle_odom_create.restype = C.c_void_p
        for name in ("oracle_odom_destroy", "oracle_odom_clear_traces"):
            getattr(L, name).argtypes = [C.c_void_p]
        L.oracle_odom_init_map.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.oracle_odom_update_selector.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                                  C.c_int]
        L.oracle_odom_update.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        L.oracle_odom_get_pose.argtypes = [C.c_void_p, c_double_p, c_double_p]
        L.oracle_odom_get_last_pose.argtypes = [C.c_void_p, c_double_p, c_double_p]
        L.oracle_odom_get_velocity.argtypes = [C.c_void_p, c_double_p]
        L.oracle_odom_map_size.argtypes = [C.c_void_p, C.c_int]
        L.oracle_odom_map_size.restype = C.c_size_t
        L.oracle_odom_get_map.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_odom_optimization_count.argtypes = [C.c_void_p]
        L.oracle_odom_optimization_count.restype = C.c_int
        L.oracle_odom_num_traces.argtypes = [C.c_void_p]
        L.oracle_odom_num_traces.restype = C.c_size_t
        L.oracle_odom_get_trace.argtypes = [C.c_void_p, C.c_size_t, c_double_p]
        L.oracle_reset_process_statics.argtypes = []
        L.oracle_stage_correspondences.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, c_double_p,
                                                   C.c_int, c_int_p, c_float_p, C.c_void_p, c_double_p]
        L.oracle_stage_associate.argtypes = [C.c_void_p, C.c_size_t, c_double_p, C.c_void_p]
        L.oracle_stage_solve.argtypes = [c_double_p, C.c_size_t, c_double_p, C.c_size_t, C.c_int, c_double_p,
                                         c_double_p]
        L.oracle_edge_residual.argtypes = [c_double_p] * 5
        L.oracle_edge_residual.restype = C.c_double
        L.oracle_surf_residual.argtypes = [c_double_p, c_double_p, C.c_double, c_double_p, c_double_p]
        L.oracle_surf_residual.restype = C.c_double
        L.oracle_se3_plus.argtypes = [c_double_p] * 3
        L.oracle_imu_filter.argtypes = [c_double_p, C.c_size_t, C.c_void_p]
        L.oracle_imu_filter.restype = C.c_size_t
        L.oracle_imu_get.argtypes = [c_double_p, c_double_p, C.c_size_t, C.c_double, c_double_p]
        L.oracle_imu_get.restype = C.c_int
        L.oracle_imu_time_contained.argtypes = [c_double_p, c_double_p, C.c_size_t, C.c_double]
        L.oracle_imu_time_contained.restype = C.c_int
        L.oracle_euler_to_quaternion.argtypes = [C.c_double, C.c_double, C.c_double, c_double_p]
        L.oracle_center_time.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64)]
        L.oracle_imu_preprocess.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint64), c_double_p,
                                            c_double_p, C.c_size_t, c_double_p, C.c_void_p]
        L.oracle_imu_preprocess.restype = C.c_int
        L.oracle_from_pointcloud2.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                              C.c_void_p, C.c_size_t, C.c_void_p]
        L.oracle_from_pointcloud2.restype = C.c_int
        L.oracle_transform_cloud.argtypes = [C.c_void_p, C.c_size_t, c_double_p, C.c_void_p]
        L.oracle_mapping_create.argtypes = [C.c_double, C.c_int]
        L.oracle_mapping_create.restype = C.c_void_p
        L.oracle_mapping_destroy.argtypes = [C.c_void_p]
        L.oracle_mapping_update.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, c_double_p, c_double_p]
        L.oracle_mapping_size.argtypes = [C.c_void_p]
        L.oracle_mapping_size.restype = C.c_size_t
        L.oracle_mapping_get_map.argtypes = [C.c_void_p, C.c_void_p]
        _LIB = L
    return _LIB


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _as_points(a: np.ndarray) -> np.ndarray:
    from floam_amd.synth import POINT_DTYPE
    a = np.ascontiguousarray(a)
    assert a.dtype.itemsize == 32, a.dtype
    return a.view(POINT_DTYPE) if a.dtype != POINT_DTYPE else a


def feature_extraction(points: np.ndarray, num_lines: int, min_dis: float = 0.5, max_dis: float = 90.0,
                       canonical: bool = False):
    """LaserProcessingClass::featureExtraction (src/laserProcessingClass.cpp:72-118).
    Returns (edge, surf, stats) with stats = (out_of_range_ring_points, sector_ties)."""
    from floam_amd.synth import POINT_DTYPE
    pts = _as_points(points)
    n = pts.shape[0]
    e = np.zeros(n, POINT_DTYPE)
    s = np.zeros(n, POINT_DTYPE)
    ne, ns = C.c_size_t(n), C.c_size_t(n)
    st = (C.c_size_t * 2)()
    rc = lib().oracle_feature_extraction(num_lines, min_dis, max_dis, _ptr(pts), n, int(canonical), _ptr(e),
                                         C.byref(ne), _ptr(s), C.byref(ns), st)
    assert rc == 0
    return e[: ne.value].copy(), s[: ns.value].copy(), (st[0], st[1])


def voxel_grid(points: np.ndarray, leaf: float, stable: bool = True) -> np.ndarray:
    from floam_amd.synth import POINT_DTYPE
    pts = _as_points(points)
    n = pts.shape[0]
    out = np.zeros(max(n, 1), POINT_DTYPE)
    no = C.c_size_t(max(n, 1))
    rc = lib().oracle_voxel_grid(_ptr(pts), n, C.c_float(leaf), int(stable), _ptr(out), C.byref(no))
    assert rc == 0
    return out[: no.value].copy()


def crop_box(points: np.ndarray, mn, mx) -> np.ndarray:
    from floam_amd.synth import POINT_DTYPE
    pts = _as_points(points)
    n = pts.shape[0]
    out = np.zeros(max(n, 1), POINT_DTYPE)
    no = C.c_size_t(max(n, 1))
    a = (C.c_float * 3)(*mn)
    b = (C.c_float * 3)(*mx)
    rc = lib().oracle_crop_box(_ptr(pts), n, a, b, _ptr(out), C.byref(no))
    assert rc == 0
    return out[: no.value].copy()


def knn(map_points: np.ndarray, queries: np.ndarray, k: int = 5):
    """KdTreeFLANN nearestKSearch restated. queries: (n, 3) float32. Returns (idx (n,k) int32, sqd (n,k) f32)."""
    mp = _as_points(map_points)
    q = np.ascontiguousarray(queries, dtype=np.float32)
    nq = q.shape[0]
    idx = np.full((nq, k), -1, np.int32)
    sqd = np.full((nq, k), np.inf, np.float32)
    lib().oracle_knn(_ptr(mp), mp.shape[0], q.ctypes.data_as(c_float_p), nq, k, idx.ctypes.data_as(c_int_p),
                     sqd.ctypes.data_as(c_float_p))
    return idx, sqd


def eig_sym3(a: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(9)
    ev = np.zeros(3)
    vec = np.zeros(9)
    lib().oracle_eig_sym3(a.ctypes.data_as(c_double_p), ev.ctypes.data_as(c_double_p),
                          vec.ctypes.data_as(c_double_p))
    return ev, vec.reshape(3, 3).T   # columns = eigenvectors


def plane_solve(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(15)
    x = np.zeros(3)
    lib().oracle_plane_solve(a.ctypes.data_as(c_double_p), x.ctypes.data_as(c_double_p))
    return x


class Odometry:
    """OdomEstimationClass restated (src/odomEstimationClass.cpp).  Poses are (q_xyzw, t)."""

    VANILLA, INITIAL_ITERATION, REFINEMENT_AND_UPDATE = 0, 1, 2

    def __init__(self, num_lines: int, scan_period: float = 0.1, min_dis: float = 0.5, max_dis: float = 90.0,
                 map_resolution: float = 0.1, loss: str = "Cauchy", stable_voxel: bool = True):
        self._L = lib()
        self._h = self._L.oracle_odom_create(num_lines, scan_period, min_dis, max_dis, map_resolution,
                                             loss.encode(), int(stable_voxel))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.oracle_odom_destroy(h)
            self._h = None

    def init_map(self, edge: np.ndarray, surf: np.ndarray):
        e, s = _as_points(edge), _as_points(surf)
        self._L.oracle_odom_init_map(self._h, _ptr(e), e.shape[0], _ptr(s), s.shape[0])

    def update_selector(self, edge: np.ndarray, surf: np.ndarray, deskew: bool = True):
        """Mutates edge/surf in place when deskew (Q5)."""
        assert edge.flags.c_contiguous and surf.flags.c_contiguous
        self._L.oracle_odom_update_selector(self._h, _ptr(edge), edge.shape[0], _ptr(surf), surf.shape[0],
                                            int(deskew))

    def update(self, edge: np.ndarray, surf: np.ndarray, update_type: int = 0):
        e, s = _as_points(edge), _as_points(surf)
        self._L.oracle_odom_update(self._h, _ptr(e), e.shape[0], _ptr(s), s.shape[0], update_type)

    def pose(self):
        q, t = np.zeros(4), np.zeros(3)
        self._L.oracle_odom_get_pose(self._h, q.ctypes.data_as(c_double_p), t.ctypes.data_as(c_double_p))
        return q, t

    def last_pose(self):
        q, t = np.zeros(4), np.zeros(3)
        self._L.oracle_odom_get_last_pose(self._h, q.ctypes.data_as(c_double_p), t.ctypes.data_as(c_double_p))
        return q, t

    def velocity(self):
        v = np.zeros(3)
        self._L.oracle_odom_get_velocity(self._h, v.ctypes.data_as(c_double_p))
        return v

    def map(self, which: int) -> np.ndarray:
        from floam_amd.synth import POINT_DTYPE
        n = self._L.oracle_odom_map_size(self._h, which)
        out = np.zeros(n, POINT_DTYPE)
        if n:
            self._L.oracle_odom_get_map(self._h, which, _ptr(out))
        return out

    @property
    def optimization_count(self) -> int:
        return self._L.oracle_odom_optimization_count(self._h)

    def traces(self):
        n = self._L.oracle_odom_num_traces(self._h)
        out = []
        for i in range(n):
            b = np.zeros(49)
            self._L.oracle_odom_get_trace(self._h, i, b.ctypes.data_as(c_double_p))
            out.append(_trace_dict(b))
        return out

    def clear_traces(self):
        self._L.oracle_odom_clear_traces(self._h)


def _trace_dict(b):
    return dict(n_edge_queries=int(b[0]), n_surf_queries=int(b[1]), n_edge_corr=int(b[2]), n_surf_corr=int(b[3]),
                iterations=int(b[4]), successful=int(b[5]), initial_cost=b[6], final_cost=b[7], x_in=b[8:15].copy(),
                x_out=b[15:22].copy(), H0=b[22:43].copy(), g0=b[43:49].copy())


def stage_correspondences(map_points: np.ndarray, queries: np.ndarray, x, edge: bool):
    """One correspondence pass (src/odomEstimationClass.cpp:144-251): pointAssociateToMap at parameters x
    (qx, qy, qz, qw, tx, ty, tz), KD-tree 5-NN, the sqd[4] < 1 gate, line / plane geometry.  Returns dict(idx (n, 5),
    sqd (n, 5), flags (n,) bit 0 factor kept / bit 2 gate passed, records (n, 9 edge | 7 surf))."""
    mp, q = _as_points(map_points), _as_points(queries)
    n = q.shape[0]
    F = 9 if edge else 7
    idx = np.full((max(n, 1), 5), -1, np.int32)
    sqd = np.full((max(n, 1), 5), np.inf, np.float32)
    flags = np.zeros(max(n, 1), np.uint8)
    rec = np.zeros((max(n, 1), F))
    xx = np.ascontiguousarray(x, dtype=np.float64)
    lib().oracle_stage_correspondences(_ptr(mp), mp.shape[0], _ptr(q), n, xx.ctypes.data_as(c_double_p), int(edge),
                                       idx.ctypes.data_as(c_int_p), sqd.ctypes.data_as(c_float_p), _ptr(flags),
                                       rec.ctypes.data_as(c_double_p))
    return dict(idx=idx[:n], sqd=sqd[:n], flags=flags[:n], records=rec[:n])


def associate_to_map(points: np.ndarray, x) -> np.ndarray:
    """pointAssociateToMap (src/odomEstimationClass.cpp:126-135) at parameters x: double math, float result."""
    p = _as_points(points)
    out = np.zeros_like(p)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    lib().oracle_stage_associate(_ptr(p), p.shape[0], xx.ctypes.data_as(c_double_p), _ptr(out))
    return out


def stage_solve(edge_records: np.ndarray, surf_records: np.ndarray, x, huber: bool = False):
    """ceres::Solve (src/odomEstimationClass.cpp:95-108) on given factor records from parameters x.
    Returns (x_out, trace dict as Odometry.traces())."""
    e = np.ascontiguousarray(edge_records, dtype=np.float64).reshape(-1, 9)
    s = np.ascontiguousarray(surf_records, dtype=np.float64).reshape(-1, 7)
    xx = np.array(x, dtype=np.float64)
    tr = np.zeros(49)
    lib().oracle_stage_solve(e.ctypes.data_as(c_double_p), e.shape[0], s.ctypes.data_as(c_double_p), s.shape[0],
                             int(huber), xx.ctypes.data_as(c_double_p), tr.ctypes.data_as(c_double_p))
    return xx, _trace_dict(tr)


def reset_process_statics():
    lib().oracle_reset_process_statics()


def _dptr(a):
    return a.ctypes.data_as(c_double_p)


def edge_residual(cp, a, b, x):
    """EdgeAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:12-43): (r, J over the 6 local params)."""
    L = lib()
    J = np.zeros(7)
    v = [np.ascontiguousarray(t, dtype=np.float64) for t in (cp, a, b, x)]
    r = L.oracle_edge_residual(_dptr(v[0]), _dptr(v[1]), _dptr(v[2]), _dptr(v[3]), _dptr(J))
    return r, J[:6]


def surf_residual(cp, n, d, x):
    """SurfNormAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:51-74)."""
    L = lib()
    J = np.zeros(7)
    v = [np.ascontiguousarray(t, dtype=np.float64) for t in (cp, n, x)]
    r = L.oracle_surf_residual(_dptr(v[0]), _dptr(v[1]), float(d), _dptr(v[2]), _dptr(J))
    return r, J[:6]


def se3_plus(x, delta):
    """PoseSE3Parameterization::Plus (src/lidarOptimization.cpp:77-92)."""
    out = np.zeros(7)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    dd = np.ascontiguousarray(delta, dtype=np.float64)
    lib().oracle_se3_plus(_dptr(xx), _dptr(dd), _dptr(out))
    return out


# ------------------------------------------------------------------ IMU pre-processing (oracle/imu.cpp, §8 f-2)
def imu_filter(stamps) -> np.ndarray:
    """ImuHandler::AddMsg over a message stream (src/dataHandler.cpp:23-38): mask of the messages kept."""
    st = np.ascontiguousarray(stamps, dtype=np.float64)
    keep = np.zeros(st.shape[0], np.uint8)
    lib().oracle_imu_filter(_dptr(st), st.shape[0], _ptr(keep))
    return keep.astype(bool)


def imu_get(stamps, q_xyzw, t: float):
    """ImuHandler::Get (src/dataHandler.cpp:48-75) over the handler built from (stamps, q) with AddMsg.
    Returns (q_xyzw, found); q is all zero when not found (default-constructed sensor_msgs::Imu)."""
    st = np.ascontiguousarray(stamps, dtype=np.float64)
    q = np.ascontiguousarray(q_xyzw, dtype=np.float64).reshape(-1, 4)
    out = np.zeros(4)
    found = lib().oracle_imu_get(_dptr(st), _dptr(q), st.shape[0], float(t), _dptr(out))
    return out, bool(found)


def imu_time_contained(stamps, q_xyzw, t: float) -> bool:
    st = np.ascontiguousarray(stamps, dtype=np.float64)
    q = np.ascontiguousarray(q_xyzw, dtype=np.float64).reshape(-1, 4)
    return bool(lib().oracle_imu_time_contained(_dptr(st), _dptr(q), st.shape[0], float(t)))


def euler_to_quaternion(roll: float, pitch: float, yaw: float) -> np.ndarray:
    """euler2Quaternion (src/lidar.cpp:8-16), degrees -> (x, y, z, w)."""
    out = np.zeros(4)
    lib().oracle_euler_to_quaternion(float(roll), float(pitch), float(yaw), _dptr(out))
    return out


def center_time(points: np.ndarray, stamp_us: int):
    """CenterTime (src/laserProcessingNode.cpp:65-78) on a copy.  Returns (points, new stamp in microseconds)."""
    p = _as_points(points).copy()
    st = C.c_uint64(int(stamp_us))
    lib().oracle_center_time(_ptr(p), p.shape[0], C.byref(st))
    return p, int(st.value)


def imu_preprocess(points: np.ndarray, stamp_us: int, stamps, q_xyzw, extrinsics_xyzw, mode: int = 7):
    """mode 7: the laser-processing node's CenterTime + Compensate + IMU alignment (src/laserProcessingNode.cpp:
    92-120); mode 2: dmapping::Compensate alone (src/dataHandler.cpp:93-122).  Works on a copy of `points`.
    Returns (ok, in_after (centred for mode 7), out, stamp_us)."""
    from floam_amd.synth import POINT_DTYPE
    p = _as_points(points).copy()
    out = np.zeros(p.shape[0], POINT_DTYPE)
    st = C.c_uint64(int(stamp_us))
    s = np.ascontiguousarray(stamps, dtype=np.float64)
    q = np.ascontiguousarray(q_xyzw, dtype=np.float64).reshape(-1, 4)
    e = np.ascontiguousarray(extrinsics_xyzw, dtype=np.float64)
    ok = lib().oracle_imu_preprocess(int(mode), _ptr(p), p.shape[0], C.byref(st), _dptr(s), _dptr(q), s.shape[0],
                                     _dptr(e), _ptr(out))
    return bool(ok), p, out, int(st.value)


# ------------------------------------------------------------------ wire formats (oracle/formats.cpp, §8 f-3)
PC2_FIELD_DTYPE = np.dtype({"names": ["name", "offset", "datatype", "count"],
                            "formats": ["S32", "<u4", "u1", "<u4"], "offsets": [0, 32, 36, 40], "itemsize": 44})


def from_pointcloud2(data: bytes, width: int, height: int, point_step: int, row_step: int, fields,
                     point_type: int = 0):
    """pcl::fromROSMsg / fromPCLPointCloud2 restated.  fields: [(name, offset, datatype, count)].
    Returns (points, number of point fields without a match)."""
    from floam_amd.synth import POINT_DTYPE
    f = np.zeros(max(1, len(fields)), PC2_FIELD_DTYPE)
    for i, (nm, off, dt, cnt) in enumerate(fields):
        f[i] = (nm.encode(), off, dt, cnt)
    buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(max(1, width * height), POINT_DTYPE)
    miss = lib().oracle_from_pointcloud2(point_type, _ptr(buf), width, height, point_step, row_step, _ptr(f),
                                         len(fields), _ptr(out))
    return out[: width * height].copy(), miss


def transform_cloud(points: np.ndarray, T) -> np.ndarray:
    """pcl::transformPointCloud with a double Affine3d (row-major 4x4)."""
    p = _as_points(points)
    out = np.zeros_like(p)
    m = np.ascontiguousarray(T, dtype=np.float64).reshape(16)
    lib().oracle_transform_cloud(_ptr(p), p.shape[0], _dptr(m), _ptr(out))
    return out


class Mapping:
    """LaserMappingClass restated (oracle/mapping.cpp, src/laserMappingClass.cpp).  Poses are (q_xyzw, t)."""

    def __init__(self, map_resolution: float = 0.4, stable_voxel: bool = True):
        self._L = lib()
        self._h = self._L.oracle_mapping_create(float(map_resolution), int(stable_voxel))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.oracle_mapping_destroy(h)
            self._h = None

    def update(self, points: np.ndarray, q_xyzw, t):
        p = _as_points(points)
        q = np.ascontiguousarray(q_xyzw, dtype=np.float64)
        tt = np.ascontiguousarray(t, dtype=np.float64)
        self._L.oracle_mapping_update(self._h, _ptr(p), p.shape[0], _dptr(q), _dptr(tt))

    def get_map(self) -> np.ndarray:
        from floam_amd.synth import POINT_DTYPE
        n = self._L.oracle_mapping_size(self._h)
        out = np.zeros(n, POINT_DTYPE)
        if n:
            self._L.oracle_mapping_get_map(self._h, _ptr(out))
        return out
