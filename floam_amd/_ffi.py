"""ctypes binding of libfloam_amd.so (the C ABI in include/floam_c.h).

The product path has no CPU fallback: if the HIP library is missing, or no gfx950 device is present, every call
raises ``FloamError`` loudly.  Loading the library itself needs no GPU (symbol checks run in CPU-only CI).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FLOAM_AMD_LIB=diag selects the diagnostic build of the same sources (libfloam_amd_diag.so: the A/B, stamp and
# test-hook environment variables, floam_amd/csrc/floam_common.hpp FLOAM_DIAG_ENV) — for the tests that need a hook
# and for measurement scripts; the product library reads only FLOAM_GRAPH and FLOAM_MAP_MERGE
PRODUCT_LIB_PATH = os.path.join(_HERE, "libfloam_amd.so")
DIAG_LIB_PATH = os.path.join(_HERE, "libfloam_amd_diag.so")
LIB_PATH = PRODUCT_LIB_PATH


def lib_path() -> str:
    """The library load() opens: the diagnostic build when FLOAM_AMD_LIB=diag, else the product library."""
    return DIAG_LIB_PATH if os.environ.get("FLOAM_AMD_LIB") == "diag" else PRODUCT_LIB_PATH

# floam_status (include/floam_c.h)
ABI_VERSION = 3   # FLOAM_ABI_VERSION of include/floam_c.h this package binds
OK = 0
ERR_INVALID_ARGUMENT = 1
ERR_DEVICE = 2
ERR_OUT_OF_MEMORY = 3
ERR_UNSUPPORTED = 4
ERR_COMM = 5
WARN_MAP_TOO_SMALL = 100
WARN_FEW_CORRESPONDENCES = 101
WARN_NO_IMU_DATA = 102
WARN_FIELD_MISSING = 103

STATUS_NAMES = {0: "OK", 1: "ERR_INVALID_ARGUMENT", 2: "ERR_DEVICE", 3: "ERR_OUT_OF_MEMORY", 4: "ERR_UNSUPPORTED",
                5: "ERR_COMM", 100: "WARN_MAP_TOO_SMALL", 101: "WARN_FEW_CORRESPONDENCES",
                102: "WARN_NO_IMU_DATA", 103: "WARN_FIELD_MISSING"}

# every entry point include/floam_c.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "floam_cloud_create", "floam_cloud_destroy", "floam_cloud_upload", "floam_cloud_download", "floam_cloud_size",
    "floam_cloud_clear", "floam_cloud_copy", "floam_cloud_device_ptr",
    "floam_lp_create", "floam_lp_destroy", "floam_lp_feature_extraction", "floam_lp_set_async", "floam_lp_wait",
    "floam_voxel_grid",
    "floam_odom_create", "floam_odom_destroy", "floam_odom_init_map", "floam_odom_update_selector",
    "floam_odom_update", "floam_odom_get_pose", "floam_odom_get_last_pose", "floam_odom_get_velocity",
    "floam_odom_get_map", "floam_odom_get_map_sizes", "floam_odom_download_maps", "floam_odom_get_stats",
    "floam_odom_set_async", "floam_odom_wait", "floam_odom_keyframe_update", "floam_odom_get_keyframe",
    "floam_odom_set_precision",
    "floam_odom_set_trace", "floam_odom_get_traces", "floam_odom_get_correspondences",
    "floam_odom_find_correspondences",
    "floam_comm_unique_id", "floam_odom_set_shard", "floam_odom_set_shard_callback",
    "floam_odom_shard_exchange", "floam_odom_set_shard_peers",
    "floam_lp_feature_extraction_host", "floam_odom_update_selector_host",
    "floam_last_error", "floam_version", "floam_abi_version", "floam_reset_process_state", "floam_device_synchronize",
    "floam_profile_enable", "floam_profile_read", "floam_profile_reset", "floam_profile_mark",
    "floam_imu_create", "floam_imu_destroy", "floam_imu_add_msg", "floam_imu_add_msgs", "floam_imu_size",
    "floam_imu_get", "floam_imu_time_contained", "floam_euler_to_quaternion", "floam_center_time",
    "floam_imu_compensate", "floam_imu_preprocess",
    "floam_pointcloud2_fields", "floam_cloud_from_pointcloud2", "floam_transform_cloud",
    "floam_mapping_create", "floam_mapping_destroy", "floam_mapping_update", "floam_mapping_get_map",
    "floam_mapping_size",
    "floam_save_pcd", "floam_save_odom", "floam_save_posegraph", "floam_save_poses_balm", "floam_save_merged",
]


class FloamError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class LidarParams(C.Structure):
    _fields_ = [("num_lines", C.c_int), ("scan_period", C.c_double), ("vertical_angle", C.c_double),
                ("max_distance", C.c_double), ("min_distance", C.c_double)]


class OdomStats(C.Structure):
    _fields_ = [("optimization_count", C.c_int), ("solves", C.c_int), ("edge_queries", C.c_int),
                ("surf_queries", C.c_int), ("edge_correspondences", C.c_int), ("surf_correspondences", C.c_int),
                ("lm_iterations", C.c_int), ("map_updated", C.c_int), ("corner_map", C.c_size_t),
                ("surf_map", C.c_size_t), ("final_cost", C.c_double)]


PRECISION_FP64, PRECISION_FP32, PRECISION_FP32_GEOMETRY = 0, 1, 2
TRACE_WORDS = 49   # per-solve trace record (include/floam_c.h floam_odom_set_trace)

ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int, C.c_void_p)


class PC2Field(C.Structure):
    """floam_pc2_field == sensor_msgs/PointField (name, offset, datatype, count)."""
    _fields_ = [("name", C.c_char * 32), ("offset", C.c_uint32), ("datatype", C.c_uint8), ("count", C.c_uint32)]


class KernelTiming(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_longlong), ("total_ms", C.c_double),
                ("algorithmic_bytes", C.c_double)]


_LIB = None


def load(path: str | None = None):
    """Load libfloam_amd.so (raises FileNotFoundError if it has not been built)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or lib_path()
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                                "or `make -C floam_amd/csrc`")
    L = C.CDLL(p)
    vp, sz, i32, dbl = C.c_void_p, C.c_size_t, C.c_int, C.c_double
    pp = C.POINTER(C.c_void_p)
    szp = C.POINTER(C.c_size_t)
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int)
    u64p = C.POINTER(C.c_uint64)
    sig = {
        "floam_cloud_create": [i32, sz, pp], "floam_cloud_destroy": [vp],
        "floam_cloud_upload": [vp, vp, sz, sz], "floam_cloud_download": [vp, vp, sz, szp],
        "floam_cloud_size": [vp, szp], "floam_cloud_clear": [vp], "floam_cloud_copy": [vp, vp],
        "floam_lp_create": [C.POINTER(LidarParams), i32, pp], "floam_lp_destroy": [vp],
        "floam_lp_feature_extraction": [vp, vp, vp, vp], "floam_lp_set_async": [vp, i32], "floam_lp_wait": [vp],
        "floam_voxel_grid": [vp, C.c_float, vp],
        "floam_odom_create": [C.POINTER(LidarParams), dbl, C.c_char_p, i32, pp], "floam_odom_destroy": [vp],
        "floam_odom_init_map": [vp, vp, vp], "floam_odom_update_selector": [vp, vp, vp, i32],
        "floam_odom_update": [vp, vp, vp, i32], "floam_odom_get_pose": [vp, dp, dp],
        "floam_odom_get_last_pose": [vp, dp, dp], "floam_odom_get_velocity": [vp, dp],
        "floam_odom_get_map": [vp, vp], "floam_odom_get_map_sizes": [vp, szp, szp],
        "floam_odom_download_maps": [vp, vp, sz, vp, sz], "floam_odom_get_stats": [vp, C.POINTER(OdomStats)],
        "floam_odom_set_async": [vp, i32], "floam_odom_wait": [vp, sz, dp, sz, szp],
        "floam_lp_feature_extraction_host": [vp, vp, sz, sz, vp, sz, szp, vp, sz, szp],
        "floam_odom_update_selector_host": [vp, vp, sz, vp, sz, sz, i32],
        "floam_odom_keyframe_update": [vp, vp, vp, dp, dp, ip],
        "floam_odom_get_keyframe": [vp, sz, dp, dp, vp, vp, szp], "floam_odom_set_precision": [vp, i32],
        "floam_odom_set_trace": [vp, sz], "floam_odom_get_traces": [vp, dp, sz, szp],
        "floam_odom_get_correspondences": [vp, i32, vp, vp, ip, C.POINTER(C.c_float), dp, sz, szp],
        "floam_odom_find_correspondences": [vp, vp, vp, dp, dp],
        "floam_comm_unique_id": [vp], "floam_odom_set_shard": [vp, i32, i32, vp],
        "floam_odom_set_shard_callback": [vp, i32, i32, ALLREDUCE_FN, vp],
        "floam_odom_shard_exchange": [vp, vp, C.POINTER(vp)], "floam_odom_set_shard_peers": [vp, i32, i32, vp, vp],
        "floam_device_synchronize": [i32], "floam_profile_enable": [i32, i32],
        "floam_profile_read": [i32, C.POINTER(KernelTiming), i32, C.POINTER(C.c_int)], "floam_profile_reset": [i32], "floam_profile_mark": [i32, i32],
        "floam_imu_create": [i32, pp], "floam_imu_destroy": [vp], "floam_imu_add_msg": [vp, dbl, dp, ip],
        "floam_imu_add_msgs": [vp, dp, dp, sz, szp], "floam_imu_size": [vp, szp],
        "floam_imu_get": [vp, dbl, dp, ip], "floam_imu_time_contained": [vp, dbl, ip],
        "floam_euler_to_quaternion": [dbl, dbl, dbl, dp], "floam_center_time": [vp, u64p],
        "floam_imu_compensate": [vp, vp, C.c_uint64, dp, vp], "floam_imu_preprocess": [vp, vp, u64p, dp, vp],
        "floam_pointcloud2_fields": [i32, C.POINTER(PC2Field), sz, szp, C.POINTER(C.c_uint32)],
        "floam_cloud_from_pointcloud2": [vp, i32, vp, sz, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.POINTER(PC2Field), sz],
        "floam_transform_cloud": [vp, dp, vp],
        "floam_mapping_create": [dbl, i32, pp], "floam_mapping_destroy": [vp], "floam_mapping_update": [vp, vp, dp, dp],
        "floam_mapping_get_map": [vp, vp], "floam_mapping_size": [vp, szp],
        "floam_save_pcd": [C.c_char_p, vp, sz],
        "floam_save_odom": [C.c_char_p, dp, dp, C.POINTER(C.c_void_p), szp, sz],
        "floam_save_posegraph": [C.c_char_p, dp, dp, C.POINTER(C.c_void_p), szp, sz],
        "floam_save_poses_balm": [C.c_char_p, dp, dp, C.POINTER(C.c_void_p), szp, sz],
        "floam_save_merged": [C.c_char_p, dp, C.POINTER(C.c_void_p), szp, sz, dbl, i32],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = C.c_int
    L.floam_cloud_device_ptr.argtypes = [vp]
    L.floam_cloud_device_ptr.restype = vp
    L.floam_last_error.argtypes = []
    L.floam_last_error.restype = C.c_char_p
    L.floam_version.argtypes = []
    L.floam_version.restype = C.c_char_p
    L.floam_abi_version.argtypes = []
    L.floam_abi_version.restype = C.c_int
    if L.floam_abi_version() != ABI_VERSION:   # a library built from another revision of include/floam_c.h
        raise FloamError(ERR_UNSUPPORTED, f"libfloam_amd ABI {L.floam_abi_version()}, this package expects "
                                          f"{ABI_VERSION} (rebuild floam_amd/csrc)")
    L.floam_reset_process_state.argtypes = []
    L.floam_reset_process_state.restype = None
    if path is None:
        _LIB = L
    return L


def check(status: int, allow_warnings: bool = True) -> int:
    if status == OK or (allow_warnings and status >= 100):
        return status
    msg = load().floam_last_error()
    raise FloamError(status, msg.decode() if msg else "")
