"""floam_amd — MI355X-native (gfx950) scan-to-map lidar odometry core with the FLOAM operator API.

Drop-in for the hot path of dan11003/floam: ``LaserProcessingClass.featureExtraction`` and
``OdomEstimationClass.UpdatePointsToMapSelector`` run as hand-written HIP kernels behind the C ABI in
include/floam_c.h (libfloam_amd.so); this package is the host-side mirror of those two classes.
"""
from ._ffi import FloamError, load  # noqa: F401
from .cloud import DeviceCloud  # noqa: F401
from .imu import CenterTime, Compensate, ImuHandler, euler2Quaternion  # noqa: F401
from .laser_processing import LaserProcessingClass, LidarParams  # noqa: F401
from .odom_estimation import OdomEstimationClass, UpdateType  # noqa: F401
from .synth import POINT_DTYPE  # noqa: F401

__version__ = "0.4.0"   # floam_version() of the library it binds (ABI 3)
