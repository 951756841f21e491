"""Seeded synthetic ring-lidar scans for tests and the benchmark.

The reference ships no data (SURVEY.md §4, §8 d), so every parity test and the bench run on scans from this
generator.  The shapes follow BASELINE.json ``configs`` / SURVEY.md §8(d):

=========  =====  =========  ====================================  ==================
config     rings  az. steps  elevations                            map prefill
=========  =====  =========  ====================================  ==================
``c1``     16     1024       VLP-16, -15..+15 deg, 2 deg step      grows from scan 0
``c2``     16     1875       VLP-16                                50k
``c3``     64     2048       HDL-64 style, +2..-24.33 deg          200k  (headline)
``c4``     128    2048       OS2 style, -11.25..+11.25 deg         500k
``c5``     128    4096       OS2 style                             2M
=========  =====  =========  ====================================  ==================

Scene (world frame, z up): ground plane at z = -1.73 m (sensor height), a ring of box buildings 22-48 m from the
centre of the trajectory plus an outer ring at 60-85 m, vertical poles (r = 0.15 m) on two circles, and car-sized
boxes.  Emission order is azimuth-major (all rings of one firing, then the next azimuth), like a spinning sensor.
Every point is ray-cast from the sensor pose *at its own firing time* (motion distortion), and ``time`` is relative
to the scan centre in [-0.05, 0.05] s, i.e. what ``CenterTime`` (src/laserProcessingNode.cpp:65-78) produces.
Range noise N(0, 0.01 m) makes exact curvature ties measure-zero (SURVEY.md §7 "Hard parts").

Trajectory: 1 m/s forward + 5 deg/s yaw at 10 Hz (SURVEY.md §8 d).

Determinism: the generator is numpy-only and seeded (``seed = 20251015 + scan_idx``); transcendental ufuncs can
differ by an ulp between CPU types, so parity tests always compare GPU and oracle on the *same* generated arrays
(fixtures under tests/golden store the inputs, never regenerate them).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# 32-byte point record == vel_point::PointXYZIRT (include/lidar.h:14-32, EIGEN_ALIGN16):
# x@0 y@4 z@8 pad@12 intensity@16 ring(u16)@20 pad@22 time@24 pad@28.  pcl::PointXYZI shares x,y,z,intensity
# offsets, so one record type serves both clouds.
POINT_DTYPE = np.dtype({
    "names": ["x", "y", "z", "pad0", "intensity", "ring", "pad1", "time", "pad2"],
    "formats": ["<f4", "<f4", "<f4", "<f4", "<f4", "<u2", "<u2", "<f4", "<f4"],
    "offsets": [0, 4, 8, 12, 16, 20, 22, 24, 28],
    "itemsize": 32,
})

SCAN_PERIOD = 0.1
SENSOR_HEIGHT = 1.73
BASE_SEED = 20251015


@dataclass(frozen=True)
class LidarModel:
    name: str
    rings: int
    steps: int
    elev_deg: np.ndarray  # per ring, ring 0 = lowest beam


def _lin(a, b, n):
    return np.linspace(a, b, n, dtype=np.float64)


def lidar_model(config: str) -> LidarModel:
    config = config.lower()
    if config == "c1":
        return LidarModel("vlp16", 16, 1024, _lin(-15.0, 15.0, 16))
    if config == "c2":
        return LidarModel("vlp16", 16, 1875, _lin(-15.0, 15.0, 16))
    if config == "c3":
        return LidarModel("hdl64", 64, 2048, _lin(-24.33, 2.0, 64))
    if config == "c4":
        return LidarModel("os2", 128, 2048, _lin(-11.25, 11.25, 128))
    if config == "c5":
        return LidarModel("os2-dense", 128, 4096, _lin(-11.25, 11.25, 128))
    if config.startswith("tiny"):  # small case for fast CPU tests: tiny<rings>x<steps>
        r, s = config[4:].split("x")
        r, s = int(r), int(s)
        return LidarModel("tiny", r, s, _lin(-15.0, 15.0, r))
    raise ValueError(f"unknown config {config!r}")


MAP_PREFILL = {"c1": 0, "c2": 50_000, "c3": 200_000, "c4": 500_000, "c5": 2_000_000}


def prefill_map(config: str, feature_extraction, target: int | None = None):
    """The raw local map initMapWithPoints receives for ``config`` (SURVEY.md §8 d: maps prefilled to the stated
    size): the edge / surf features of scan 0 (sensor frame == map frame) plus the features of earlier scans on the
    ground-truth trajectory (scans -3, -6, ...) transformed into the map frame, until ``target`` points (the surf tail
    trimmed to hit it exactly).  ``feature_extraction(raw, rings) -> (edge, surf)`` is the caller's
    featureExtraction (the GPU operator in the bench, the CPU restatement in the tests: byte-identical outputs)."""
    target = MAP_PREFILL.get(config, 0) if target is None else target
    R = lidar_model(config).rings
    e0, s0 = feature_extraction(generate_scan(config, 0), R)
    E, S = [to_xyzi(e0)], [to_xyzi(s0)]
    n = e0.shape[0] + s0.shape[0]
    k = -3
    while n < target:
        e, s = feature_extraction(generate_scan(config, k), R)
        T = gt_pose_matrix(k)
        E.append(to_xyzi(transform_points(e, T)))
        S.append(to_xyzi(transform_points(s, T)))
        n += e.shape[0] + s.shape[0]
        k -= 3
    E, S = np.concatenate(E), np.concatenate(S)
    extra = E.shape[0] + S.shape[0] - target
    if target and extra > 0:
        S = S[: S.shape[0] - extra]
    return E, S


# ----------------------------------------------------------------------------------------------- trajectory
V_FWD = 1.0                       # m/s
YAW_RATE = math.radians(5.0)      # rad/s


def pose_at(tau: np.ndarray | float):
    """Ground-truth sensor pose at absolute time tau (s): returns (x, y, z, yaw)."""
    tau = np.asarray(tau, dtype=np.float64)
    yaw = YAW_RATE * tau
    r = V_FWD / YAW_RATE
    x = r * np.sin(yaw)
    y = r * (1.0 - np.cos(yaw))
    z = np.zeros_like(tau)
    return x, y, z, yaw


def gt_pose_matrix(scan_idx: int) -> np.ndarray:
    """4x4 ground-truth pose of the sensor at the centre of scan ``scan_idx``."""
    x, y, z, yaw = (float(v) for v in pose_at(scan_idx * SCAN_PERIOD))
    c, s = math.cos(yaw), math.sin(yaw)
    T = np.eye(4)
    T[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    T[:3, 3] = [x, y, z]
    return T


# ----------------------------------------------------------------------------------------------- scene
@dataclass
class Scene:
    boxes: np.ndarray      # (B, 6) xmin ymin zmin xmax ymax zmax
    poles: np.ndarray      # (C, 5) cx cy r zmin zmax
    ground_z: float = -SENSOR_HEIGHT


def make_scene(seed: int = 7) -> Scene:
    rng = np.random.default_rng(seed)
    cx, cy = 0.0, V_FWD / YAW_RATE   # centre of the circular trajectory
    boxes = []
    # inner ring of buildings
    n_in = 18
    for k in range(n_in):
        a = 2 * math.pi * (k + rng.uniform(0.1, 0.4)) / n_in
        rad = rng.uniform(24.0, 34.0)
        w = rng.uniform(5.0, 9.0)
        d = rng.uniform(4.0, 10.0)
        h = rng.uniform(6.0, 22.0)
        bx, by = cx + rad * math.cos(a), cy + rad * math.sin(a)
        boxes.append([bx - w / 2, by - d / 2, -SENSOR_HEIGHT, bx + w / 2, by + d / 2, -SENSOR_HEIGHT + h])
    # outer ring
    n_out = 26
    for k in range(n_out):
        a = 2 * math.pi * (k + rng.uniform(0.0, 0.5)) / n_out
        rad = rng.uniform(62.0, 82.0)
        w = rng.uniform(8.0, 16.0)
        d = rng.uniform(6.0, 14.0)
        h = rng.uniform(10.0, 35.0)
        bx, by = cx + rad * math.cos(a), cy + rad * math.sin(a)
        boxes.append([bx - w / 2, by - d / 2, -SENSOR_HEIGHT, bx + w / 2, by + d / 2, -SENSOR_HEIGHT + h])
    # car-sized boxes between trajectory and the inner ring
    for k in range(14):
        a = 2 * math.pi * (k + rng.uniform(0.0, 0.6)) / 14
        rad = rng.uniform(17.5, 20.5)
        bx, by = cx + rad * math.cos(a), cy + rad * math.sin(a)
        L, W, H = rng.uniform(3.8, 4.8), rng.uniform(1.7, 2.0), rng.uniform(1.3, 1.8)
        if rng.uniform() < 0.5:
            L, W = W, L
        boxes.append([bx - L / 2, by - W / 2, -SENSOR_HEIGHT, bx + L / 2, by + W / 2, -SENSOR_HEIGHT + H])
    poles = []
    for rad, spacing in ((15.5, 6.0), (4.5, 6.0)):
        n = max(3, int(2 * math.pi * rad / spacing))
        for k in range(n):
            a = 2 * math.pi * k / n + rng.uniform(-0.05, 0.05)
            poles.append([cx + rad * math.cos(a), cy + rad * math.sin(a), 0.15, -SENSOR_HEIGHT,
                          -SENSOR_HEIGHT + rng.uniform(4.0, 7.0)])
    return Scene(np.asarray(boxes, np.float64), np.asarray(poles, np.float64))


_SCENE: Scene | None = None


def scene() -> Scene:
    global _SCENE
    if _SCENE is None:
        _SCENE = make_scene()
    return _SCENE


def raycast(origins: np.ndarray, dirs: np.ndarray, sc: Scene, t_max: float = 120.0) -> np.ndarray:
    """Distance along each unit ray to the first hit (inf if none within t_max)."""
    n = origins.shape[0]
    t = np.full(n, np.inf)
    ox, oy, oz = origins[:, 0], origins[:, 1], origins[:, 2]
    dx, dy, dz = dirs[:, 0], dirs[:, 1], dirs[:, 2]
    # ground
    with np.errstate(divide="ignore", invalid="ignore"):
        tg = (sc.ground_z - oz) / dz
    tg = np.where((dz < -1e-9) & (tg > 0), tg, np.inf)
    t = np.minimum(t, tg)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / np.stack([dx, dy, dz], axis=1)
    for b in sc.boxes:
        with np.errstate(invalid="ignore"):
            t1 = (b[0:3][None, :] - origins) * inv
            t2 = (b[3:6][None, :] - origins) * inv
        tn = np.nanmax(np.minimum(t1, t2), axis=1)
        tf = np.nanmin(np.maximum(t1, t2), axis=1)
        hit = (tn <= tf) & (tn > 1e-6)
        t = np.where(hit & (tn < t), tn, t)
    dxy2 = dx * dx + dy * dy
    for p in sc.poles:
        ex, ey = ox - p[0], oy - p[1]
        b_ = ex * dx + ey * dy
        c_ = ex * ex + ey * ey - p[2] * p[2]
        disc = b_ * b_ - dxy2 * c_
        ok = (disc > 0) & (dxy2 > 1e-12)
        with np.errstate(invalid="ignore", divide="ignore"):
            tc = (-b_ - np.sqrt(np.where(ok, disc, 0.0))) / dxy2
        zc = oz + tc * dz
        hit = ok & (tc > 1e-6) & (zc >= p[3]) & (zc <= p[4])
        t = np.where(hit & (tc < t), tc, t)
    t[t > t_max] = np.inf
    return t


def generate_scan(config: str, scan_idx: int, seed: int | None = None, noise: float = 0.01) -> np.ndarray:
    """One synthetic scan as a POINT_DTYPE array in the sensor frame of each firing (motion-distorted)."""
    m = lidar_model(config)
    rng = np.random.default_rng(BASE_SEED + scan_idx if seed is None else seed)
    sc = scene()
    A, R = m.steps, m.rings
    a_idx = np.repeat(np.arange(A), R)             # azimuth-major
    ring = np.tile(np.arange(R), A)
    t_rel = (a_idx + 0.5) / A * SCAN_PERIOD - 0.5 * SCAN_PERIOD
    tau = scan_idx * SCAN_PERIOD + t_rel
    px, py, pz, yaw = pose_at(tau)
    az = 2.0 * math.pi * (a_idx + 0.5) / A - math.pi
    el = np.radians(m.elev_deg)[ring]
    ce = np.cos(el)
    dl = np.stack([ce * np.cos(az), ce * np.sin(az), np.sin(el)], axis=1)   # local ray dir
    cy_, sy_ = np.cos(yaw), np.sin(yaw)
    dw = np.stack([cy_ * dl[:, 0] - sy_ * dl[:, 1], sy_ * dl[:, 0] + cy_ * dl[:, 1], dl[:, 2]], axis=1)
    org = np.stack([px, py, pz], axis=1)
    rng_t = raycast(org, dw, sc)
    keep = np.isfinite(rng_t)
    r = rng_t[keep] + rng.normal(0.0, noise, size=int(keep.sum()))
    pts = dl[keep] * r[:, None]
    out = np.zeros(int(keep.sum()), dtype=POINT_DTYPE)
    out["x"] = pts[:, 0]
    out["y"] = pts[:, 1]
    out["z"] = pts[:, 2]
    out["pad0"] = 1.0
    out["intensity"] = rng.uniform(0.0, 255.0, size=out.shape[0]).astype(np.float32)
    out["ring"] = ring[keep].astype(np.uint16)
    out["time"] = t_rel[keep].astype(np.float32)
    return out


def transform_points(pts: np.ndarray, T: np.ndarray) -> np.ndarray:
    """Apply a 4x4 transform to a POINT_DTYPE array (float64 math, float32 result)."""
    out = pts.copy()
    xyz = np.stack([pts["x"], pts["y"], pts["z"]], axis=1).astype(np.float64)
    w = xyz @ T[:3, :3].T + T[:3, 3]
    out["x"], out["y"], out["z"] = w[:, 0], w[:, 1], w[:, 2]
    return out


def to_xyzi(pts: np.ndarray) -> np.ndarray:
    """VelToIntensityCopy (src/odomEstimationClass.cpp:308-318): keep x, y, z, intensity; zero the rest."""
    out = np.zeros(pts.shape[0], dtype=POINT_DTYPE)
    for f in ("x", "y", "z", "intensity"):
        out[f] = pts[f]
    out["pad0"] = 1.0
    return out


# ----------------------------------------------------------------------------------------------- IMU stream
EPOCH = 1_700_000_000.0   # absolute time of scan 0's centre (s); ROS stamps are absolute


def _quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Hamilton product of (..., 4) quaternions in (x, y, z, w) order (generator only, not a reference formula)."""
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz], axis=-1)


def imu_stream(t_begin: float, t_end: float, rate: float = 200.0, extrinsics_xyzw=(0.0, 0.0, 1.0, 0.0),
               wobble_deg: float = 1.5, seed: int = 11):
    """IMU messages (stamps, orientations (n, 4) x,y,z,w) covering [t_begin, t_end] (seconds relative to EPOCH).

    The orientation is the ground-truth sensor yaw plus a slow roll/pitch wobble, expressed so that
    q_imu * extrinsics = q_sensor (the node composes Imu2Orientation(...) * extrinsics, src/dataHandler.cpp:108,112).
    Stamps are absolute (EPOCH + t) with a small seeded jitter; one duplicated stamp is injected to exercise
    AddMsg's de-duplication (src/dataHandler.cpp:23-38)."""
    rng = np.random.default_rng(seed)
    n = int(math.ceil((t_end - t_begin) * rate)) + 1
    t = t_begin + np.arange(n) / rate + rng.uniform(-0.1, 0.1, n) / rate
    yaw = YAW_RATE * t
    roll = np.radians(wobble_deg) * np.sin(2.0 * math.pi * 0.7 * t)
    pitch = np.radians(wobble_deg) * np.cos(2.0 * math.pi * 0.45 * t)
    def axis_q(ang, k):
        q = np.zeros((ang.shape[0], 4))
        q[:, k] = np.sin(0.5 * ang)
        q[:, 3] = np.cos(0.5 * ang)
        return q
    q_sensor = _quat_mul(_quat_mul(axis_q(yaw, 2), axis_q(pitch, 1)), axis_q(roll, 0))
    e = np.asarray(extrinsics_xyzw, dtype=np.float64)
    e_inv = np.array([-e[0], -e[1], -e[2], e[3]]) / float(e @ e)
    q_imu = _quat_mul(q_sensor, np.broadcast_to(e_inv, q_sensor.shape))
    stamps = EPOCH + t
    if n > 4:
        stamps[n // 2] = stamps[n // 2 - 1]   # a duplicate the handler must drop
    return stamps, q_imu


def driver_scan(config: str, scan_idx: int):
    """A scan as the driver publishes it: point times from the start of the sweep (0 .. 0.1 s) and the header
    stamp at the sweep start, in PCL microseconds — the input CenterTime (src/laserProcessingNode.cpp:65-78)
    re-centres.  Returns (points, stamp_us)."""
    pts = generate_scan(config, scan_idx)
    pts["time"] = (pts["time"].astype(np.float64) + 0.5 * SCAN_PERIOD).astype(np.float32)
    stamp_us = int(round((EPOCH + scan_idx * SCAN_PERIOD - 0.5 * SCAN_PERIOD) * 1e6))
    return pts, stamp_us
