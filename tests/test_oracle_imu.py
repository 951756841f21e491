"""CPU: the oracle's IMU pre-processing (oracle/imu.cpp) against an independent numpy
restatement of the reference (src/dataHandler.cpp:23-122, src/laserProcessingNode.cpp:65-113, src/lidar.cpp:8-16),
bit for bit, plus known-answer checks.  numpy float64 elementwise arithmetic is IEEE double without contraction, so
the same operation order gives the same bits.

Parity is pinned against these restatements and the committed golden vectors (tests/golden/imu_c1.npz): the
reference has no tests or fixtures for this path and cannot be built here (needs ROS, PCL, Eigen)."""
import bisect
import math
import os

import numpy as np
import pytest

from floam_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "imu_c1.npz")


# ------------------------------------------------------------------ numpy restatement (x, y, z, w quaternions)
def q_mul_sse2(a, b):
    """Eigen 3.3 Geometry_SSE.h quat_product<SSE, double> (SSE2 mask path)."""
    ax, ay, az, aw = (a[..., k] for k in range(4))
    bx, by, bz, bw = (b[..., k] for k in range(4))
    return np.stack([(aw * bx + ay * bz) - (az * by - ax * bw), (aw * by + ay * bw) + (az * bx - ax * bz),
                     (aw * bz - ay * bx) + (az * bw + ax * by), (aw * bw - ay * by) - (az * bz + ax * bx)], axis=-1)


def q_inverse(q):
    n2 = (q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3])
    if n2 > 0:
        return np.array([-q[0] / n2, -q[1] / n2, -q[2] / n2, q[3] / n2])
    return np.zeros(4)


def q_rotate(q, v):
    """Eigen _transformVector, q (..., 4), v (..., 3)."""
    qv = q[..., :3]
    uv = np.cross(qv, v)
    uv = uv + uv
    return (v + q[..., 3:4] * uv) + np.cross(qv, uv)


def q_matrix(q):
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy], [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


class PyImuHandler:
    def __init__(self):
        self.t, self.q = [], []

    def add(self, stamp, q):
        if self.t and not (stamp - self.t[-1] > 0.00001):
            return False
        self.t.append(float(stamp))
        self.q.append(np.asarray(q, dtype=np.float64))
        return True

    def get(self, ts):
        a = bisect.bisect_left(self.t, ts)
        if a != len(self.t) and a != 0 and a - 1 != 0:
            return self.q[a - 1], True
        return np.zeros(4), False

    def contained(self, ts):
        return bool(self.t) and self.t[0] <= ts <= self.t[-1]


def stamp_to_sec(us):
    ns = us * 1000
    return float(ns // 1_000_000_000) + 1e-9 * float(ns % 1_000_000_000)


def sec_to_stamp(t):
    sec = math.floor(t)
    x = (t - float(sec)) * 1e9
    nsec = int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))
    sec += nsec // 1_000_000_000
    nsec %= 1_000_000_000
    return (sec * 1_000_000_000 + nsec) // 1000


def py_preprocess(pts, stamp_us, h, extr):
    """CenterTime + Compensate + ImuNowT alignment, vectorised over points with the reference's operation order."""
    pts = pts.copy()
    t = pts["time"].astype(np.float64)
    tScan = stamp_to_sec(stamp_us)
    tEnd, tBegin = tScan + t[-1], tScan + t[0]
    tCenter = tBegin + (tEnd - tBegin) / 2.0
    stamp2 = sec_to_stamp(tCenter)
    pts["time"] = ((t + tScan) - tCenter).astype(np.float32)
    tScan2 = stamp_to_sec(stamp2)
    tc = pts["time"].astype(np.float64)
    if not (h.contained(tc[0] + tScan2) and h.contained(tc[-1] + tScan2)):
        return False, pts, None, stamp2
    qInit = q_mul_sse2(h.get(tScan2)[0], extr)
    qInv = q_inverse(qInit)
    qs = np.stack([h.get(tScan2 + x)[0] for x in tc])
    qDiff = q_mul_sse2(np.broadcast_to(qInv, qs.shape), q_mul_sse2(qs, np.broadcast_to(extr, qs.shape)))
    v = np.stack([pts["x"], pts["y"], pts["z"]], axis=1).astype(np.float64)
    c = q_rotate(qDiff, v).astype(np.float32).astype(np.float64)
    R = q_matrix(qInit)
    out = pts.copy()
    for r, f in enumerate("xyz"):
        out[f] = (((R[r, 0] * c[:, 0] + R[r, 1] * c[:, 1]) + R[r, 2] * c[:, 2]) + 0.0).astype(np.float32)
    return True, pts, out, stamp2


def _handler(stamps, q):
    h = PyImuHandler()
    for s, qq in zip(stamps, q):
        h.add(s, qq)
    return h


# ------------------------------------------------------------------------------------------------- tests
def test_addmsg_deduplicates(oracle_lib):
    stamps, _ = synth.imu_stream(-0.5, 0.5)
    stamps = np.concatenate([stamps, [stamps[-1] + 5e-6, stamps[-1] + 2e-5, stamps[-1] - 1.0]])
    keep = oracle_lib.imu_filter(stamps)
    h = PyImuHandler()
    ref = [h.add(s, (0, 0, 0, 1)) for s in stamps]
    np.testing.assert_array_equal(keep, ref)
    assert not keep.all()


def test_get_returns_sample_before_lower_bound(oracle_lib):
    stamps, q = synth.imu_stream(-0.3, 0.3, rate=100.0)
    h = _handler(stamps, q)
    kept_t = np.array(h.t)
    probes = np.concatenate([kept_t[:4], kept_t[-3:], kept_t[:-1] + 1e-4, [kept_t[0] - 1, kept_t[-1] + 1]])
    for ts in probes:
        got, found = oracle_lib.imu_get(stamps, q, ts)
        want, wfound = h.get(ts)
        assert found == wfound, ts
        np.testing.assert_array_equal(got, want)
        assert oracle_lib.imu_time_contained(stamps, q, ts) == h.contained(ts)
    # the first two samples are never returned (itr_before != first) and a stamp equal to a sample returns the one
    # before it (lower_bound finds the equal element)
    assert not oracle_lib.imu_get(stamps, q, kept_t[1])[1]
    got, found = oracle_lib.imu_get(stamps, q, kept_t[5])
    assert found and np.array_equal(got, h.q[4])


def test_euler2quaternion(oracle_lib):
    q = oracle_lib.euler_to_quaternion(0, 0, 180)   # the node's extrinsics (src/laserProcessingNode.cpp:196)
    assert q[0] == 0 and q[1] == 0 and q[2] == 1.0 and abs(q[3]) < 1e-16
    from scipy.spatial.transform import Rotation
    for r, p, y in [(10, -20, 30), (0, 45, 0), (-170, 5, 95)]:
        q = oracle_lib.euler_to_quaternion(r, p, y)
        # rollAngle * yawAngle * pitchAngle = R_x(r) R_z(y) R_y(p)
        ref = (Rotation.from_euler("x", r, degrees=True) * Rotation.from_euler("z", y, degrees=True)
               * Rotation.from_euler("y", p, degrees=True)).as_quat()
        if np.dot(q, ref) < 0:
            ref = -ref
        np.testing.assert_allclose(q, ref, atol=1e-15)


def test_center_time_matches_restatement(oracle_lib):
    pts, st = synth.driver_scan("c1", 4)
    got, st2 = oracle_lib.center_time(pts, st)
    t = pts["time"].astype(np.float64)
    tScan = stamp_to_sec(st)
    tCenter = (tScan + t[0]) + ((tScan + t[-1]) - (tScan + t[0])) / 2.0
    assert st2 == sec_to_stamp(tCenter)
    np.testing.assert_array_equal(got["time"], ((t + tScan) - tCenter).astype(np.float32))
    for f in ("x", "y", "z", "intensity", "ring"):
        np.testing.assert_array_equal(got[f], pts[f])
    assert abs(float(got["time"][0]) + float(got["time"][-1])) < 2e-6   # centred


@pytest.mark.parametrize("scan", [0, 3])
def test_preprocess_matches_restatement(oracle_lib, scan):
    pts, st = synth.driver_scan("c1", scan)
    stamps, q = synth.imu_stream(-1.0, 1.0)
    extr = oracle_lib.euler_to_quaternion(0, 0, 180)
    ok, cin, out, st2 = oracle_lib.imu_preprocess(pts, st, stamps, q, extr)
    rok, rin, rout, rst = py_preprocess(pts, st, _handler(stamps, q), extr)
    assert ok and rok and st2 == rst
    np.testing.assert_array_equal(cin["time"], rin["time"])
    for f in ("x", "y", "z", "intensity", "ring", "time"):
        np.testing.assert_array_equal(out[f], rout[f], err_msg=f)


def test_preprocess_known_answer(oracle_lib):
    """With the IMU orientation equal to the sensor's true orientation (yaw + wobble) the aligned cloud is the scan
    rotated into the gravity-aligned frame of the scan centre: compare with the generator's own geometry."""
    pts, st = synth.driver_scan("c1", 2)
    stamps, q = synth.imu_stream(-1.0, 1.0, wobble_deg=0.0)
    extr = np.array([0.0, 0.0, 1.0, 0.0])
    ok, cin, out, _ = oracle_lib.imu_preprocess(pts, st, stamps, q, extr)
    assert ok
    # q_imu * extr = yaw quaternion, so the alignment rotates by the scan-centre yaw (to the 5-ms IMU sample)
    yaw = synth.YAW_RATE * (2 * synth.SCAN_PERIOD)
    c, s = math.cos(yaw), math.sin(yaw)
    x, y = pts["x"].astype(np.float64), pts["y"].astype(np.float64)
    r_in = np.hypot(x, y)
    r_out = np.hypot(out["x"].astype(np.float64), out["y"].astype(np.float64))
    np.testing.assert_allclose(r_out, r_in, rtol=1e-5, atol=1e-4)   # rotations about z keep the xy range
    np.testing.assert_allclose(out["z"], pts["z"], atol=1e-4)
    ang = np.arctan2(out["y"], out["x"]) - np.arctan2(y, x)
    ang = (ang + np.pi) % (2 * np.pi) - np.pi
    # per-point yaw difference = scan-centre yaw + the within-sweep motion (<= 0.05 s * 5 deg/s) + sample quantisation
    assert np.all(np.abs(ang - yaw) < math.radians(0.3) + 1e-6), np.abs(ang - yaw).max()
    assert abs(c * c + s * s - 1) < 1e-12


def test_no_imu_data(oracle_lib):
    pts, st = synth.driver_scan("c1", 5)
    stamps, q = synth.imu_stream(-1.0, 0.3)   # ends before the scan
    ok, cin, out, st2 = oracle_lib.imu_preprocess(pts, st, stamps, q, (0, 0, 1, 0))
    assert not ok
    rok, rin, _, rst = py_preprocess(pts, st, _handler(stamps, q), np.array([0.0, 0.0, 1.0, 0.0]))
    assert not rok and st2 == rst
    np.testing.assert_array_equal(cin["time"], rin["time"])   # CenterTime ran before the skip


def test_golden_imu_vectors(oracle_lib):
    g = np.load(GOLDEN)
    pts = g["input"].view(synth.POINT_DTYPE)
    ok, cin, out, st2 = oracle_lib.imu_preprocess(pts, int(g["stamp_us"]), g["imu_stamps"], g["imu_q"],
                                                  g["extrinsics"])
    assert ok and st2 == int(g["stamp_out_us"])
    np.testing.assert_array_equal(cin.view(np.uint8), g["centred"])
    np.testing.assert_array_equal(out.view(np.uint8), g["aligned"])
