"""KeyFrameUpdate through the C ABI with the reference's signature (include/odomEstimationClass.h:80):
KeyFrameUpdate(surf_cloud, edge_cloud, pose), the 3-deep keyframe history it maintains
(src/odomEstimationClass.cpp:320-343), and the inline GetVelocity of the header (:78) over the mirrored poses."""
import math

import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu


def _params(R):
    from floam_amd import LidarParams
    return LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)


def _yaw_q(a):
    return np.array([0.0, 0.0, math.sin(a / 2), math.cos(a / 2)])


def _is_new_keyframe(last, cur):
    """src/odomEstimationClass.cpp:329-333: delta = last^-1 * cur; |delta.t| > 0.07 or angle(delta.R) > 2 deg."""
    from scipy.spatial.transform import Rotation
    (ql, tl), (qc, tc) = last, cur
    Rl, Rc = Rotation.from_quat(ql), Rotation.from_quat(qc)
    dt = Rl.inv().apply(np.asarray(tc) - np.asarray(tl))
    drot = (Rl.inv() * Rc).magnitude()
    return np.linalg.norm(dt) > 0.07 or drot > 2 * math.pi / 180.0


def test_keyframe_update_signature_and_history(floam_gpu):
    from floam_amd.odom_estimation import reset_process_state
    reset_process_state()
    odo = floam_gpu.OdomEstimationClass()
    odo.init(_params(16), 0.1, "Cauchy")
    raw = synth.generate_scan("c1", 0)
    poses = [(_yaw_q(0.0), np.zeros(3)),             # first call of the process: keyframe (`first`, :324-327)
             (_yaw_q(0.0), np.array([0.05, 0, 0])),  # 5 cm: not a keyframe
             (_yaw_q(0.0), np.array([0.08, 0, 0])),  # 8 cm from the last keyframe: keyframe
             (_yaw_q(0.03), np.array([0.08, 0, 0])), # 1.7 deg: not
             (_yaw_q(0.04), np.array([0.08, 0, 0])), # 2.3 deg: keyframe
             (_yaw_q(0.04), np.array([0.2, 0, 0])),  # keyframe; history trimmed to 3 (:335-337)
             (_yaw_q(0.04), np.array([0.4, 0.1, 0]))]
    history = []
    for k, pose in enumerate(poses):
        surf = floam_gpu.DeviceCloud(raw[k * 100:(k + 1) * 100 + 7])
        edge = floam_gpu.DeviceCloud(raw[5000 + k * 10:5000 + k * 10 + 3])
        expect = k == 0 or _is_new_keyframe(history[-1][0], pose)
        got = odo.KeyFrameUpdate(surf, edge, pose)
        assert got == expect, (k, got, expect)
        if expect:
            history.append((pose, surf.download(), edge.download()))
            if k > 0 and len(history) > 3:
                history.pop(0)
        kf = odo.keyframes()
        assert len(kf) == len(history)
        for (q, t, s, e), ((qh, th), sh, eh) in zip(kf, history):
            np.testing.assert_allclose(q, qh, atol=1e-15)
            np.testing.assert_array_equal(t, th)
            np.testing.assert_array_equal(s.view(np.uint8), sh.view(np.uint8))   # device copies, byte for byte
            np.testing.assert_array_equal(e.view(np.uint8), eh.view(np.uint8))
    # null clouds (a null Ptr in the reference) are accepted; a 4x4 isometry is accepted as the pose
    T = np.eye(4)
    T[:3, 3] = [2.0, 0, 0]
    assert odo.KeyFrameUpdate(None, None, T)
    q, t, s, e = odo.keyframes()[-1]
    assert t[0] == 2.0 and len(s) == 0 and len(e) == 0


def test_keyframe_history_of_updates_and_velocity(floam_gpu, oracle_lib):
    """The updates' own keyframes enter the same history (pose only), the decision follows an explicit
    KeyFrameUpdate's keyframe, and GetVelocity equals the header's inline body over odom / last_odom."""
    from floam_amd.odom_estimation import reset_process_state
    R = 16
    reset_process_state()
    lp = floam_gpu.LaserProcessingClass()
    lp.init(_params(R))
    odo = floam_gpu.OdomEstimationClass()
    odo.init(_params(R), 0.1, "Cauchy")
    kf_poses = []
    for k in range(7):
        de, ds = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(synth.generate_scan("c1", k)), de, ds)
        if k == 0:
            odo.initMapWithPoints(de, ds)
            continue
        odo.UpdatePointsToMapSelector(de, ds, True)
        st = odo.stats()
        if st["map_updated"]:
            kf_poses.append(odo.pose())
        (q, t), (ql, tl) = odo.pose(), odo.last_pose()
        np.testing.assert_array_equal(odo.GetVelocity(), (t - tl) / 0.1)
    assert len(kf_poses) >= 4
    kf = odo.keyframes()
    assert len(kf) == 3
    for (q, t, s, e), (qp, tp) in zip(kf, kf_poses[-3:]):
        np.testing.assert_allclose(q, qp, atol=1e-15)
        np.testing.assert_array_equal(t, tp)
        assert len(s) == 0 and len(e) == 0
    # a pose next to the last keyframe is not a keyframe; one 1 m away is, and it becomes the reference pose
    q, t = kf_poses[-1]
    assert not odo.KeyFrameUpdate(None, None, (q, t + np.array([0.01, 0, 0])))
    assert odo.KeyFrameUpdate(None, None, (q, t + np.array([1.0, 0, 0])))
    assert not odo.KeyFrameUpdate(None, None, (q, t + np.array([1.02, 0, 0])))
    assert len(odo.keyframes()) == 3
