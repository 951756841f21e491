"""CPU check of the LM control step's gradient-test shortcut (floam_amd/csrc/lm.hip `gradient_step_far`): when the
rotation angle th of the projected step -g is > 1.5625 and th / 4 is more than 1e-6 from every multiple of pi, the
SE(3) plus (src/lidarOptimization.cpp:77-140) moves some quaternion component by more than the gradient tolerance
1e-10 (src/odomEstimationClass.cpp:100-108 uses Ceres' default), so the test fails without computing the projection.
The angle criterion is restated here in numpy and checked against the exact quaternion update."""
import numpy as np


def far(th):
    if not (1.5625 < th < 1e15):
        return False
    u = 0.25 * th
    k = np.rint(u * 0.31830988618379067154)
    r = u - k * 3.141592653589793116   # (two-constant reduction in lm.hip; one constant suffices for this range)
    r = r - k * 1.2246467991473532072e-16
    return 1e-6 < abs(r) < 3.1415916


def quat_mul(a, b):   # (x, y, z, w)
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def test_far_angles_fail_the_gradient_test():
    rng = np.random.default_rng(3)
    checked = 0
    for _ in range(20000):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        th = float(np.exp(rng.uniform(np.log(1.6), np.log(1e6))))
        w = rng.normal(size=3)
        w *= th / np.linalg.norm(w)
        if not far(th):
            continue
        half = 0.5 * th
        dq = np.r_[np.sin(half) / th * w, np.cos(half)]
        qn = quat_mul(dq, q)
        assert np.max(np.abs(q - qn)) > 1e-10, th
        checked += 1
    assert checked > 19000


def test_near_multiples_of_4pi_are_not_shortcut():
    for k in (1, 2, 7, 1000):
        th = 4 * np.pi * k
        assert not far(th)
        assert not far(np.nextafter(th, 0))
    assert not far(1.0) and not far(1.5625)
