"""Control-path guards of the odometry handle on the GPU: the per-evaluation fallback of the LM solve (taken when the
resident solve's grid cannot be co-resident), trace overflow reporting, and the refusal of neighbour indices from an
untraced correspondence pass."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu


def _params(R):
    from floam_amd import LidarParams
    return LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)


def _run(floam_gpu, n, loss="Cauchy", trace=0):
    from floam_amd.odom_estimation import reset_process_state
    reset_process_state()
    lp = floam_gpu.LaserProcessingClass()
    lp.init(_params(16))
    odo = floam_gpu.OdomEstimationClass()
    odo.init(_params(16), 0.1, loss)
    if trace:
        odo.set_trace(trace)
    poses = []
    for k in range(n):
        de, ds = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(synth.generate_scan("c1", k)), de, ds)
        if k == 0:
            odo.initMapWithPoints(de, ds)
        else:
            odo.UpdatePointsToMapSelector(de, ds, True)
        poses.append(odo.pose())
    return poses, odo


def _poses_child(n, loss):
    import floam_amd
    return [tuple(np.asarray(v) for v in pose) for pose in _run(floam_amd, n, loss)[0]]


@pytest.mark.parametrize("loss", ["Cauchy", "huber"])
def test_per_evaluation_fallback_matches_resident_solve(floam_gpu, loss):
    """the resident lm_solve needs its whole grid co-resident; where the occupancy check fails the handle
    runs one launch per evaluation (lm_shard_eval on one rank).  Forced here (FLOAM_LM_PER_EVAL=1, diagnostic build):
    same LM decisions, poses to ulps."""
    from tests.diag import run_diag
    ref, _ = _run(floam_gpu, 6, loss)
    alt = run_diag(_poses_child, 6, loss, env={"FLOAM_LM_PER_EVAL": "1"})
    for k, ((qa, ta), (qb, tb)) in enumerate(zip(ref, alt)):
        np.testing.assert_allclose(tb, ta, rtol=0, atol=1e-12, err_msg=f"scan {k}")
        np.testing.assert_allclose(qb, qa, rtol=0, atol=1e-12, err_msg=f"scan {k}")


def test_trace_overflow_is_reported(floam_gpu):
    """a trace capacity below the number of solves is reported (n_out > capacity), not hidden."""
    from floam_amd import FloamError
    _, odo = _run(floam_gpu, 2, trace=1)   # one deskewed update with optimization_count 11 + 10 solves
    with pytest.raises(FloamError, match="truncated"):
        odo.traces()
    _, odo = _run(floam_gpu, 2, trace=64)
    assert len(odo.traces()) == 21


def test_untraced_pass_has_no_neighbour_indices(floam_gpu):
    """neighbour indices / distances exist only for a traced pass; switching tracing on after an
    untraced update does not hand out stale ones."""
    from floam_amd import FloamError
    _, odo = _run(floam_gpu, 2)
    odo.set_trace(16)
    with pytest.raises(FloamError, match="untraced"):
        odo.correspondences(0)


def _failure_child():
    import floam_amd
    from floam_amd import FloamError
    from floam_amd.odom_estimation import reset_process_state
    reset_process_state()
    lp = floam_amd.LaserProcessingClass()
    lp.init(_params(16))
    odo = floam_amd.OdomEstimationClass()
    odo.init(_params(16), 0.1, "Cauchy")
    clouds = []
    for k in range(3):
        de, ds = floam_amd.DeviceCloud(), floam_amd.DeviceCloud()
        lp.featureExtraction(floam_amd.DeviceCloud(synth.generate_scan("c1", k)), de, ds)
        clouds.append((de, ds))
    odo.initMapWithPoints(*clouds[0])
    msgs = []
    for k in (1, 2):
        try:
            odo.UpdatePointsToMapSelector(*clouds[k], True)
            msgs.append(None)
        except FloamError as e:
            msgs.append((e.status, str(e)))
    return msgs


def test_device_failure_poisons_the_handle(floam_gpu):
    """a solve whose blocks' hand-off timed out freezes the device controller (OdomDev::failed: no pose,
    no keyframe, no map update from then on).  The update that failed raises FLOAM_ERR_DEVICE, and so must every later
    update of the same handle — never a silent FLOAM_OK with stale odometry.  FLOAM_LM_FAIL_TEST=1 (diagnostic build)
    makes every resident solve report its first hand-off as timed out."""
    from tests.diag import run_diag
    from floam_amd import _ffi
    m1, m2 = run_diag(_failure_child, env={"FLOAM_LM_FAIL_TEST": "1"})
    assert m1 is not None and m1[0] == _ffi.ERR_DEVICE and "did not arrive" in m1[1], m1
    assert m2 is not None and m2[0] == _ffi.ERR_DEVICE and "earlier update" in m2[1] and "did not arrive" in m2[1], m2
    # a fresh handle (product library) is unaffected
    poses, _ = _run(floam_gpu, 3)
    assert np.all(np.isfinite(poses[-1][1]))
