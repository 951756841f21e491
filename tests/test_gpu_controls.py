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


@pytest.mark.parametrize("loss", ["Cauchy", "huber"])
def test_per_evaluation_fallback_matches_resident_solve(floam_gpu, monkeypatch, loss):
    """the resident lm_solve needs its whole grid co-resident; where the occupancy check fails the handle
    runs one launch per evaluation (lm_shard_eval on one rank).  Forced here: same LM decisions, poses to ulps."""
    ref, _ = _run(floam_gpu, 6, loss)
    monkeypatch.setenv("FLOAM_LM_PER_EVAL", "1")
    alt, _ = _run(floam_gpu, 6, loss)
    for k, ((qa, ta), (qb, tb)) in enumerate(zip(ref, alt)):
        np.testing.assert_allclose(tb, ta, rtol=0, atol=1e-12, err_msg=f"scan {k}")
        np.testing.assert_allclose(qb, qa, rtol=0, atol=1e-12, err_msg=f"scan {k}")


def test_iteration_zero_from_geometry_matches(floam_gpu, monkeypatch):
    """FLOAM_LM_PRE0=1 (off by default, measured slower): the geometry launch evaluates iteration zero's edge half
    and the solve starts with its first control step.  Only the summation order of that evaluation differs: same LM
    decisions, poses to ulps."""
    ref, _ = _run(floam_gpu, 6)
    monkeypatch.setenv("FLOAM_LM_PRE0", "1")
    alt, _ = _run(floam_gpu, 6)
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


def test_device_failure_poisons_the_handle(floam_gpu, monkeypatch):
    """a solve whose blocks' hand-off timed out freezes the device controller (OdomDev::failed: no pose,
    no keyframe, no map update from then on).  The update that failed raises FLOAM_ERR_DEVICE, and so must every later
    update of the same handle — never a silent FLOAM_OK with stale odometry.  FLOAM_LM_FAIL_TEST=1 makes every resident
    solve report its first hand-off as timed out."""
    from floam_amd import FloamError
    from floam_amd.odom_estimation import reset_process_state
    monkeypatch.setenv("FLOAM_LM_FAIL_TEST", "1")
    reset_process_state()
    lp = floam_gpu.LaserProcessingClass()
    lp.init(_params(16))
    odo = floam_gpu.OdomEstimationClass()
    odo.init(_params(16), 0.1, "Cauchy")
    monkeypatch.delenv("FLOAM_LM_FAIL_TEST")   # (read once, when the handle is created)
    clouds = []
    for k in range(3):
        de, ds = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(synth.generate_scan("c1", k)), de, ds)
        clouds.append((de, ds))
    odo.initMapWithPoints(*clouds[0])
    with pytest.raises(FloamError) as e1:
        odo.UpdatePointsToMapSelector(*clouds[1], True)
    assert "did not arrive" in str(e1.value)
    with pytest.raises(FloamError) as e2:
        odo.UpdatePointsToMapSelector(*clouds[2], True)
    assert "earlier update" in str(e2.value) and "did not arrive" in str(e2.value)
    # a fresh handle is unaffected
    poses, _ = _run(floam_gpu, 3)
    assert np.all(np.isfinite(poses[-1][1]))
