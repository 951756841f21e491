"""The drop-in adapter's host-resident entry points (include/floam_c.h floam_lp_feature_extraction_host,
floam_odom_update_selector_host): the processing node's featureExtraction on a host cloud and the
odometry node's UpdatePointsToMapSelector on host clouds (src/odomEstimationNode.cpp:205-244) must give exactly what
the device-resident calls give — the same feature clouds byte for byte, the same poses bit for bit, and the caller's
clouds deskewed in place (Q5) exactly as the device clouds are."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu


def _params(R):
    from floam_amd import LidarParams
    return LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)


@pytest.mark.parametrize("config,nscan,graph", [("c1", 6, False), ("c3", 3, False), ("c1", 6, True)])
def test_host_entry_points_match_device_path(floam_gpu, monkeypatch, config, nscan, graph):
    """graph: the host-path odometry created with FLOAM_GRAPH=1 (hipGraph capture of each update, a documented
    product variable): the one-call entry point's write-back copy stream must stay out of the capture."""
    from floam_amd.odom_estimation import reset_process_state
    R = synth.lidar_model(config).rings
    pipes = []
    for j in range(2):
        lp = floam_gpu.LaserProcessingClass()
        lp.init(_params(R))
        if graph and j == 1:
            monkeypatch.setenv("FLOAM_GRAPH", "1")   # (read when the handle is created)
        odo = floam_gpu.OdomEstimationClass()
        odo.init(_params(R), 0.1, "Cauchy")
        monkeypatch.delenv("FLOAM_GRAPH", raising=False)
        pipes.append((lp, odo))
    poses = {0: [], 1: []}
    for k in range(nscan):
        raw = synth.generate_scan(config, k)
        # device path
        reset_process_state()   # (KeyFrameUpdate's process-wide `first`, Q6: each pipeline takes it at its first update)
        lp, odo = pipes[0]
        de, ds = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(raw), de, ds)
        e_dev, s_dev = de.download(), ds.download()
        if k == 0:
            odo.initMapWithPoints(de, ds)
        else:
            odo.UpdatePointsToMapSelector(de, ds, True)
        poses[0].append(odo.pose())
        deskewed = (de.download(), ds.download())
        # host path
        if k > 0:
            reset_process_state()
        lp, odo = pipes[1]
        e_host, s_host = lp.featureExtractionHost(raw)
        assert e_host.shape == e_dev.shape and s_host.shape == s_dev.shape
        np.testing.assert_array_equal(e_host.view(np.uint8), e_dev.view(np.uint8))
        np.testing.assert_array_equal(s_host.view(np.uint8), s_dev.view(np.uint8))
        if k == 0:
            odo.initMapWithPoints(floam_gpu.DeviceCloud(e_host), floam_gpu.DeviceCloud(s_host))
        else:
            odo.UpdatePointsToMapSelectorHost(e_host, s_host, True)
            np.testing.assert_array_equal(e_host.view(np.uint8), deskewed[0].view(np.uint8), err_msg="edge write-back")
            np.testing.assert_array_equal(s_host.view(np.uint8), deskewed[1].view(np.uint8), err_msg="surf write-back")
        poses[1].append(odo.pose())
    for k, ((qa, ta), (qb, tb)) in enumerate(zip(poses[0], poses[1])):
        np.testing.assert_array_equal(qa, qb, err_msg=f"scan {k} q")
        np.testing.assert_array_equal(ta, tb, err_msg=f"scan {k} t")


def test_host_entry_points_validate(floam_gpu):
    from floam_amd import FloamError
    lp = floam_gpu.LaserProcessingClass()
    lp.init(_params(16))
    e, s = lp.featureExtractionHost(np.zeros(0, synth.POINT_DTYPE))
    assert e.shape[0] == 0 and s.shape[0] == 0
    odo = floam_gpu.OdomEstimationClass()
    odo.init(_params(16), 0.1, "Cauchy")
    with pytest.raises(FloamError):
        odo.UpdatePointsToMapSelectorHost(np.zeros(4, np.float32), np.zeros(4, np.float32), True)
