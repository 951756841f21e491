"""GPU parity of LaserMappingClass through the C ABI against the CPU oracle: after every
updateCurrentPointsToMap the device map (getMap order: cells in (x, y, z) order, VoxelGrid output order inside the
filtered cells, push_back order elsewhere) must equal the oracle's bit for bit, over a pose sequence that crosses
50-m cell boundaries (the filtered neighbourhood moves; cells outside it keep unfiltered points) and at two map
resolutions."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "z", "intensity")


def _features(oracle_lib, k, config="c1"):
    raw = synth.generate_scan(config, k)
    e, s, _ = oracle_lib.feature_extraction(raw, synth.lidar_model(config).rings, 0.5, 90.0, canonical=True)
    return synth.to_xyzi(np.concatenate([e, s]))   # /velodyne_points_filtered as PointXYZI


def _pose(k):
    """Yaw + a 40 m/step walk in x and y (crosses cell boundaries every step or two) and a little height."""
    yaw = 0.3 * k
    q = np.array([0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2)])
    t = np.array([40.0 * k - 10.0, 23.0 * k + 3.0, 0.4 * k])
    return q, t


@pytest.mark.parametrize("res", [0.4, 0.15])
def test_mapping_bit_exact(floam_gpu, oracle_lib, res):
    from floam_amd.mapping import LaserMappingClass
    gm = LaserMappingClass()
    gm.init(res)
    om = oracle_lib.Mapping(res, stable_voxel=True)
    for k in range(5):
        pts = _features(oracle_lib, k)
        q, t = _pose(k)
        om.update(pts, q, t)
        gm.updateCurrentPointsToMap(floam_gpu.DeviceCloud(pts), q, t)
        ref = om.get_map()
        got = gm.getMap().download()
        assert got.shape == ref.shape, (k, got.shape, ref.shape)
        assert gm.size() == ref.shape[0]
        for f in FIELDS:
            np.testing.assert_array_equal(got[f], ref[f], err_msg=f"update {k}: {f}")


def test_mapping_far_points_and_empty(floam_gpu, oracle_lib):
    """Points 100-200 m out (outside the filtered neighbourhood: kept unfiltered in their cells) and an empty scan."""
    from floam_amd.mapping import LaserMappingClass
    gm = LaserMappingClass()
    gm.init(0.4)
    om = oracle_lib.Mapping(0.4)
    pts = _features(oracle_lib, 1)
    far = pts[:500].copy()
    far["x"] = far["x"] * 4.0 + 120.0
    pts = np.concatenate([pts, far])
    q, t = np.array([0.0, 0.0, 0.0, 1.0]), np.zeros(3)
    for cloud in (pts, pts[:0], pts):
        om.update(cloud, q, t)
        gm.updateCurrentPointsToMap(floam_gpu.DeviceCloud(cloud) if cloud.shape[0] else floam_gpu.DeviceCloud(), q, t)
        ref, got = om.get_map(), gm.getMap().download()
        assert got.shape == ref.shape
        for f in FIELDS:
            np.testing.assert_array_equal(got[f], ref[f], err_msg=f)
