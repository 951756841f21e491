"""Device clouds: floam_cloud_clear is deferred to the cloud's next operation (on that operation's stream), so a
clear followed by any operation must behave exactly like an immediate clear (include/floam_c.h floam_cloud_clear;
the reference's nodes clear / reassign their clouds every scan)."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu


def _pts(n, seed):
    rng = np.random.default_rng(seed)
    p = np.zeros(n, dtype=synth.POINT_DTYPE)
    p["x"], p["y"], p["z"] = rng.uniform(-20, 20, (3, n)).astype(np.float32)
    p["intensity"] = rng.uniform(0, 255, n).astype(np.float32)
    return p


def test_clear_then_size_download_upload(floam_gpu):
    c = floam_gpu.DeviceCloud(_pts(1000, 1))
    assert len(c) == 1000
    c.clear()
    assert len(c) == 0
    assert c.download().shape[0] == 0
    c.clear()   # twice in a row is still a clear
    p = _pts(300, 2)
    c.upload(p)
    assert len(c) == 300
    np.testing.assert_array_equal(c.download()["x"], p["x"])


def test_clear_then_copy_and_voxel(floam_gpu):
    a = floam_gpu.DeviceCloud(_pts(500, 3))
    b = floam_gpu.DeviceCloud(_pts(700, 4))
    b.clear()
    b.copy_from(a)   # the copy overwrites; the pending clear must not zero it afterwards
    assert len(b) == 500
    np.testing.assert_array_equal(b.download()["y"], a.download()["y"])
    a.clear()
    out = a.voxel_grid(0.5)
    assert len(out) == 0


def test_clear_then_feature_extraction_appends_from_zero(floam_gpu):
    """The bench's per-scan pattern: clear the feature buffers, then featureExtraction appends into them (on the
    extraction's own stream).  The result must equal extraction into fresh clouds."""
    R = synth.lidar_model("c1").rings
    p = floam_gpu.LidarParams(num_lines=R, scan_period=0.1, max_distance=90.0, min_distance=0.5)
    raw0, raw1 = synth.generate_scan("c1", 0), synth.generate_scan("c1", 1)
    for asynchronous in (False, True):
        lp = floam_gpu.LaserProcessingClass(asynchronous=asynchronous)
        lp.init(p)
        e, s = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(raw0), e, s)
        e.clear()
        s.clear()
        lp.featureExtraction(floam_gpu.DeviceCloud(raw1), e, s)
        lp.wait()
        fe, fs = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(raw1), fe, fs)
        lp.wait()
        for a, b in ((e, fe), (s, fs)):
            da, db = a.download(), b.download()
            assert da.shape == db.shape and da.shape[0] > 0
            for f in ("x", "y", "z", "intensity", "ring", "time"):
                np.testing.assert_array_equal(da[f], db[f])
        lp.close()
