"""GPU parity of the IMU pre-processing through the C ABI against the CPU oracle: the fused
CenterTime + Compensate + IMU-alignment kernel, Compensate alone and CenterTime alone must be bit-identical to the
oracle (integer/byte-exact bar: every output is a float computed in double with the reference's operation order).
Edge cases: no IMU coverage (the node's skip), point times outside the LDS stamp window, NaN points, an empty cloud,
the golden vectors, and the handler's AddMsg / Get / TimeContained look-ups."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "z", "intensity", "ring", "time")


def _same(a, b, what):
    assert a.shape == b.shape, f"{what}: {a.shape} vs {b.shape}"
    for f in FIELDS:
        np.testing.assert_array_equal(a[f], b[f], err_msg=f"{what}.{f}")


def _handler(floam_gpu, stamps, q):
    h = floam_gpu.ImuHandler()
    h.add_msgs(stamps, q)
    return h


@pytest.mark.parametrize("config,scan", [("c1", 0), ("c1", 6), ("c3", 2)])
def test_preprocess_bit_exact(floam_gpu, oracle_lib, config, scan):
    from floam_amd import imu
    pts, st = synth.driver_scan(config, scan)
    stamps, q = synth.imu_stream(-1.0, 1.5)
    extr = imu.euler2Quaternion(0, 0, 180)
    np.testing.assert_array_equal(extr, oracle_lib.euler_to_quaternion(0, 0, 180))
    ok, c_ref, a_ref, st_ref = oracle_lib.imu_preprocess(pts, st, stamps, q, extr)
    h = _handler(floam_gpu, stamps, q)
    din, dal = floam_gpu.DeviceCloud(pts), floam_gpu.DeviceCloud()
    ok_g, st_g = imu.preprocess(din, st, h, extr, dal)
    assert ok and ok_g and st_g == st_ref
    _same(din.download(), c_ref, "centred")
    _same(dal.download(), a_ref, "aligned")


def test_compensate_and_center_time_alone(floam_gpu, oracle_lib):
    from floam_amd import imu
    pts, st = synth.driver_scan("c1", 3)
    stamps, q = synth.imu_stream(-1.0, 1.0)
    extr = np.array([0.0, 0.0, 1.0, 0.0])
    c_ref, st2 = oracle_lib.center_time(pts, st)
    d = floam_gpu.DeviceCloud(pts)
    assert imu.CenterTime(d, st) == st2
    _same(d.download(), c_ref, "CenterTime")
    ok, _, comp_ref, _ = oracle_lib.imu_preprocess(c_ref, st2, stamps, q, extr, mode=2)
    h = _handler(floam_gpu, stamps, q)
    dc = floam_gpu.DeviceCloud()
    assert ok and imu.Compensate(d, dc, h, extr, st2)
    _same(dc.download(), comp_ref, "Compensate")


def test_no_imu_data_skips(floam_gpu, oracle_lib):
    from floam_amd import imu
    pts, st = synth.driver_scan("c1", 8)
    stamps, q = synth.imu_stream(-1.0, 0.5)   # ends before scan 8
    ok, c_ref, _, st_ref = oracle_lib.imu_preprocess(pts, st, stamps, q, (0, 0, 1, 0))
    h = _handler(floam_gpu, stamps, q)
    din, dal = floam_gpu.DeviceCloud(pts), floam_gpu.DeviceCloud()
    ok_g, st_g = imu.preprocess(din, st, h, (0, 0, 1, 0), dal)
    assert not ok and not ok_g and st_g == st_ref
    _same(din.download(), c_ref, "centred")
    assert len(dal) == 0


def test_times_outside_window_and_nan(floam_gpu, oracle_lib):
    """Points whose times lie outside [front, back] (unsorted times) search the whole stream; a few land outside
    the IMU stream entirely (zero orientation -> point unchanged by the compensation); NaN coordinates propagate."""
    from floam_amd import imu
    pts, st = synth.driver_scan("c1", 1)
    rng = np.random.default_rng(5)
    sel = rng.choice(pts.shape[0] - 2, 200, replace=False) + 1
    pts["time"][sel] = rng.uniform(-3.0, 3.0, sel.shape[0]).astype(np.float32)
    pts["x"][sel[:5]] = np.nan
    stamps, q = synth.imu_stream(-1.5, 1.5)
    extr = np.array([0.0, 0.0, 1.0, 0.0])
    ok, c_ref, a_ref, st_ref = oracle_lib.imu_preprocess(pts, st, stamps, q, extr)
    h = _handler(floam_gpu, stamps, q)
    din, dal = floam_gpu.DeviceCloud(pts), floam_gpu.DeviceCloud()
    ok_g, st_g = imu.preprocess(din, st, h, extr, dal)
    assert ok and ok_g and st_g == st_ref
    _same(din.download(), c_ref, "centred")
    _same(dal.download(), a_ref, "aligned")


def test_golden_vectors(floam_gpu):
    import os
    from floam_amd import imu
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "imu_c1.npz"))
    pts = g["input"].view(synth.POINT_DTYPE)
    h = _handler(floam_gpu, g["imu_stamps"], g["imu_q"])
    din, dal = floam_gpu.DeviceCloud(pts), floam_gpu.DeviceCloud()
    ok, st = imu.preprocess(din, int(g["stamp_us"]), h, g["extrinsics"], dal)
    assert ok and st == int(g["stamp_out_us"])
    _same(din.download(), g["centred"].view(synth.POINT_DTYPE), "centred")
    _same(dal.download(), g["aligned"].view(synth.POINT_DTYPE), "aligned")


def test_empty_cloud(floam_gpu):
    from floam_amd import imu
    stamps, q = synth.imu_stream(-1.0, 1.0)
    h = _handler(floam_gpu, stamps, q)
    din, dal = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
    ok, st = imu.preprocess(din, 1234, h, (0, 0, 1, 0), dal)
    assert not ok and st == 1234
    assert imu.CenterTime(din, 99) == 99


def test_handler_lookups(floam_gpu, oracle_lib):
    stamps, q = synth.imu_stream(-0.5, 0.5, rate=150.0)
    h = floam_gpu.ImuHandler()
    added = [h.AddMsg(s, qq) for s, qq in zip(stamps, q)]
    np.testing.assert_array_equal(added, oracle_lib.imu_filter(stamps))
    assert h.size() == int(np.sum(added))
    kept = stamps[np.asarray(added)]
    for ts in np.concatenate([kept[:3], kept[-2:], kept[:-1] + 1e-4, [kept[0] - 1.0, kept[-1] + 1.0]]):
        got, found = h.Get(ts)
        want, wfound = oracle_lib.imu_get(stamps, q, ts)
        assert found == wfound
        np.testing.assert_array_equal(got, want)
        assert h.TimeContained(ts) == oracle_lib.imu_time_contained(stamps, q, ts)
