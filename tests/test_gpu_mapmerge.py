"""The incremental map update (floam_amd/csrc/mapmerge.hip): the downsampled scan's voxels merged into the
voxel-ordered map must give exactly the reference's whole-map re-voxelisation (addPointsToMap,
src/odomEstimationClass.cpp:253-294) — the same maps byte for byte and the same poses as (1) the merge pipeline forced
onto its full-sort path and (2) the round-2 whole-map VoxelGrid (FLOAM_MAP_MERGE=0)."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu

VARIANTS = {"merge": {}, "full": {"FLOAM_MAP_FULL": "1"}, "voxelgrid": {"FLOAM_MAP_MERGE": "0"},
            # every other merge reports its keys out of order: the next update takes the full sort, then merges again
            "fallback": {"FLOAM_MM_VIOLATE": "2"}}
KNOBS = ("FLOAM_MAP_FULL", "FLOAM_MAP_MERGE", "FLOAM_MM_VIOLATE")


def _params(R):
    from floam_amd import LidarParams
    return LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)


def _run(floam_gpu, monkeypatch, variant, config, nscan, prefill=None, repeat=()):
    from floam_amd.odom_estimation import reset_process_state
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in VARIANTS[variant].items():
        monkeypatch.setenv(k, v)
    R = synth.lidar_model(config).rings
    reset_process_state()
    lp = floam_gpu.LaserProcessingClass()
    lp.init(_params(R))
    odo = floam_gpu.OdomEstimationClass()
    odo.init(_params(R), 0.1, "Cauchy")
    out = []
    first = 0
    if prefill is not None:
        odo.initMapWithPoints(floam_gpu.DeviceCloud(prefill[0]), floam_gpu.DeviceCloud(prefill[1]))
        first = 1
    for k in range(first, first + nscan):
        scan = k - 1 if k in repeat else k   # a repeated scan: the pose barely moves -> no keyframe, map kept
        de, ds = floam_gpu.DeviceCloud(), floam_gpu.DeviceCloud()
        lp.featureExtraction(floam_gpu.DeviceCloud(synth.generate_scan(config, scan)), de, ds)
        if k == 0:
            odo.initMapWithPoints(de, ds)
            continue
        odo.UpdatePointsToMapSelector(de, ds, True)
        st = odo.stats()
        out.append((odo.pose(), odo.laserCloudCornerMap, odo.laserCloudSurfMap, st["map_updated"]))
    return out


def _same(a, b, what):
    for k, ((pa, ea, sa, ua), (pb, eb, sb, ub)) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(pa[0], pb[0], err_msg=f"{what} scan {k} q")
        np.testing.assert_array_equal(pa[1], pb[1], err_msg=f"{what} scan {k} t")
        assert ua == ub, (what, k)
        for m, (x, y) in enumerate(((ea, eb), (sa, sb))):
            assert x.shape == y.shape, (what, k, m, x.shape, y.shape)
            np.testing.assert_array_equal(x.view(np.uint8), y.view(np.uint8), err_msg=f"{what} scan {k} map {m}")


@pytest.mark.parametrize("config,nscan", [("c1", 8), ("c3", 4)])
def test_merge_equals_full_voxelgrid(floam_gpu, monkeypatch, prefilled_map, config, nscan):
    """From a raw map (initMapWithPoints: the first update re-voxelises it by the full sort, later ones merge): maps
    byte-identical after every scan, poses bit-identical, across the three paths."""
    prefill = prefilled_map(config) if config != "c1" else None
    runs = {v: _run(floam_gpu, monkeypatch, v, config, nscan, prefill) for v in VARIANTS}
    assert any(r[3] for r in runs["merge"]), "no keyframe: the merge never ran"
    _same(runs["merge"], runs["full"], f"{config} merge vs full")
    _same(runs["merge"], runs["voxelgrid"], f"{config} merge vs whole-map VoxelGrid")
    _same(runs["merge"], runs["fallback"], f"{config} merge vs merge with full-sort fallbacks")


def test_merge_after_skipped_keyframe(floam_gpu, monkeypatch):
    """A non-keyframe update copies the maps and their cell keys; the next keyframe merges into the copy."""
    runs = {v: _run(floam_gpu, monkeypatch, v, "c1", 7, repeat=(4,)) for v in ("merge", "voxelgrid")}
    assert not all(r[3] for r in runs["merge"]), "every update was a keyframe: the copy path never ran"
    _same(runs["merge"], runs["voxelgrid"], "c1 with a repeated scan")


def test_merge_long_sequence(floam_gpu, monkeypatch, prefilled_map):
    """20 C2 updates from the prefilled map: every map after every update byte-identical to the whole-map VoxelGrid's
    (the merge's order invariant checked on the device all along; a violation would take the full sort, which is
    also exact)."""
    prefill = prefilled_map("c2")
    runs = {v: _run(floam_gpu, monkeypatch, v, "c2", 20, prefill) for v in ("merge", "voxelgrid")}
    assert sum(r[3] for r in runs["merge"]) >= 10, "too few keyframes to exercise the merge"
    _same(runs["merge"], runs["voxelgrid"], "c2 x 20 merge vs whole-map VoxelGrid")
