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
            "fallback": {"FLOAM_MM_VIOLATE": "2"},
            # 512-element merge tiles: more runs cross a tile edge
            "merge512": {"FLOAM_MM_PER": "2"}}
KNOBS = ("FLOAM_MAP_FULL", "FLOAM_MAP_MERGE", "FLOAM_MM_VIOLATE", "FLOAM_MM_PER")


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


def _slab(x, y, z):
    """map records on the grid x (outer) * y * z (inner): one per 0.1-m cell centre"""
    from floam_amd.synth import POINT_DTYPE
    X, Y, Z = np.meshgrid(np.asarray(x, np.float32), np.asarray(y, np.float32), np.asarray(z, np.float32),
                          indexing="ij")
    out = np.zeros(X.size, POINT_DTYPE)
    out["x"], out["y"], out["z"] = X.ravel(), Y.ravel(), Z.ravel()
    out["pad0"] = 1.0
    out["intensity"] = (np.arange(X.size) % 251).astype(np.float32)
    return out


@pytest.mark.parametrize("variant", ["merge", "merge512"])
def test_merge_crops_map_points(floam_gpu, monkeypatch, prefilled_map, variant):
    """CropBox [t - 100, t + 100] removes map points once the sensor has moved; the merge saturates
    a cropped point's index to the first / last cell of its row or plane (map_idx), so runs of several cropped points
    — and a cropped point sharing its voxel index with a kept map point — occur and cross tile edges.  The C2 map is
    prefilled with two slabs right inside the first update's crop box: one behind the sensor's direction of travel
    (+x: a 0.1-m slice per scan leaves the box; its cropped points share a row's first index with the next kept
    slice) and one at y = -100 (the trajectory drifts +y: whole slices leave at once and all of a z plane's cropped
    points share one index).  Maps after every update byte-identical to the whole-map VoxelGrid's, never a NaN."""
    E, S = prefilled_map("c2")
    zs = np.arange(-1.45, 2.5, 0.1)
    xslab = _slab(np.arange(-99.85, -97.9, 0.1), np.arange(-9.95, 10.0, 0.1), zs)
    yslab = _slab(np.arange(-19.95, 20.0, 0.1), [-99.98, -99.94, -99.9, -99.86, -99.82], zs)
    prefill = (np.concatenate([E, xslab, yslab]), np.concatenate([S, xslab, yslab]))
    nscan = 20
    runs = {v: _run(floam_gpu, monkeypatch, v, "c2", nscan, prefill) for v in (variant, "voxelgrid")}
    assert sum(r[3] for r in runs[variant]) >= 10, "too few keyframes to exercise the merge"
    for (_, e, s, _) in runs[variant]:
        for m in (e, s):
            assert np.all(np.isfinite(m["x"]) & np.isfinite(m["y"]) & np.isfinite(m["z"])), "NaN in the merged map"
    # the slabs really were cropped along the way (the run's last map lost most of both)
    e_last = runs[variant][-1][1]
    assert np.count_nonzero(e_last["x"] < -97.8) < xslab.size // 4, "the x slab was not cropped"
    assert np.count_nonzero(e_last["y"] < -99.8) < yslab.size // 2, "the y slab was not cropped"
    _same(runs[variant], runs["voxelgrid"], f"c2 cropping slabs {variant} vs whole-map VoxelGrid")
