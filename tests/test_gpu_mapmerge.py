"""The incremental map update (floam_amd/csrc/mapmerge.hip): the downsampled scan's voxels merged into the
voxel-ordered map must give exactly the reference's whole-map re-voxelisation (addPointsToMap,
src/odomEstimationClass.cpp:253-294) — the same maps byte for byte and the same poses as (1) the merge pipeline forced
onto its full-sort path and (2) the round-2 whole-map VoxelGrid (FLOAM_MAP_MERGE=0)."""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu

# product-library variants (FLOAM_MAP_MERGE is a product variable) and diagnostic-build ones (tests/diag.py)
VARIANTS = {"merge": {}, "voxelgrid": {"FLOAM_MAP_MERGE": "0"},
            # the merge pipeline forced onto its full-sort path
            "full": {"FLOAM_MAP_FULL": "1"},
            # every other merge reports its keys out of order: the next update takes the full sort, then merges again
            "fallback": {"FLOAM_MM_VIOLATE": "2"},
            # 512-element merge tiles (twice the tile edges for runs, cropped-point runs included, to cross)
            "tiles512": {"FLOAM_MM_PER": "2"}}
DIAG_VARIANTS = ("full", "fallback", "tiles512")


def _params(R):
    from floam_amd import LidarParams
    return LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)


def _sequence(floam, config, nscan, prefill=None, repeat=()):
    from floam_amd.odom_estimation import reset_process_state
    R = synth.lidar_model(config).rings
    reset_process_state()
    lp = floam.LaserProcessingClass()
    lp.init(_params(R))
    odo = floam.OdomEstimationClass()
    odo.init(_params(R), 0.1, "Cauchy")
    out = []
    first = 0
    if prefill is not None:
        odo.initMapWithPoints(floam.DeviceCloud(prefill[0]), floam.DeviceCloud(prefill[1]))
        first = 1
    for k in range(first, first + nscan):
        scan = k - 1 if k in repeat else k   # a repeated scan: the pose barely moves -> no keyframe, map kept
        de, ds = floam.DeviceCloud(), floam.DeviceCloud()
        lp.featureExtraction(floam.DeviceCloud(synth.generate_scan(config, scan)), de, ds)
        if k == 0:
            odo.initMapWithPoints(de, ds)
            continue
        odo.UpdatePointsToMapSelector(de, ds, True)
        st = odo.stats()
        out.append((odo.pose(), odo.laserCloudCornerMap, odo.laserCloudSurfMap, st["map_updated"]))
    return out


def _sequence_child(config, nscan, prefill, repeat):
    import floam_amd
    return _sequence(floam_amd, config, nscan, prefill, repeat)


def _run(floam_gpu, monkeypatch, variant, config, nscan, prefill=None, repeat=()):
    if variant in DIAG_VARIANTS:
        from tests.diag import run_diag
        return run_diag(_sequence_child, config, nscan, prefill, tuple(repeat), env=VARIANTS[variant])
    monkeypatch.delenv("FLOAM_MAP_MERGE", raising=False)
    for k, v in VARIANTS[variant].items():
        monkeypatch.setenv(k, v)
    return _sequence(floam_gpu, config, nscan, prefill, repeat)


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
    _same(runs["merge"], runs["tiles512"], f"{config} merge vs merge with 512-element tiles")


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


def _c2_crop_prefill(prefilled_map):
    """the C2 prefill plus two slabs right inside the first update's crop box (test_merge_crops_map_points)"""
    E, S = prefilled_map("c2")
    zs = np.arange(-1.45, 2.5, 0.1)
    xslab = _slab(np.arange(-99.85, -97.9, 0.1), np.arange(-9.95, 10.0, 0.1), zs)
    yslab = _slab(np.arange(-19.95, 20.0, 0.1), [-99.98, -99.94, -99.9, -99.86, -99.82], zs)
    return (np.concatenate([E, xslab, yslab]), np.concatenate([S, xslab, yslab])), xslab, yslab


def _c3_crop_prefill(prefilled_map):
    """the C3 prefill plus points OUTSIDE the first update's crop box [t - 100, t + 100] (t near the origin): a slab
    straddling the -x face (x in -100.55 .. -99.45, half of it cropped at once), a slab beyond +y (cropped whole) and a
    block past +z"""
    E, S = prefilled_map("c3")
    zs = np.arange(-1.45, 2.5, 0.1)
    a = _slab(np.arange(-100.55, -99.4, 0.1), np.arange(-9.95, 10.0, 0.1), zs)
    b = _slab(np.arange(-19.95, 20.0, 0.1), np.arange(100.35, 101.0, 0.1), zs)
    c = _slab(np.arange(-4.95, 5.0, 0.1), np.arange(-4.95, 5.0, 0.1), np.arange(100.25, 100.9, 0.1))
    extra = np.concatenate([a, b, c])
    return (np.concatenate([E, extra]), np.concatenate([S, extra])), extra


def _oracle_sequence(oracle_lib, config, nscan, prefill):
    R = synth.lidar_model(config).rings
    ref = oracle_lib.Odometry(R, 0.1, 0.5, 90.0, 0.1, "Cauchy", stable_voxel=True)
    oracle_lib.reset_process_statics()
    ref.init_map(*prefill)
    out = []
    for k in range(1, nscan + 1):
        e, s_, _ = oracle_lib.feature_extraction(synth.generate_scan(config, k), R, 0.5, 90.0, canonical=True)
        ref.update_selector(e, s_, True)
        out.append((ref.pose(), ref.map(0), ref.map(1)))
    return out


def _outside_box(m, t):
    """map points outside CropBox [t - 100, t + 100] (inclusive bounds, float compare: src/odomEstimationClass.cpp
    :270-287)"""
    lo, hi = (t - 100.0).astype(np.float32), (t + 100.0).astype(np.float32)
    xyz = np.stack([m["x"], m["y"], m["z"]], axis=1)
    return int(np.count_nonzero(np.any((xyz < lo) | (xyz > hi), axis=1)))


@pytest.mark.parametrize("config,nscan", [("c2", 20), ("c3", 4)])
def test_crop_box_matches_oracle(floam_gpu, oracle_lib, monkeypatch, prefilled_map, config, nscan):
    """VERDICT r04 Weak 2: the map update's CropBox (addPointsToMap, src/odomEstimationClass.cpp:270-294) against the
    oracle on runs that really crop — C2 with the two slabs that leave the box scan by scan, C3 with a prefill that
    extends past the first update's box.  Both GPU paths (the merge and the whole-map VoxelGrid) after every update:
    the same voxels in the same order as the oracle's maps, coordinates within 1 ulp, poses within 1e-6; and points
    were actually cropped."""
    from tests.test_gpu_parity import _angle_between, _assert_map_close
    if config == "c2":
        prefill, xslab, yslab = _c2_crop_prefill(prefilled_map)
    else:
        prefill, extra = _c3_crop_prefill(prefilled_map)
    ref = _oracle_sequence(oracle_lib, config, nscan, prefill)
    for variant in ("merge", "voxelgrid"):
        run = _run(floam_gpu, monkeypatch, variant, config, nscan, prefill)
        for k, ((pose, e, s_, _), ((qr, tr), er, sr)) in enumerate(zip(run, ref)):
            dt, dr = float(np.linalg.norm(pose[1] - tr)), _angle_between(pose[0], qr)
            assert dt < 1e-6 and dr < 1e-6, (variant, config, k, dt, dr)
            _assert_map_close(e, er, f"{variant} {config} scan {k + 1} corner map")
            _assert_map_close(s_, sr, f"{variant} {config} scan {k + 1} surf map")
            # CropBox at this update's pose: nothing outside the box survives (voxel centroids of kept points stay
            # inside it too: every kept point of a voxel lies in the box, which is convex)
            assert _outside_box(e, tr) == 0 and _outside_box(s_, tr) == 0, (variant, config, k)
    # the runs really cropped: prefill points were outside the first box, or left it along the way
    (q1, t1), e1, _ = ref[0]
    if config == "c3":
        assert _outside_box(extra, t1) > extra.size // 3, "the C3 prefill did not extend past the first crop box"
        assert np.count_nonzero(np.abs(e1["y"]) > 100.0) == 0
    else:
        e_last = ref[-1][1]
        assert np.count_nonzero(e_last["x"] < -97.8) < xslab.size // 4, "the x slab was not cropped"
        assert np.count_nonzero(e_last["y"] < -99.8) < yslab.size // 2, "the y slab was not cropped"


def test_merge_crops_map_points(floam_gpu, monkeypatch, prefilled_map):
    """CropBox [t - 100, t + 100] removes map points once the sensor has moved; the merge saturates
    a cropped point's index to the first / last cell of its row or plane (map_idx), so runs of several cropped points
    — and a cropped point sharing its voxel index with a kept map point — occur and cross tile edges.  The C2 map is
    prefilled with two slabs right inside the first update's crop box: one behind the sensor's direction of travel
    (+x: a 0.1-m slice per scan leaves the box; its cropped points share a row's first index with the next kept
    slice) and one at y = -100 (the trajectory drifts +y: whole slices leave at once and all of a z plane's cropped
    points share one index).  Maps after every update byte-identical to the whole-map VoxelGrid's, never a NaN."""
    prefill, xslab, yslab = _c2_crop_prefill(prefilled_map)
    nscan = 20
    variant = "merge"
    runs = {v: _run(floam_gpu, monkeypatch, v, "c2", nscan, prefill) for v in (variant, "voxelgrid", "tiles512")}
    assert sum(r[3] for r in runs[variant]) >= 10, "too few keyframes to exercise the merge"
    for (_, e, s, _) in runs[variant]:
        for m in (e, s):
            assert np.all(np.isfinite(m["x"]) & np.isfinite(m["y"]) & np.isfinite(m["z"])), "NaN in the merged map"
    # the slabs really were cropped along the way (the run's last map lost most of both)
    e_last = runs[variant][-1][1]
    assert np.count_nonzero(e_last["x"] < -97.8) < xslab.size // 4, "the x slab was not cropped"
    assert np.count_nonzero(e_last["y"] < -99.8) < yslab.size // 2, "the y slab was not cropped"
    _same(runs[variant], runs["voxelgrid"], f"c2 cropping slabs {variant} vs whole-map VoxelGrid")
    _same(runs["tiles512"], runs["voxelgrid"], "c2 cropping slabs, 512-element merge tiles, vs whole-map VoxelGrid")
