"""GPU parity of the VoxelGrid pipeline (floam_voxel_grid, voxel.hip) against the CPU oracle's PCL 1.8.1 restatement
(oracle/pcl_filters.cpp, stable within-voxel order): centroids bit-identical, same order, same count.

Covers the cases the single-pass compaction has to get right: voxels whose run of sorted points crosses one or
several 1024-element tiles, the index-overflow pass-through (Q9), empty input, and both leaf sizes of the path.
"""
import numpy as np
import pytest

from floam_amd import synth

pytestmark = pytest.mark.gpu


def _cloud(xyz, intensity=None):
    a = np.zeros(xyz.shape[0], synth.POINT_DTYPE)
    a["x"], a["y"], a["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    a["pad0"] = 1.0
    a["intensity"] = intensity if intensity is not None else np.arange(xyz.shape[0]) % 255
    return a


def _check(floam_gpu, oracle_lib, pts, leaf):
    ref = oracle_lib.voxel_grid(pts, leaf, stable=True)
    got = floam_gpu.DeviceCloud(pts).voxel_grid(leaf).download()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    for f in ("x", "y", "z", "intensity"):
        np.testing.assert_array_equal(got[f], ref[f], err_msg=f)
    return got


@pytest.mark.parametrize("leaf", [0.1, 0.2, 0.4])
def test_voxel_random(floam_gpu, oracle_lib, leaf):
    rng = np.random.default_rng(7)
    pts = _cloud(rng.uniform(-20, 20, (50000, 3)).astype(np.float32))
    _check(floam_gpu, oracle_lib, pts, leaf)


def test_voxel_scan_features(floam_gpu, oracle_lib):
    raw = synth.generate_scan("c3", 1)
    e, s, _ = oracle_lib.feature_extraction(raw, 64, 0.5, 90.0, canonical=True)
    _check(floam_gpu, oracle_lib, synth.to_xyzi(s), 0.2)
    _check(floam_gpu, oracle_lib, synth.to_xyzi(e), 0.1)


def test_voxel_runs_cross_tiles(floam_gpu, oracle_lib):
    """5000 points in one voxel (a sorted run spanning ~5 compaction tiles) amid scattered points."""
    rng = np.random.default_rng(3)
    dense = rng.uniform(1.01, 1.09, (5000, 3))
    sparse = rng.uniform(-5, 5, (3000, 3))
    pts = _cloud(np.concatenate([sparse[:1500], dense, sparse[1500:]]).astype(np.float32))
    got = _check(floam_gpu, oracle_lib, pts, 0.1)
    assert got.shape[0] < pts.shape[0]


def test_voxel_overflow_passthrough(floam_gpu, oracle_lib):
    """dx*dy*dz > INT_MAX: PCL returns the input unchanged (Q9)."""
    rng = np.random.default_rng(5)
    pts = _cloud(rng.uniform(-1e5, 1e5, (2000, 3)).astype(np.float32))
    got = _check(floam_gpu, oracle_lib, pts, 0.05)
    assert got.shape[0] == pts.shape[0]


def test_voxel_empty(floam_gpu):
    out = floam_gpu.DeviceCloud(_cloud(np.zeros((0, 3), np.float32))).voxel_grid(0.1)
    assert len(out) == 0


def test_voxel_dense_bucket_streams(floam_gpu, oracle_lib):
    """bucket.hip: 20000 points in 12 voxels of one thin slab share one fine-histogram bin, so one bucket exceeds
    the 8192 elements a block sorts in LDS and is sorted through global memory (stream_sort, two digit passes over
    the slab's key range); runs of ~1700 points also cross many compaction tiles.  Sparse points around it fill
    the other buckets."""
    rng = np.random.default_rng(11)
    dense = np.stack([rng.uniform(1.0, 1.6, 20000), rng.uniform(1.0, 1.2, 20000), rng.uniform(1.0, 1.1, 20000)], 1)
    sparse = rng.uniform(-50, 50, (6000, 3))
    pts = _cloud(np.concatenate([sparse[:3000], dense, sparse[3000:]]).astype(np.float32))
    got = _check(floam_gpu, oracle_lib, pts, 0.1)
    assert got.shape[0] < pts.shape[0]


@pytest.mark.parametrize("n", [1, 63, 257, 8193])
def test_voxel_small_and_ragged(floam_gpu, oracle_lib, n):
    """Counts around the sort's block and wave sizes, a few voxels each (one bucket, one digit pass or none)."""
    rng = np.random.default_rng(n)
    pts = _cloud(rng.uniform(0.0, 0.35, (n, 3)).astype(np.float32))
    _check(floam_gpu, oracle_lib, pts, 0.1)


def test_voxel_run_lengths(floam_gpu, oracle_lib):
    """Voxels of every run length 1..40 plus 100 and 257 points, shuffled: every residue of the compaction's 8-point
    groups (bucket.hip emit loop: full groups added without tests, the last group tested per element), runs that end
    on a group boundary or at the end of a bucket, and runs long enough for several double-buffered groups.  The
    second call sorts with the splitters the first one wrote (balanced buckets: the in-LDS path)."""
    rng = np.random.default_rng(17)
    lens = list(range(1, 41)) + [100, 257]
    blocks = []
    for _ in range(12):
        for n in lens:
            base = rng.integers(-60, 60, 3) * 3 * 0.1   # voxel corners three cells apart (no index overflow)
            blocks.append(base + rng.uniform(0.01, 0.09, (n, 3)))
    xyz = np.concatenate(blocks)
    xyz = xyz[rng.permutation(len(xyz))].astype(np.float32)
    pts = _cloud(xyz, intensity=rng.uniform(0.0, 255.0, len(xyz)).astype(np.float32))
    first = _check(floam_gpu, oracle_lib, pts, 0.1)
    second = _check(floam_gpu, oracle_lib, pts, 0.1)
    assert first.shape[0] <= 12 * len(lens) and second.shape == first.shape


def test_voxel_stale_splitters_overflow(floam_gpu, oracle_lib):
    """bucket.hpp bucket_append: a bucket's region holds twice the mean bucket; appends past it go to the overflow
    list, which the bucket's block gathers back (bucket.hip bucket_source).  Splitters seeded by a spread-out cloud,
    then clouds whose points crowd into a few of those buckets: one bucket past its region but within the in-LDS
    network (3000 points in a 0.3-m cube), one past the network too (20000 points of a thin slab: streamed, sorted by
    (key, value) through global memory), then the spread-out cloud again with the crowded splitters."""
    rng = np.random.default_rng(23)
    spread = _cloud(rng.uniform(-30, 30, (40000, 3)).astype(np.float32))
    _check(floam_gpu, oracle_lib, spread, 0.1)
    _check(floam_gpu, oracle_lib, spread, 0.1)   # (sorted with its own splitters: balanced)
    cube = np.concatenate([rng.uniform(2.0, 2.3, (3000, 3)), rng.uniform(-30, 30, (500, 3))])
    _check(floam_gpu, oracle_lib, _cloud(cube[rng.permutation(len(cube))].astype(np.float32)), 0.1)
    _check(floam_gpu, oracle_lib, spread, 0.1)
    slab = np.stack([rng.uniform(4.0, 4.6, 20000), rng.uniform(4.0, 4.2, 20000), rng.uniform(4.0, 4.1, 20000)], 1)
    slab = np.concatenate([slab, rng.uniform(-30, 30, (2000, 3))])
    _check(floam_gpu, oracle_lib, _cloud(slab[rng.permutation(len(slab))].astype(np.float32)), 0.1)
    _check(floam_gpu, oracle_lib, spread, 0.1)
