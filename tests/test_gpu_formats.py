"""GPU parity of the wire formats through the C ABI against the CPU oracle: PointCloud2 decoding
(pcl::fromROSMsg) byte-identical to the oracle's restatement on driver-like layouts (whole-record copy, coalesced
and scattered field mappings, organised clouds with row padding, a mismatched field), toROSMsg -> fromROSMsg round
trips, the double-affine transform, and SaveMerged's device transform + VoxelGrid against the oracle."""
import numpy as np
import pytest

from floam_amd import synth
from tests import pc2_layouts as L

pytestmark = pytest.mark.gpu


def _msg(formats, raw):
    data, w, h, ps, rs, fields = raw
    return formats.PointCloud2(height=h, width=w, fields=[formats.PointField(*f) for f in fields], point_step=ps,
                               row_step=rs, data=data)


@pytest.mark.parametrize("layout,ptype", [("velodyne", 0), ("ouster_like", 0), ("packed_reordered", 0),
                                          ("ouster_like", 1)])
def test_decode_bit_exact(floam_gpu, oracle_lib, layout, ptype):
    from floam_amd import formats
    pts = synth.generate_scan("c1", 2)
    raw = getattr(L, layout)(pts)
    ref, missing = oracle_lib.from_pointcloud2(*raw, point_type=ptype)
    d = floam_gpu.DeviceCloud()
    ok = formats.fromROSMsg(_msg(formats, raw), d, ptype)
    assert ok == (missing == 0)
    got = d.download()
    np.testing.assert_array_equal(got.view(np.uint8), ref.view(np.uint8))   # every byte, padding included


def test_roundtrip_and_empty(floam_gpu):
    from floam_amd import formats
    pts = synth.generate_scan("c1", 4)
    d = floam_gpu.DeviceCloud(pts)
    msg = formats.toROSMsg(d, formats.XYZIRT, stamp=12.5, frame_id="base_link")
    assert msg.point_step == 32 and msg.width == pts.shape[0] and msg.row_step == 32 * pts.shape[0]
    d2 = floam_gpu.DeviceCloud()
    assert formats.fromROSMsg(msg, d2)
    np.testing.assert_array_equal(d2.download().view(np.uint8), pts.view(np.uint8))
    empty = formats.PointCloud2(width=0, height=1, fields=msg.fields, point_step=32, row_step=0, data=b"")
    assert formats.fromROSMsg(empty, d2) and len(d2) == 0


def test_transform_bit_exact(floam_gpu, oracle_lib):
    from floam_amd import formats
    pts = synth.generate_scan("c3", 1)
    T = synth.gt_pose_matrix(37)
    T[:3, :3] = T[:3, :3] @ np.array([[1, 0, 0], [0, 0.6, -0.8], [0, 0.8, 0.6]])
    d_in, d_out = floam_gpu.DeviceCloud(pts), floam_gpu.DeviceCloud()
    formats.transformPointCloud(d_in, d_out, T)
    np.testing.assert_array_equal(d_out.download().view(np.uint8), oracle_lib.transform_cloud(pts, T).view(np.uint8))
    formats.transformPointCloud(d_in, d_in, T)   # in place
    np.testing.assert_array_equal(d_in.download().view(np.uint8), oracle_lib.transform_cloud(pts, T).view(np.uint8))


def test_save_merged(floam_gpu, oracle_lib, tmp_path):
    from floam_amd import formats
    clouds = [synth.to_xyzi(synth.generate_scan("c1", k)) for k in range(3)]
    P = [synth.gt_pose_matrix(k) for k in range(3)]
    d = str(tmp_path / "merged") + "/"
    formats.SaveMerged(clouds, P, d, 0.5)
    merged = formats.loadPCDFileBinary(d + "floam_merged.pcd")
    ref = np.concatenate([oracle_lib.transform_cloud(c, T) for c, T in zip(clouds, P)])
    for f in ("x", "y", "z", "intensity"):
        np.testing.assert_array_equal(merged[f], ref[f])
    down = formats.loadPCDFileBinary(d + "floam_merged_downsampled_leaf_0.500000.pcd")
    vref = oracle_lib.voxel_grid(ref, 0.5, stable=True)
    for f in ("x", "y", "z", "intensity"):
        np.testing.assert_array_equal(down[f], vref[f])
