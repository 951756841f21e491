"""CPU: wire / disk formats.  The oracle's fromPCLPointCloud2 restatement against an independent
per-field numpy decode on driver-like layouts, the field table the library reports (host call, no GPU), the PCD
writer, and the exporters' text formats.  The reference has no tests for these; the expected text is derived from
the C++ stream / boost::format / Eigen printing rules the reference's code relies on (parity unpinned against real
files, none ship with the reference)."""
import math
import os

import numpy as np
import pytest

from floam_amd import synth
from tests import pc2_layouts as L

NAMED = ("x", "y", "z", "intensity", "ring", "time")


def _named_equal(a, b, fields=NAMED):
    for f in fields:
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


def test_field_table_matches_toROSMsg():
    from floam_amd import formats
    f, step = formats.fields_of(formats.XYZIRT)
    assert step == 32
    assert [(x.name, x.offset, x.datatype, x.count) for x in f] == [
        ("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1), ("intensity", 16, 7, 1), ("ring", 20, 4, 1), ("time", 24, 7, 1)]
    f, _ = formats.fields_of(formats.XYZI)
    assert [x.name for x in f] == ["x", "y", "z", "intensity"]


@pytest.mark.parametrize("layout", ["velodyne", "ouster_like", "packed_reordered"])
def test_oracle_decode_matches_numpy(oracle_lib, layout):
    pts = synth.generate_scan("tiny16x200", 1)
    msg = getattr(L, layout)(pts)
    out, missing = oracle_lib.from_pointcloud2(*msg)
    ref = L.reference_decode(*msg)
    _named_equal(out, ref)
    assert missing == (1 if layout == "packed_reordered" else 0)   # ring declared uint8: no match
    if layout == "packed_reordered":
        assert not out["ring"].any()
    else:
        n = out.shape[0]
        _named_equal(out, pts[:n])
    if layout == "velodyne":   # one coalesced mapping, point_step 32: whole records copied, padding included
        np.testing.assert_array_equal(out.view(np.uint8), np.frombuffer(msg[0], np.uint8))


def test_oracle_decode_xyzi(oracle_lib):
    pts = synth.generate_scan("tiny16x200", 2)
    out, missing = oracle_lib.from_pointcloud2(*L.ouster_like(pts), point_type=1)
    assert missing == 0
    n = out.shape[0]
    _named_equal(out, pts[:n], ("x", "y", "z", "intensity"))
    assert not out["ring"].any() and not out["time"].any()


def test_oracle_transform(oracle_lib):
    pts = synth.generate_scan("tiny16x200", 3)
    T = synth.gt_pose_matrix(7)
    out = oracle_lib.transform_cloud(pts, T)
    x, y, z = (pts[f].astype(np.float64) for f in "xyz")
    for r, f in enumerate("xyz"):
        want = (((T[r, 0] * x + T[r, 1] * y) + T[r, 2] * z) + T[r, 3]).astype(np.float32)
        np.testing.assert_array_equal(out[f], want)
    _named_equal(out, pts, ("intensity", "ring", "time"))


def test_pcd_binary_roundtrip(tmp_path):
    from floam_amd import formats
    pts = synth.to_xyzi(synth.generate_scan("tiny16x200", 4))
    p = str(tmp_path / "c.pcd")
    formats.savePCDFileBinary(p, pts)
    raw = open(p, "rb").read()
    hdr = raw[: raw.index(b"DATA binary\n") + 12].decode()
    assert hdr == ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\nSIZE 4 4 4 4\n"
                   "TYPE F F F F\nCOUNT 1 1 1 1\nWIDTH %d\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS %d\nDATA binary\n"
                   % (pts.shape[0], pts.shape[0]))
    assert len(raw) == len(hdr) + 16 * pts.shape[0]
    back = formats.loadPCDFileBinary(p)
    _named_equal(back, pts, ("x", "y", "z", "intensity"))


def test_text_helpers():
    from floam_amd import formats
    assert formats._g(1.0) == "1" and formats._g(0.1234567) == "0.123457" and formats._g(1e-7) == "1e-07"
    assert formats._g(-0.0) == "-0" and formats._g(123456789.0) == "1.23457e+08"
    m = np.array([[1.0, 0.0, 0.0, 12.5], [0.0, -1.0, 0.0, 0.0], [0.0, 0.0, 1.0, -3.25], [0.0, 0.0, 0.0, 1.0]])
    assert formats.eigen_str(m) == ("    1     0     0  12.5\n    0    -1     0     0\n"
                                    "    0     0     1 -3.25\n    0     0     0     1")
    assert formats.ros_time(1700000000.25) == (1700000000, 250000000)
    assert formats.ros_time(1700000000.0999999) == (1700000000, 99999905)   # (t - sec) * 1e9 in double
    assert formats.ros_time(2.9999999999) == (3, 0)


def _poses(n):
    return [synth.gt_pose_matrix(k) for k in range(n)]


def test_save_odom_and_posegraph(tmp_path):
    from floam_amd import formats
    P = _poses(3)
    stamps = [synth.EPOCH + 0.1 * k for k in range(3)]
    clouds = [synth.to_xyzi(synth.generate_scan("tiny16x200", k)) for k in range(3)]
    d = str(tmp_path / "odom")
    formats.SaveOdom(d, P, stamps, clouds)
    sec, nsec = formats.ros_time(stamps[1])
    txt = open(os.path.join(d, f"{sec}_{nsec}.odom")).read().splitlines()
    assert len(txt) == 4 and txt[3] == "0 0 0 1"
    assert [float(v) for v in txt[0].split()] == pytest.approx(list(P[1][0]), rel=1e-5, abs=1e-6)
    g = str(tmp_path / "graph")
    formats.SavePosegraph(g, P, stamps, clouds)
    lines = open(os.path.join(g, "graph.g2o")).read().splitlines()
    assert lines[0].startswith("VERTEX_SE3:QUAT 0 0 0 0 0 0 0 1") and lines[3] == "FIX 0"
    e = lines[4].split()
    assert e[:3] == ["EDGE_SE3:QUAT", "0", "1"] and len(e) == 3 + 7 + 21
    # relative motion of one scan: 0.1 m forward, 0.5 deg yaw
    assert float(e[3]) == pytest.approx(0.1, abs=1e-3) and float(e[9]) == pytest.approx(math.cos(math.radians(0.25)))
    assert e[10:] == ["0.01", "0", "0", "0", "0", "0", "0.01", "0", "0", "0", "0", "0.01", "0", "0", "0",
                      "0.001", "0", "0", "0.001", "0", "0.001"]
    data = open(os.path.join(g, "000002", "data")).read()
    assert data.startswith(f"stamp {formats.ros_time(stamps[2])[0]} ") and data.endswith("accum_distance -1\nid 2\n")
    assert os.path.exists(os.path.join(g, "000002", "cloud.pcd"))


def test_save_balm(tmp_path):
    from floam_amd import formats
    P = _poses(2)
    clouds = [synth.to_xyzi(synth.generate_scan("tiny16x200", k)) for k in range(2)]
    d = str(tmp_path / "balm") + "/"
    formats.SavePosesHomogeneousBALM(clouds, P, [10.5, 10.6], d)
    rows = open(d + "alidarPose.csv").read().splitlines()
    assert len(rows) == 8 and rows[3] == "0.000000,0.000000,0.000000,10.500000,"
    assert os.path.exists(d + "full1.pcd")
