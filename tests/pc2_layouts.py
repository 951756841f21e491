"""PointCloud2 test messages in the layouts drivers publish (test helper, no GPU).

Each builder returns (data bytes, width, height, point_step, row_step, fields) with fields as
(name, offset, datatype, count) tuples, datatype codes as sensor_msgs/PointField (UINT16 = 4, FLOAT32 = 7)."""
import numpy as np

F32, U16, U8, U32 = 7, 4, 2, 6


def _pack(pts, layout, point_step, width, height, row_pad=0, seed=0):
    """layout: list of (name, offset, numpy type, datatype code, source field or None for filler)."""
    rng = np.random.default_rng(seed)
    n = pts.shape[0]
    assert n == width * height
    row_step = width * point_step + row_pad
    buf = np.frombuffer(rng.bytes(row_step * height), np.uint8).copy()   # garbage padding everywhere
    for r in range(height):
        for name, off, nptype, _, src in layout:
            vals = np.ascontiguousarray(pts[src][r * width:(r + 1) * width] if src else
                              rng.integers(0, 200, width), dtype=nptype)
            view = buf[r * row_step: r * row_step + width * point_step].reshape(width, point_step)
            view[:, off:off + vals.dtype.itemsize] = vals.view(np.uint8).reshape(width, vals.dtype.itemsize)
    fields = [(name, off, dt, 1) for name, off, _, dt, _ in layout]
    return buf.tobytes(), width, height, point_step, row_step, fields


def velodyne(pts):
    """velodyne_pointcloud PointXYZIRT as published: the PCL struct itself (point_step 32)."""
    lay = [("x", 0, np.float32, F32, "x"), ("y", 4, np.float32, F32, "y"), ("z", 8, np.float32, F32, "z"),
           ("intensity", 16, np.float32, F32, "intensity"), ("ring", 20, np.uint16, U16, "ring"),
           ("time", 24, np.float32, F32, "time")]
    return _pack(pts, lay, 32, pts.shape[0], 1)


def ouster_like(pts):
    """An Ouster-style layout: extra fields, different offsets, 48-B points, time as float at 20, ring at 34, and
    an organised 2-row cloud with row padding."""
    lay = [("x", 0, np.float32, F32, "x"), ("y", 4, np.float32, F32, "y"), ("z", 8, np.float32, F32, "z"),
           ("intensity", 16, np.float32, F32, "intensity"), ("time", 20, np.float32, F32, "time"),
           ("reflectivity", 24, np.uint16, U16, None), ("ring", 34, np.uint16, U16, "ring"),
           ("range", 36, np.uint32, U32, None)]
    n = pts.shape[0] - pts.shape[0] % 2
    return _pack(pts[:n], lay, 48, n // 2, 2, row_pad=24, seed=1)


def packed_reordered(pts):
    """Fields in another order, packed with no padding (point_step 22), ring declared with the wrong datatype (so
    PCL leaves it zero and warns)."""
    lay = [("time", 0, np.float32, F32, "time"), ("ring", 4, np.uint8, U8, "ring"),
           ("z", 5, np.float32, F32, "z"), ("x", 9, np.float32, F32, "x"), ("y", 13, np.float32, F32, "y"),
           ("intensity", 17, np.float32, F32, "intensity")]
    return _pack(pts, lay, 22, pts.shape[0], 1, seed=2)


def reference_decode(data, width, height, point_step, row_step, fields, point_type=0):
    """Independent numpy statement of fromPCLPointCloud2 for non-coalescing layouts: each matched field copied
    from its message offset into its struct offset, everything else zero."""
    from floam_amd.synth import POINT_DTYPE
    reg = [("x", 0, F32), ("y", 4, F32), ("z", 8, F32), ("intensity", 16, F32), ("ring", 20, U16), ("time", 24, F32)]
    reg = reg if point_type == 0 else reg[:4]
    raw = np.frombuffer(data, np.uint8)
    out = np.zeros(width * height * 32, np.uint8).reshape(-1, 32)
    for name, soff, dt in reg:
        m = [f for f in fields if f[0] == name and f[2] == dt and f[3] in (0, 1)]
        if not m:
            continue
        moff, size = m[0][1], 2 if dt == U16 else 4
        for r in range(height):
            rows = raw[r * row_step: r * row_step + width * point_step].reshape(width, point_step)
            out[r * width:(r + 1) * width, soff:soff + size] = rows[:, moff:moff + size]
    return out.reshape(-1).view(POINT_DTYPE)
