"""The oracle's third-party restatements against independent numpy / scipy computations:
PCL VoxelGrid + CropBox (numpy restatement of the PCL 1.8.1 semantics), FLANN exact 5-NN (scipy cKDTree), Eigen
SelfAdjointEigenSolver (numpy.linalg.eigh), ColPivHouseholderQR least squares (numpy.linalg.lstsq), and the analytic
cost-function Jacobians (central differences through the SE3 Plus)."""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from floam_amd.synth import POINT_DTYPE


def _cloud(rng, n, scale=10.0):
    p = np.zeros(n, POINT_DTYPE)
    xyz = (rng.standard_normal((n, 3)) * scale).astype(np.float32)
    p["x"], p["y"], p["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    p["intensity"] = rng.uniform(0, 255, n).astype(np.float32)
    p["pad0"] = 1.0
    return p


def numpy_voxel_grid(p, leaf):
    """PCL 1.8.1 VoxelGrid::applyFilter restated with numpy (stable within-voxel order)."""
    leaf = np.float32(leaf)
    inv = np.float32(1.0) / leaf
    x, y, z = p["x"], p["y"], p["z"]
    mn = np.array([x.min(), y.min(), z.min()], np.float32)
    mx = np.array([x.max(), y.max(), z.max()], np.float32)
    d = [int(np.float32(mx[k] - mn[k]) * inv) + 1 for k in range(3)]
    if d[0] * d[1] * d[2] > 2**31 - 1:
        return p.copy()
    min_b = [int(np.floor(np.float32(mn[k] * inv))) for k in range(3)]
    max_b = [int(np.floor(np.float32(mx[k] * inv))) for k in range(3)]
    div = [max_b[k] - min_b[k] + 1 for k in range(3)]
    ijk = [(np.floor((c * inv).astype(np.float32)) - np.float32(min_b[k])).astype(np.int64)
           for k, c in enumerate((x, y, z))]
    idx = ijk[0] + ijk[1] * div[0] + ijk[2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    sidx = idx[order]
    heads = np.flatnonzero(np.r_[True, sidx[1:] != sidx[:-1]])
    ends = np.r_[heads[1:], len(sidx)]
    out = np.zeros(len(heads), POINT_DTYPE)
    out["pad0"] = 1.0
    for o, (h, e) in enumerate(zip(heads, ends)):
        sel = order[h:e]
        for f in ("x", "y", "z", "intensity"):
            acc = np.float32(0)
            acc = p[f][sel[0]]
            for t in sel[1:]:
                acc = np.float32(acc + p[f][t])
            out[f][o] = np.float32(acc / np.float32(e - h))
    return out


@pytest.mark.parametrize("leaf,n,scale", [(0.1, 3000, 2.0), (0.2, 5000, 5.0), (0.4, 800, 1.0)])
def test_voxel_grid_matches_numpy(oracle_lib, leaf, n, scale):
    rng = np.random.default_rng(int(leaf * 1000) + n)
    p = _cloud(rng, n, scale)
    got = oracle_lib.voxel_grid(p, leaf, stable=True)
    ref = numpy_voxel_grid(p, leaf)
    assert got.shape == ref.shape
    for f in ("x", "y", "z", "intensity"):
        np.testing.assert_array_equal(got[f], ref[f], err_msg=f)


def test_voxel_grid_unstable_differs_only_in_summation_order(oracle_lib):
    rng = np.random.default_rng(3)
    p = _cloud(rng, 20000, 1.0)
    a = oracle_lib.voxel_grid(p, 0.2, stable=True)
    b = oracle_lib.voxel_grid(p, 0.2, stable=False)   # std::sort like PCL
    assert a.shape == b.shape
    for f in ("x", "y", "z"):
        np.testing.assert_allclose(a[f], b[f], rtol=0, atol=2e-6)


def test_voxel_grid_overflow_returns_input_q9(oracle_lib):
    rng = np.random.default_rng(5)
    p = _cloud(rng, 500, 1000.0)   # extent ~ 8 km at 1 mm leaf -> > 2^31 voxels
    out = oracle_lib.voxel_grid(p, 0.001, stable=True)
    assert out.shape == p.shape
    np.testing.assert_array_equal(out["x"], p["x"])


def test_crop_box_inclusive_order_preserving(oracle_lib):
    rng = np.random.default_rng(7)
    p = _cloud(rng, 4000, 5.0)
    p["x"][0] = 3.0   # exactly on the boundary: kept (inclusive)
    mn, mx = (-3.0, -4.0, -5.0), (3.0, 4.0, 5.0)
    out = oracle_lib.crop_box(p, mn, mx)
    keep = ((p["x"] >= -3) & (p["x"] <= 3) & (p["y"] >= -4) & (p["y"] <= 4) & (p["z"] >= -5) & (p["z"] <= 5))
    np.testing.assert_array_equal(out["x"], p["x"][keep])
    assert out["x"][0] == 3.0


def test_knn_matches_cKDTree(oracle_lib):
    rng = np.random.default_rng(11)
    m = _cloud(rng, 6000, 3.0)
    q = (rng.standard_normal((500, 3)) * 3.0).astype(np.float32)
    idx, sqd = oracle_lib.knn(m, q, 5)
    xyz = np.stack([m["x"], m["y"], m["z"]], 1).astype(np.float64)
    d_ref, i_ref = cKDTree(xyz).query(q.astype(np.float64), k=5)
    np.testing.assert_array_equal(np.sort(idx, 1), np.sort(i_ref, 1))
    # FLANN L2_Simple in float: ((0 + dx^2) + dy^2) + dz^2
    diff = (q[:, None, :] - xyz[idx].astype(np.float32)).astype(np.float32)
    f = np.zeros(idx.shape, np.float32)
    for k in range(3):
        f = (f + diff[..., k] * diff[..., k]).astype(np.float32)
    np.testing.assert_array_equal(sqd, f)
    assert np.all(np.diff(sqd, axis=1) >= 0)


def test_eig_sym3_matches_eigh(oracle_lib):
    rng = np.random.default_rng(13)
    for _ in range(200):
        P = rng.standard_normal((5, 3)) * rng.uniform(0.01, 1.0, 3)
        c = P.mean(0)
        A = (P - c).T @ (P - c)
        ev, V = oracle_lib.eig_sym3(A)
        w, U = np.linalg.eigh(A)
        np.testing.assert_allclose(ev, w, rtol=1e-10, atol=1e-14)
        assert abs(abs(float(V[:, 2] @ U[:, 2])) - 1.0) < 1e-9
        np.testing.assert_allclose(A @ V, V * ev, atol=1e-10 * max(1.0, abs(w).max()))


def test_plane_lstsq_matches_numpy(oracle_lib):
    rng = np.random.default_rng(17)
    for _ in range(200):
        c = rng.uniform(-50, 50, 3)
        n = rng.standard_normal(3)
        n /= np.linalg.norm(n)
        B = np.linalg.svd(np.eye(3) - np.outer(n, n))[0][:, :2]
        P = c + (rng.uniform(-0.5, 0.5, (5, 2)) @ B.T) + rng.normal(0, 0.01, (5, 1)) * n
        x = oracle_lib.plane_solve(P)
        ref = np.linalg.lstsq(P, -np.ones(5), rcond=None)[0]
        np.testing.assert_allclose(x, ref, rtol=1e-7, atol=1e-12)


def _numeric_jacobian(f, x, h=1e-6):
    import oracle
    J = np.zeros(6)
    for k in range(6):
        d = np.zeros(6)
        d[k] = h
        rp = f(oracle.se3_plus(x, d))
        rm = f(oracle.se3_plus(x, -d))
        J[k] = (rp - rm) / (2 * h)
    return J


def test_analytic_jacobians_match_central_differences(oracle_lib):
    rng = np.random.default_rng(19)
    for _ in range(50):
        q = rng.standard_normal(4)
        q /= np.linalg.norm(q)
        x = np.r_[q, rng.uniform(-5, 5, 3)]
        cp = rng.uniform(-20, 20, 3)
        a = rng.uniform(-20, 20, 3)
        b = a + rng.standard_normal(3) * 0.2
        r, J = oracle_lib.edge_residual(cp, a, b, x)
        Jn = _numeric_jacobian(lambda xx: oracle_lib.edge_residual(cp, a, b, xx)[0], x)
        np.testing.assert_allclose(J, Jn, rtol=1e-5, atol=1e-6)
        n = rng.standard_normal(3)
        n /= np.linalg.norm(n)
        d = rng.uniform(-3, 3)
        r, J = oracle_lib.surf_residual(cp, n, d, x)
        Jn = _numeric_jacobian(lambda xx: oracle_lib.surf_residual(cp, n, d, xx)[0], x)
        np.testing.assert_allclose(J, Jn, rtol=1e-5, atol=1e-6)


def test_se3_plus_small_angle_series_and_composition(oracle_lib):
    x = np.array([0.0, 0.0, np.sin(0.2), np.cos(0.2), 1.0, 2.0, 3.0])
    y = oracle_lib.se3_plus(x, np.zeros(6))
    np.testing.assert_allclose(y, x, atol=1e-15)
    y = oracle_lib.se3_plus(x, [1e-12, 0, 0, 0, 0, 0])   # theta < 1e-10: series branch
    assert abs(np.linalg.norm(y[:4]) - 1.0) < 1e-12
    # pure translation step moves t by upsilon
    y = oracle_lib.se3_plus(x, [0, 0, 0, 0.1, -0.2, 0.3])
    np.testing.assert_allclose(y[4:], x[4:] + [0.1, -0.2, 0.3], atol=1e-15)
