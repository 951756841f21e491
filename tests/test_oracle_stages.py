"""The oracle's stage hooks (stage_correspondences, stage_solve, associate_to_map) against the oracle's own
updatePointsToMap: one pass + one solve restated stage by stage reproduces the full update's first solve bit for
bit, so the GPU stage tests (tests/test_gpu_stages.py) compare against exactly what the sequence tests use."""
import numpy as np

from floam_amd import synth


def test_stage_hooks_reproduce_update(oracle_lib):
    R = 16
    fe = lambda raw: oracle_lib.feature_extraction(raw, R, 0.5, 90.0, canonical=True)[:2]
    e0, s0 = fe(synth.generate_scan("c1", 0))
    e1, s1 = fe(synth.generate_scan("c1", 1))
    mapE, mapS = synth.to_xyzi(e0), synth.to_xyzi(s0)
    ref = oracle_lib.Odometry(R, 0.1, 0.5, 90.0, 0.1, "Cauchy", stable_voxel=True)
    ref.init_map(mapE, mapS)
    ref.update(e1, s1, oracle_lib.Odometry.INITIAL_ITERATION)
    tr = ref.traces()[0]
    x_in = tr["x_in"]
    dE = oracle_lib.voxel_grid(synth.to_xyzi(e1), 0.1, stable=True)
    dS = oracle_lib.voxel_grid(synth.to_xyzi(s1), 0.2, stable=True)
    pe = oracle_lib.stage_correspondences(mapE, dE, x_in, edge=True)
    ps = oracle_lib.stage_correspondences(mapS, dS, x_in, edge=False)
    erec = pe["records"][(pe["flags"] & 1) != 0]
    srec = ps["records"][(ps["flags"] & 1) != 0]
    assert erec.shape[0] == tr["n_edge_corr"] and srec.shape[0] == tr["n_surf_corr"]
    x_out, st = oracle_lib.stage_solve(erec, srec, x_in)
    np.testing.assert_array_equal(x_out, tr["x_out"])
    for f in ("iterations", "successful", "initial_cost", "final_cost"):
        assert st[f] == tr[f], f
    np.testing.assert_array_equal(st["H0"], tr["H0"])
    np.testing.assert_array_equal(st["g0"], tr["g0"])
    # the gate: flags bit 2 iff the 5th float squared distance < 1, and the neighbours are the KD-tree's
    assert np.all(((pe["flags"] & 4) != 0) == (pe["sqd"][:, 4] < 1.0))
    idx, sqd = oracle_lib.knn(mapE, np.stack([oracle_lib.associate_to_map(dE, x_in)[f] for f in "xyz"], 1))
    np.testing.assert_array_equal(idx, pe["idx"])
    np.testing.assert_array_equal(sqd, pe["sqd"])
