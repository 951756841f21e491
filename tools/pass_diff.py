#!/usr/bin/env python3
"""Index-level comparison of one correspondence pass where the GPU path and the oracle part ways (diagnostic, GPU box).

Usage: python tools/pass_diff.py [config] [scan] [solve]
Runs the oracle through scan-1 (its maps are the pass's map), runs the GPU odometry through `scan` (its deskewed clouds
and the starting pose of `solve` of that scan are the pass's queries and pose), then runs that one pass on both sides
on identical inputs (floam_odom_find_correspondences vs oracle.stage_correspondences) and reports the queries whose
neighbour sets differ, whether each is an exact float-distance tie, and whether any record differs without one.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import floam_amd  # noqa: E402
import oracle  # noqa: E402
from floam_amd import synth  # noqa: E402
from floam_amd.odom_estimation import reset_process_state  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
scan = int(sys.argv[2]) if len(sys.argv) > 2 else 42
solve = int(sys.argv[3]) if len(sys.argv) > 3 else 2
R = synth.lidar_model(cfg).rings
p = floam_amd.LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)
lp = floam_amd.LaserProcessingClass(device=0)
lp.init(p)


def gpu_fe(raw, _r):
    de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
    lp.featureExtraction(floam_amd.DeviceCloud(raw, device=0), de, ds)
    return de.download(), ds.download()


def float_sqd(map_points, q):
    dx = np.float32(q["x"]) - map_points["x"]
    dy = np.float32(q["y"]) - map_points["y"]
    dz = np.float32(q["z"]) - map_points["z"]
    return ((np.float32(0) + dx * dx) + dy * dy) + dz * dz


mapE, mapS = synth.prefill_map(cfg, gpu_fe, synth.MAP_PREFILL.get(cfg, 0))
feats = []
for k in range(1, scan + 1):
    e, s, _ = oracle.feature_extraction(synth.generate_scan(cfg, k), R, 0.5, 90.0, canonical=True)
    feats.append((e, s))
# the oracle through scan - 1: the pass's maps
oracle.reset_process_statics()
ref = oracle.Odometry(R, 0.1, 0.5, 90.0, 0.1, "Cauchy", stable_voxel=True)
ref.init_map(mapE, mapS)
for e, s in feats[:-1]:
    ref.update_selector(e.copy(), s.copy(), True)
maps = (ref.map(0), ref.map(1))
# the GPU through scan: the pass's queries (the clouds deskewed in place) and starting pose
reset_process_state()
odo = floam_amd.OdomEstimationClass(device=0)
odo.init(p, 0.1, "Cauchy")
odo.set_trace(4096)
odo.initMapWithPoints(floam_amd.DeviceCloud(mapE, device=0), floam_amd.DeviceCloud(mapS, device=0))
for k, (e, s) in enumerate(feats, start=1):
    de, ds = floam_amd.DeviceCloud(e, device=0), floam_amd.DeviceCloud(s, device=0)
    odo.UpdatePointsToMapSelector(de, ds, True)
    tr = odo.traces()
x = np.asarray(tr[solve]["x_in"], dtype=np.float64)
e_d, s_d = de.download(), ds.download()
odo.close()
# the one pass on both sides
reset_process_state()
one = floam_amd.OdomEstimationClass(device=0)
one.init(p, 0.1, "Cauchy")
one.set_trace(8)
one.initMapWithPoints(floam_amd.DeviceCloud(maps[0], device=0), floam_amd.DeviceCloud(maps[1], device=0))
one.find_correspondences(floam_amd.DeviceCloud(e_d, device=0), floam_amd.DeviceCloud(s_d, device=0), x[:4], x[4:])
print(f"{cfg} scan {scan} solve {solve}: maps {maps[0].shape[0]} + {maps[1].shape[0]}, x_in {x.tolist()}")
for which, leaf, src in ((0, 0.1, e_d), (1, 0.2, s_d)):
    mp = maps[which]
    gpu = one.correspondences(which)
    vox = oracle.voxel_grid(synth.to_xyzi(src), leaf, stable=True)
    same_q = all(np.array_equal(gpu["queries"][f], vox[f]) for f in ("x", "y", "z"))
    rp = oracle.stage_correspondences(mp, vox, x, edge=which == 0)
    world = oracle.associate_to_map(vox, x)
    gf, rf = gpu["flags"], rp["flags"]
    gated = np.nonzero((rf & 4) != 0)[0]
    gate_diff = int(np.sum((gf & 4) != (rf & 4)))
    sqd_diff = int(np.sum(np.any(gpu["sqd"][gated] != rp["sqd"][gated], axis=1)))
    gi, ri = gpu["idx"][gated], rp["idx"][gated]
    diff = np.nonzero(~np.all(np.sort(gi, axis=1) == np.sort(ri, axis=1), axis=1))[0]
    tied = 0
    for k in diff:
        d = np.sort(float_sqd(mp, world[gated[k]]))
        tied += int(len(set(d[:5].tolist())) < 5 or d[4] == d[5])
    acc = gated[(rf[gated] & 1) != 0]
    factor_diff = int(np.sum((gf[gated] & 1) != (rf[gated] & 1)))
    rec_diff = np.nonzero(np.any(gpu["records"][acc] != rp["records"][acc], axis=1))[0]
    print(f"  set {which}: queries identical {same_q}, {vox.shape[0]} queries, gated {gated.size}, gate differs "
          f"{gate_diff}, sqd differ {sqd_diff}, index sets differ {diff.size} (exact ties {tied}), factor decision "
          f"differs {factor_diff}, records differ {rec_diff.size}")
    for k in diff[:5]:
        q = gated[k]
        print(f"    query {q}: gpu idx {sorted(gi[k].tolist())} oracle idx {sorted(ri[k].tolist())} "
              f"sqd {gpu['sqd'][q].tolist()}")
