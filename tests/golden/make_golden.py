#!/usr/bin/env python3
"""Generate the committed golden fixtures (run from the repo root: python tests/golden/make_golden.py).

The reference ships no fixtures and cannot be built here (SURVEY.md §8 c), so these vectors pin the CPU oracle
(oracle/) against regressions and give the GPU tests inputs that do not depend on the host's libm (the synthetic
generator's transcendental ufuncs may differ by an ulp across CPUs).  Inputs AND expected outputs are stored.

fe_tiny.npz   a 16x400 synthetic scan + the indices (into the input) of featureExtraction's edge / surf outputs
odom_c1.npz   4 consecutive VLP-16-style scans (scan 0 seeds the map) + per-scan poses, map sizes and per-solve
              correspondence counts / costs of OdomEstimationClass::UpdatePointsToMapSelector (deskew on)
imu_c1.npz    a 16x400 driver-style scan (times from the sweep start) + an IMU stream + extrinsics, and the node's
              CenterTime + Compensate + IMU alignment outputs (centred input, aligned cloud, centred stamp) as raw
              32-B records

Usage: python tests/golden/make_golden.py [fe] [odom] [imu]   (default: all)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from floam_amd import synth  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
PACK = ["x", "y", "z", "intensity", "ring", "time"]


def pack(pts):
    return {f: pts[f].copy() for f in PACK}


def make_fe():
    raw = synth.generate_scan("tiny16x400", 3)
    e, s, (bad, ties) = oracle.feature_extraction(raw, 16, 0.5, 90.0)
    assert bad == 0 and ties == 0
    key = {(float(p["x"]), float(p["y"]), float(p["z"]), float(p["time"])): i for i, p in enumerate(raw)}
    ei = np.array([key[(float(p["x"]), float(p["y"]), float(p["z"]), float(p["time"]))] for p in e], np.int32)
    si = np.array([key[(float(p["x"]), float(p["y"]), float(p["z"]), float(p["time"]))] for p in s], np.int32)
    np.savez_compressed(os.path.join(OUT, "fe_tiny.npz"), **{"in_" + k: v for k, v in pack(raw).items()},
                        edge_idx=ei, surf_idx=si, num_lines=16, min_dis=0.5, max_dis=90.0)
    print("fe_tiny:", raw.shape[0], "pts ->", len(ei), "edge,", len(si), "surf")


def make_odom():
    R, n = 16, 4
    scans = [synth.generate_scan("c1", k) for k in range(n)]
    oracle.reset_process_statics()
    odo = oracle.Odometry(R, 0.1, 0.5, 90.0, 0.1, "Cauchy", stable_voxel=True)
    poses, maps, solves = [], [], []
    for k, raw in enumerate(scans):
        e, s, _ = oracle.feature_extraction(raw, R, 0.5, 90.0, canonical=True)
        if k == 0:
            odo.init_map(synth.to_xyzi(e), synth.to_xyzi(s))
        else:
            odo.clear_traces()
            odo.update_selector(e, s, True)
            for t in odo.traces():
                solves.append([k, t["n_edge_queries"], t["n_surf_queries"], t["n_edge_corr"], t["n_surf_corr"],
                               t["iterations"], t["initial_cost"], t["final_cost"]])
        q, t = odo.pose()
        poses.append(np.r_[q, t])
        maps.append([odo.map(0).shape[0], odo.map(1).shape[0]])
    arrs = {}
    for k, raw in enumerate(scans):
        for f, v in pack(raw).items():
            arrs[f"scan{k}_{f}"] = v
    np.savez_compressed(os.path.join(OUT, "odom_c1.npz"), poses=np.array(poses), maps=np.array(maps),
                        solves=np.array(solves), nscans=n, num_lines=R, **arrs)
    print("odom_c1:", n, "scans, final pose", np.array(poses[-1]).round(5).tolist())


def make_imu():
    pts, stamp_us = synth.driver_scan("tiny16x400", 1)
    stamps, q = synth.imu_stream(-0.5, 0.6, rate=200.0)
    extr = oracle.euler_to_quaternion(0, 0, 180)
    ok, centred, aligned, stamp2 = oracle.imu_preprocess(pts, stamp_us, stamps, q, extr)
    assert ok
    np.savez_compressed(os.path.join(OUT, "imu_c1.npz"), input=pts.view(np.uint8), stamp_us=np.uint64(stamp_us),
                        imu_stamps=stamps, imu_q=q, extrinsics=extr, centred=centred.view(np.uint8),
                        aligned=aligned.view(np.uint8), stamp_out_us=np.uint64(stamp2))
    print("imu_c1:", pts.shape[0], "pts,", stamps.shape[0], "IMU messages, stamp", stamp_us, "->", stamp2)


if __name__ == "__main__":
    oracle.build()
    which = set(sys.argv[1:]) or {"fe", "odom", "imu"}
    if "fe" in which:
        make_fe()
    if "odom" in which:
        make_odom()
    if "imu" in which:
        make_imu()
