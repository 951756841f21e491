#!/usr/bin/env python3
"""First LM solve at which the GPU path and the oracle part ways on a bench sequence (diagnostic, GPU box).

Usage: python tools/trace_diff.py [config] [scans]
Runs UpdatePointsToMapSelector(deskew) synchronously on the GPU and in the oracle over the bench's sequence and map
prefill (synth.prefill_map), with per-solve traces on both (floam_odom_set_trace / the oracle's traces), and prints
the first solve whose iteration counts, correspondence counts or costs differ, with the scans' pose agreement.
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import floam_amd  # noqa: E402
import oracle  # noqa: E402
from floam_amd import synth  # noqa: E402
from floam_amd.odom_estimation import reset_process_state  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 45
R = synth.lidar_model(cfg).rings
p = floam_amd.LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)
lp = floam_amd.LaserProcessingClass(device=0)
lp.init(p)


def gpu_fe(raw, _r):
    de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
    lp.featureExtraction(floam_amd.DeviceCloud(raw, device=0), de, ds)
    return de.download(), ds.download()


mapE, mapS = synth.prefill_map(cfg, gpu_fe, synth.MAP_PREFILL.get(cfg, 0))
reset_process_state()
oracle.reset_process_statics()
odo = floam_amd.OdomEstimationClass(device=0)
odo.init(p, 0.1, "Cauchy")
odo.set_trace(4096)
odo.initMapWithPoints(floam_amd.DeviceCloud(mapE, device=0), floam_amd.DeviceCloud(mapS, device=0))
ref = oracle.Odometry(R, 0.1, 0.5, 90.0, 0.1, "Cauchy", stable_voxel=True)
ref.init_map(mapE, mapS)
fields = ("n_edge_queries", "n_surf_queries", "n_edge_corr", "n_surf_corr", "iterations", "successful")
reported = False
for k in range(1, n + 1):
    raw = synth.generate_scan(cfg, k)
    e, s, _ = oracle.feature_extraction(raw, R, 0.5, 90.0, canonical=True)
    odo.UpdatePointsToMapSelector(floam_amd.DeviceCloud(e, device=0), floam_amd.DeviceCloud(s, device=0), True)
    ref.update_selector(e, s, True)
    (qg, tg), (qr, tr) = odo.pose(), ref.pose()
    dt = float(np.linalg.norm(tg - tr))
    dr = 2.0 * math.acos(min(1.0, abs(float(np.dot(qg, qr)))))
    g_tr, r_tr = odo.traces(), ref.traces()   # this scan's solves (both cleared after reading)
    ref.clear_traces()
    for j in range(min(len(g_tr), len(r_tr))):
        g, r = g_tr[j], r_tr[j]
        bad = [f for f in fields if g[f] != r[f]]
        xin = float(np.max(np.abs(np.asarray(g["x_in"]) - np.asarray(r["x_in"]))))
        xout = float(np.max(np.abs(np.asarray(g["x_out"]) - np.asarray(r["x_out"]))))
        if (bad or xout > 1e-9) and not reported:
            reported = True
            print(f"scan {k} solve {j} (of the scan): differing {bad}, |x_in| {xin:.2e}, |x_out| {xout:.2e}")
            for f in fields + ("initial_cost", "final_cost"):
                print(f"   {f:16s} gpu {g[f]!r:>24}  oracle {r[f]!r:>24}")
            ic = r["initial_cost"]
            print(f"   final/initial cost change gpu {abs(g['final_cost'] - ic) / ic:.3e}, "
                  f"oracle {abs(r['final_cost'] - ic) / ic:.3e} (function tolerance 1e-6)")
    print(f"scan {k}: pose {dt:.3e} m {dr:.3e} rad, solves {len(g_tr)} / {len(r_tr)}", flush=True)
