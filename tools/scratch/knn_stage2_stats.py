"""GPU: the share of kNN queries that need stage 2, edge vs surf, and how they fall into waves of 4 query groups, on
the C3 bench sequence after a few scans (stage inspection: floam_odom_find_correspondences at the current pose).
Usage: python tools/scratch/knn_stage2_stats.py [config] [scans]"""
import sys
import numpy as np
sys.path.insert(0, ".")
import floam_amd
from floam_amd import synth
from floam_amd.odom_estimation import reset_process_state

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
R = synth.lidar_model(cfg).rings
params = floam_amd.LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0, min_distance=0.5)
lp = floam_amd.LaserProcessingClass()
lp.init(params)


def fe(raw, R_):
    de, ds = floam_amd.DeviceCloud(), floam_amd.DeviceCloud()
    lp.featureExtraction(floam_amd.DeviceCloud(raw), de, ds)
    return de.download(), ds.download()


mapE, mapS = synth.prefill_map(cfg, fe, synth.MAP_PREFILL.get(cfg, 0))
reset_process_state()
odo = floam_amd.OdomEstimationClass()
odo.init(params, 0.1, "Cauchy")
odo.set_trace(64)
odo.initMapWithPoints(floam_amd.DeviceCloud(mapE), floam_amd.DeviceCloud(mapS))
for k in range(1, n + 1):
    e, s = fe(synth.generate_scan(cfg, k), R)
    de, ds = floam_amd.DeviceCloud(e), floam_amd.DeviceCloud(s)
    odo.UpdatePointsToMapSelector(de, ds, True)
q, t = odo.pose()
odo.find_correspondences(floam_amd.DeviceCloud(e), floam_amd.DeviceCloud(s), q, t)
for which, name in ((0, "edge"), (1, "surf")):
    g = odo.correspondences(which)
    fl = g["flags"]
    st2 = (fl & 2) != 0
    w = st2[: len(st2) // 4 * 4].reshape(-1, 4).sum(1)   # queries 4i..4i+3 share a wave (16-lane groups)
    print(f"{name}: {len(fl)} queries, stage 2 {st2.mean():.3f}; waves with 0/1/2/3/4 stage-2 queries: "
          f"{[int((w == c).sum()) for c in range(5)]}")
odo.close()
lp.close()
