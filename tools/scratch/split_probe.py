# (diagnostic) a few C1 / C3 scans with whatever library and switches the environment selects; prints per-scan time
# and pose, so two runs can be compared
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import floam_amd
from floam_amd import synth
from floam_amd.odom_estimation import reset_process_state
cfg = sys.argv[1] if len(sys.argv) > 1 else "c1"
R = synth.lidar_model(cfg).rings
p = floam_amd.LidarParams(num_lines=R, scan_period=0.1, max_distance=90.0, min_distance=0.5)
lp = floam_amd.LaserProcessingClass(device=0); lp.init(p)
odo = floam_amd.OdomEstimationClass(device=0); odo.init(p, 0.1, "Cauchy")
reset_process_state()
for k in range(5):
    t0 = time.time()
    de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
    lp.featureExtraction(floam_amd.DeviceCloud(synth.generate_scan(cfg, k), device=0), de, ds)
    if k == 0:
        odo.initMapWithPoints(de, ds)
    else:
        odo.UpdatePointsToMapSelector(de, ds, True)
    q, t = odo.pose()
    print("scan", k, "%.3f s" % (time.time() - t0), np.array2string(np.r_[q, t], precision=12), flush=True)
