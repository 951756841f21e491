"""Per-solve LM traces of the GPU path on the golden C1 sequence (tests/golden/odom_c1.npz) next to the fixture's
oracle solves: where a library first departs from the oracle (diagnostic for a failing test_golden_odometry_gpu).
Usage: python tools/golden_trace.py OUT.json"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import floam_amd as fa  # noqa: E402
from test_golden import _load_odom  # noqa: E402


def main():
    from floam_amd.odom_estimation import reset_process_state
    scans, poses, maps, solves, R = _load_odom()
    p = fa.LidarParams(num_lines=R, scan_period=0.1, max_distance=90.0, min_distance=0.5)
    lp = fa.LaserProcessingClass()
    lp.init(p)
    odo = fa.OdomEstimationClass()
    odo.init(p, 0.1, "Cauchy")
    odo.set_trace(64)
    reset_process_state()
    rows = []
    for k, raw in enumerate(scans):
        de, ds = fa.DeviceCloud(), fa.DeviceCloud()
        lp.featureExtraction(fa.DeviceCloud(raw), de, ds)
        if k == 0:
            odo.initMapWithPoints(de, ds)
            odo.traces()
            continue
        odo.UpdatePointsToMapSelector(de, ds, True)
        q, t = odo.pose()
        for j, tr in enumerate(odo.traces()):
            rows.append({"scan": k, "solve": j, "ne": int(tr["n_edge_corr"]), "ns": int(tr["n_surf_corr"]),
                         "it": int(tr["iterations"]), "c0": float(tr["initial_cost"]), "c1": float(tr["final_cost"]),
                         "x_out": [float(v) for v in tr["x_out"]]})
        rows.append({"scan": k, "pose_err_m": float(np.linalg.norm(t - poses[k][4:]))})
    ref = [[float(v) for v in s] for s in solves]
    json.dump({"gpu": rows, "oracle_solves": ref}, open(sys.argv[1], "w"), indent=1)
    for r in rows[:40]:
        print(r if "pose_err_m" in r else {kk: r[kk] for kk in ("scan", "solve", "ne", "ns", "it", "c0", "c1")})
    for s in ref[:24]:
        print("oracle", s)


if __name__ == "__main__":
    main()
