#!/usr/bin/env python3
"""fp64 vs fp32 geometry/Jacobian sweep (BASELINE.json configs[4]: "Dense 512k-pt scan vs 2M-pt local map, fp64 vs
fp32 Jacobian tolerance sweep").

One seeded sequence of a config (default C5: 128 x 4096-point rings, 2M-point prefilled map) through three paths:
  gpu64  the HIP path in the reference's precision (fp64 line/plane fits, residuals, Jacobians and LM, fp32 kNN);
  gpu32  floam_odom_set_precision(FP32): residuals, Jacobians and the per-thread J^T J / J^T r sums in float (line /
         plane fits, reductions across threads and the LM control step stay fp64);
  gpu32g FP32_GEOMETRY: the line (eigen) and plane (QR) fits in float as well;
  oracle the CPU restatement (oracle/, fp64 like the reference: src/odomEstimationClass.cpp:156-243,
         src/lidarOptimization.cpp:12-74).
Per scan: translation / rotation distance of each GPU pose to the oracle's, gpu32 to gpu64, and each path's error
against the synthetic ground truth.  Writes one JSON document (--out) and prints a table.  (Throughput per precision:
bench.py --config c5 --precision fp32.)

Run on the GPU box:  python tools/precision_sweep.py --config c5 --scans 8 --out gpurun_out/prec/c5.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MAP_RES, MIN_DIS, MAX_DIS, SCAN_PERIOD = 0.1, 0.5, 90.0, 0.1


def angle(qa, qb):
    return 2.0 * math.acos(min(1.0, abs(float(np.dot(qa, qb)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--scans", type=int, default=8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import floam_amd
    import oracle
    from floam_amd import _ffi, synth
    from floam_amd.odom_estimation import reset_process_state

    L = _ffi.load()
    cfg = args.config
    R = synth.lidar_model(cfg).rings
    params = floam_amd.LidarParams(num_lines=R, scan_period=SCAN_PERIOD, vertical_angle=2.0, max_distance=MAX_DIS,
                                   min_distance=MIN_DIS)
    fe = lambda raw, R_: oracle.feature_extraction(raw, R_, MIN_DIS, MAX_DIS, canonical=True)[:2]
    t0 = time.time()
    mapE, mapS = synth.prefill_map(cfg, fe, synth.MAP_PREFILL.get(cfg, 0))
    n_all = args.scans
    raws = [synth.generate_scan(cfg, k) for k in range(1, n_all + 1)]
    print(f"[sweep] {cfg}: map {mapE.shape[0]}+{mapS.shape[0]}, {n_all} scans of {raws[0].shape[0]} pts "
          f"generated in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    d_raw = [floam_amd.DeviceCloud(r) for r in raws]
    d_mapE, d_mapS = floam_amd.DeviceCloud(mapE), floam_amd.DeviceCloud(mapS)

    def pipeline(level):
        fp32, geom = level
        reset_process_state()
        lp = floam_amd.LaserProcessingClass()
        lp.init(params)
        odo = floam_amd.OdomEstimationClass()
        odo.init(params, MAP_RES, "Cauchy")
        odo.set_precision(fp32, geometry=geom)
        odo.initMapWithPoints(d_mapE, d_mapS)
        return lp, odo

    def gpu_poses(level):
        lp, odo = pipeline(level)
        out = []
        for k in range(args.scans):
            de, ds = floam_amd.DeviceCloud(), floam_amd.DeviceCloud()
            lp.featureExtraction(d_raw[k], de, ds)
            odo.UpdatePointsToMapSelector(de, ds, True)
            out.append(odo.pose())
        odo.close()
        lp.close()
        return out

    LEVELS = {"gpu64": (False, False), "gpu32": (True, False), "gpu32g": (True, True)}
    P = {name: gpu_poses(lv) for name, lv in LEVELS.items()}
    oracle.reset_process_statics()
    ref = oracle.Odometry(R, SCAN_PERIOD, MIN_DIS, MAX_DIS, MAP_RES, "Cauchy", stable_voxel=True)
    ref.init_map(mapE, mapS)
    rows = []
    for k in range(args.scans):
        e, s = fe(raws[k], R)
        ref.update_selector(e, s, True)
        qr, tr = ref.pose()
        gt = synth.gt_pose_matrix(k + 1)[:3, 3]
        row = {"scan": k + 1, "gt_err_m": {"oracle": float(np.linalg.norm(tr - gt))}}
        for name in LEVELS:
            q, t = P[name][k]
            row[name + "_vs_oracle"] = [float(np.linalg.norm(t - tr)), angle(q, qr)]
            row["gt_err_m"][name] = float(np.linalg.norm(t - gt))
        q64, t64 = P["gpu64"][k]
        for name in ("gpu32", "gpu32g"):
            q, t = P[name][k]
            row[name + "_vs_gpu64"] = [float(np.linalg.norm(t - t64)), angle(q, q64)]
        rows.append(row)
    keys = [k for k in rows[0] if k.endswith("_vs_oracle") or k.endswith("_vs_gpu64")]
    worst = {key: [max(r[key][0] for r in rows), max(r[key][1] for r in rows)] for key in keys}
    doc = {"config": cfg, "rings": R, "points_per_scan": int(raws[0].shape[0]),
           "map_prefill": int(mapE.shape[0] + mapS.shape[0]), "scans": rows, "max": worst,
           "tolerance": {"north_star_m": 1e-3, "north_star_rad": 1e-3}}
    print("scan " + " ".join(f"{n + '_vs_oracle (m, rad)':>30}" for n in LEVELS) + "  gt err (m): oracle / 64 / 32 / 32g")
    for r in rows:
        print(f"{r['scan']:>4} " + " ".join(f"{r[n + '_vs_oracle'][0]:15.3e} {r[n + '_vs_oracle'][1]:14.3e}"
                                           for n in LEVELS)
              + "  " + " / ".join(f"{r['gt_err_m'][n]:.5f}" for n in ("oracle",) + tuple(LEVELS)))
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
