#!/usr/bin/env python3
"""Benchmark: scans/sec of the FLOAM scan-to-map odometry hot path on MI355X.

One step = one scan through the reference's two operators, exactly as the nodes drive them:
LaserProcessingClass::featureExtraction (src/laserProcessingNode.cpp:129) followed by
OdomEstimationClass::UpdatePointsToMapSelector(edge, surf, deskew=true) (src/odomEstimationNode.cpp:228), with the
launch-file defaults (launch/structor_odom.launch: map_resolution 0.1, deskew on, loss "Cauchy" -> no robust
loss, min/max_dis 0.5/90).  The raw scans are resident in HBM before the timed region; the host reads the pose
back after every update call like the node does.

Workload (BASELINE.json configs[2], the headline): 64-ring HDL-64-style synthetic scans (~130k points), local map
prefilled with 200k edge+surf points through initMapWithPoints, steady state (the warm-up covers the
optimization_count 12 -> 2 ramp).

--gpus N > 1 (launched by torch.distributed.run), default --mode replica: every rank runs its own odometry
pipeline (one per sensor, no collective on the data path) over a copy of the same synthetic sequence; value = scans
of all ranks per second (weak scaling).  --mode shard is the north star's partition of ONE sequence (SURVEY.md §8 e): every rank runs the same
sequence, shards the correspondence queries and sums the normal equations with one RCCL all-reduce per LM
evaluation; value = scans of the one sequence per second (strong scaling).  At C3 a scan is ~0.7 ms of
latency-bound launches, so the ~20 all-reduces per scan cost more than the sharded work saves.

Prints ONE JSON line on rank 0 (contract in the task statement), with "roofline" for the dominant kernel
(the surf correspondence kernel, HIP events on the library stream over the timed region) and "cpu_baseline"
(the CPU oracle — the reference path restated, single-threaded — timed on this host on a bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "scans/sec scan-to-map odometry, 64-ring ~130k pts; pose RMSE vs reference"
MAP_RES, LOSS, MIN_DIS, MAX_DIS, SCAN_PERIOD = 0.1, "Cauchy", 0.5, 90.0, 0.1
# updates in flight (floam_odom_set_async) and feature buffers: the host issues scan k+DEPTH-1 while scan k runs
DEPTH = int(os.environ.get("FLOAM_BENCH_DEPTH", "2"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def hbm_traffic(kernel_substr):
    """HBM bytes per launch of the dominant kernel from the newest committed rocprofv3 PMC summary
    (profiles/<tag>/hbm_traffic.json, written by tools/prof_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE
    runs of this bench).  (None, None) when no profile is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "hbm_traffic.json")))
    for f in reversed(files):
        d = json.load(open(f))
        for name, v in d.get("kernels", {}).items():
            if kernel_substr in name:
                return round(v["total_bytes"]), os.path.relpath(f, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--mode", choices=["shard", "replica"], default="replica")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist   # control plane only (barrier, id broadcast, max-time); data: RCCL
        dist.init_process_group(backend="gloo")

    import floam_amd
    import oracle
    from floam_amd import _ffi, synth
    from floam_amd.odom_estimation import comm_unique_id, reset_process_state

    L = _ffi.load()
    dev = int(os.environ.get("FLOAM_BENCH_DEVICE", local_rank))   # override: several ranks on one GPU (testing)
    cfg = args.config
    model = synth.lidar_model(cfg)
    R = model.rings
    target = synth.MAP_PREFILL.get(cfg, 0)

    def oracle_fe(raw, R_):   # the CPU baseline leg only
        e, s, _ = oracle.feature_extraction(raw, R_, MIN_DIS, MAX_DIS, canonical=True)
        return e, s

    params = floam_amd.LidarParams(num_lines=R, scan_period=SCAN_PERIOD, vertical_angle=2.0, max_distance=MAX_DIS,
                                   min_distance=MIN_DIS)
    fe_lp = floam_amd.LaserProcessingClass(device=dev)
    fe_lp.init(params)

    def gpu_fe(raw, R_):   # featureExtraction on the GPU (untimed: the prefill's earlier scans)
        de, ds = floam_amd.DeviceCloud(device=dev), floam_amd.DeviceCloud(device=dev)
        fe_lp.featureExtraction(floam_amd.DeviceCloud(raw, device=dev), de, ds)
        return de.download(), ds.download()

    t0 = time.time()
    n_scans = args.warmup + args.steps
    # replica ranks run independent pipelines over the same synthetic sequence (same work per rank as at N = 1;
    # a sequence that starts elsewhere on the trajectory would not match the map prefilled around the origin)
    scan_offset = 0
    raws = [synth.generate_scan(cfg, scan_offset + k) for k in range(1, n_scans + 1)]
    mapE, mapS = synth.prefill_map(cfg, gpu_fe, target)
    fe_lp.close()
    log(f"[rank {rank}] generated {n_scans} scans ({raws[0].shape[0]} pts) + map {mapE.shape[0]}+{mapS.shape[0]} "
        f"in {time.time() - t0:.1f}s")

    d_raw = [floam_amd.DeviceCloud(r, device=dev) for r in raws]       # inputs resident in HBM
    d_mapE, d_mapS = floam_amd.DeviceCloud(mapE, device=dev), floam_amd.DeviceCloud(mapS, device=dev)
    allreduce_impl = None
    uid = None
    if world > 1 and args.mode == "shard":
        uid = [(comm_unique_id(), comm_unique_id()) if rank == 0 else None]   # timed run, byte-count replay
        dist.broadcast_object_list(uid, src=0)
    n_pipelines = 0

    def make_pipeline():
        nonlocal allreduce_impl, n_pipelines
        reset_process_state()
        lp = floam_amd.LaserProcessingClass(device=dev, asynchronous=True)   # one sync per scan (the pose read)
        lp.init(params)
        odo = floam_amd.OdomEstimationClass(device=dev)
        odo.init(params, MAP_RES, LOSS)
        if uid is not None:
            try:
                odo.set_shard(rank, world, uid[0][n_pipelines])   # RCCL over xGMI
                allreduce_impl = "rccl"
            except floam_amd.FloamError as e:   # e.g. several ranks on one GPU: host all-reduce over gloo
                log(f"[rank {rank}] RCCL unavailable ({e}); using the gloo host all-reduce")
                import torch

                def _allreduce(arr):
                    t = torch.from_numpy(arr)
                    dist.all_reduce(t, op=dist.ReduceOp.SUM)
                odo.set_shard_callback(rank, world, _allreduce)
                allreduce_impl = "gloo-host"
        odo.initMapWithPoints(d_mapE, d_mapS)
        odo.set_async(DEPTH)
        n_pipelines += 1
        return lp, odo

    lp, odo = make_pipeline()
    # two feature buffers: the extraction of scan k+1 (its own stream) is issued before the odometry of scan k, so
    # the two overlap on the device, as the reference's laserProcessingNode runs beside odomEstimationNode
    bufs = [(floam_amd.DeviceCloud(device=dev), floam_amd.DeviceCloud(device=dev)) for _ in range(max(2, DEPTH))]

    def extract(lp, k):
        e, s = bufs[k % len(bufs)]
        e.clear()
        s.clear()
        lp.featureExtraction(d_raw[k], e, s)

    host_split = [0.0, 0.0]   # host seconds issuing / waiting (diagnostic, FLOAM_BENCH_HOST=1)

    def run(lp, odo, a, b, poses):
        """scans [a, b): featureExtraction + UpdatePointsToMapSelector each, extraction one scan ahead; the odometry
        streams (floam_odom_set_async): scan k's pose is collected after scan k+1 has been issued"""
        if a < b:
            extract(lp, a)
        for k in range(a, b):
            t0 = time.perf_counter()
            if k + 1 < b:
                extract(lp, k + 1)
            e, s = bufs[k % len(bufs)]
            odo.UpdatePointsToMapSelector(e, s, True)
            t1 = time.perf_counter()
            poses.extend(odo.wait(DEPTH - 1))
            host_split[0] += t1 - t0
            host_split[1] += time.perf_counter() - t1
        poses.extend(odo.wait(0))

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        _ffi.check(L.floam_device_synchronize(dev))

    poses = []
    run(lp, odo, 0, args.warmup, poses)
    barrier_sync()
    host_split[:] = [0.0, 0.0]
    t_start = time.perf_counter()
    run(lp, odo, args.warmup, n_scans, poses)
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    if os.environ.get("FLOAM_BENCH_HOST"):
        log(f"[host] per timed scan: issue {1e6 * host_split[0] / args.steps:.0f} us, "
            f"wait {1e6 * host_split[1] / args.steps:.0f} us")
    _ffi.check(L.floam_profile_enable(dev, 0))
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stats = odo.stats()

    def read_timings():
        arr = (_ffi.KernelTiming * 16)()
        n = C.c_int()
        _ffi.check(L.floam_profile_read(dev, arr, 16, C.byref(n)))
        return {arr[i].name.decode(): (arr[i].launches, arr[i].total_ms, arr[i].algorithmic_bytes)
                for i in range(min(n.value, 16))}

    roof = None
    if not args.no_roofline:
        odo.close()
        lp.close()
        # The dominant kernel — the exact 5-NN search (knn_kernel, edge + surf queries in one launch) — measured on an
        # identical replay of the same sequence (the pipeline is deterministic; the poses are checked bit for bit):
        # HIP events on the library stream around every search launch (FLOAM_PROF_KNN_DETAIL) and the byte-counting
        # kernel after each pass (FLOAM_PROF_KNN_BYTES, SURVEY.md §8 d).  Profiling issues the updates launch by
        # launch: the timed run above replays each update as one hipGraph, and timing events recorded inside a graph
        # cannot be read back on this ROCm (hipEventElapsedTime fails for them).
        lp, odo = make_pipeline()
        replay = []
        run(lp, odo, 0, args.warmup, replay)
        _ffi.check(L.floam_profile_reset(dev))
        _ffi.check(L.floam_profile_enable(dev, 1 | 16 | 32))
        run(lp, odo, args.warmup, n_scans, replay)
        _ffi.check(L.floam_profile_enable(dev, 0))
        timed = read_timings()
        same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(poses, replay))
        kt = timed.get("knn_search")
        if kt is not None and kt[0] > 0:
            avg_ms = kt[1] / kt[0]
            bytes_per = kt[2] / kt[0]
            ach = bytes_per / (avg_ms * 1e-3) / 1e9
            traffic, traffic_src = hbm_traffic("knn_kernel<")
            roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": "knn_kernel (exact 5-NN search over the hash grid, edge + surf queries)",
                    "avg_us": round(avg_ms * 1e3, 2), "launches": int(kt[0]),
                    "algorithmic_bytes_per_launch": round(bytes_per), "replay_bitwise_identical": bool(same)}
            for sub in ("knn", "knn_geometry"):
                ks = timed.get(sub)
                if ks is not None and ks[0]:
                    roof[("correspondence_pass" if sub == "knn" else sub) + "_avg_us"] = round(ks[1] / ks[0] * 1e3, 2)

    cpu = None
    pose_err = None
    if rank == 0 and args.cpu_baseline_seconds > 0:
        # the reference path restated (oracle), single-threaded, same scans from scan 1 and the same prefilled
        # map; warm-up scans (optimization_count ramp) untimed, then steady-state scans for ~N seconds.
        oracle.reset_process_statics()
        ref = oracle.Odometry(R, SCAN_PERIOD, MIN_DIS, MAX_DIS, MAP_RES, LOSS, stable_voxel=True)
        ref.init_map(mapE, mapS)
        t_cpu, n_cpu, errs = 0.0, 0, []
        for k in range(n_scans):
            t1 = time.perf_counter()
            e, s = oracle_fe(raws[k], R)
            ref.update_selector(e, s, True)
            dt = time.perf_counter() - t1
            qr, tr = ref.pose()
            qg, tg = poses[k]
            errs.append((float(np.linalg.norm(tr - tg)), 2 * math.acos(min(1.0, abs(float(np.dot(qr, qg)))))))
            if k >= min(args.warmup, 6):
                t_cpu += dt
                n_cpu += 1
                if t_cpu >= args.cpu_baseline_seconds:
                    break
        if n_cpu:
            cpu = {"value": round(n_cpu / t_cpu, 4), "unit": "scans/s", "cores": 1, "kind": "port",
                   "sample": f"{cfg} scans {min(args.warmup, 6) + 1}..{min(args.warmup, 6) + n_cpu} (steady state) "
                             f"of the same sequence, featureExtraction + UpdatePointsToMapSelector, oracle/ "
                             f"single thread, {os.cpu_count()} host cores present"}
        pose_err = {"scans_compared": len(errs), "max_dt_m": max(e[0] for e in errs),
                    "max_drot_rad": max(e[1] for e in errs)}

    if rank == 0:
        gt_err = []
        for k, (q, t) in enumerate(poses):
            T = synth.gt_pose_matrix(scan_offset + k + 1)
            gt_err.append(float(np.linalg.norm(T[:3, 3] - t)))
        total_scans = args.steps * (world if args.mode == "replica" else 1)
        value = total_scans / elapsed
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "scans/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "weak" if args.mode == "replica" else "strong", "vs_baseline": None, "dtype": "fp32+fp64",
            "data": "synthetic (seeded ring-lidar ray-cast scene, floam_amd/synth.py)",
            "config": {"workload": f"{cfg}: {R}-ring synthetic scans ({raws[0].shape[0]} pts), map prefilled "
                                   f"{target} pts, deskew on, loss {LOSS} (no robust loss, Q3), map_res {MAP_RES}",
                       "rings": R, "points_per_scan": int(raws[0].shape[0]), "map_prefill": target,
                       "parallelism": (f"query-shard x{world} ({allreduce_impl or 'no'} all-reduce of J^T J)"
                                       if args.mode == "shard" else f"replica x{world}")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "pose_vs_oracle": pose_err,
            "pose_vs_ground_truth_rmse_m": round(math.sqrt(sum(e * e for e in gt_err) / len(gt_err)), 5),
            "last_scan_stats": {k: (int(v) if isinstance(v, int) else v) for k, v in stats.items()},
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    odo.close()
    lp.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
