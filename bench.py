#!/usr/bin/env python3
"""Benchmark: scans/sec of the FLOAM scan-to-map odometry hot path on MI355X.

One step = one scan through the reference's two operators, exactly as the nodes drive them:
LaserProcessingClass::featureExtraction (src/laserProcessingNode.cpp:129) followed by
OdomEstimationClass::UpdatePointsToMapSelector(edge, surf, deskew=true) (src/odomEstimationNode.cpp:228), with the
launch-file defaults (launch/structor_odom.launch: map_resolution 0.1, deskew on, loss "Cauchy" -> no robust
loss, min/max_dis 0.5/90).  The raw scans are resident in HBM before the timed region; the host collects every
update's pose (streamed, two updates in flight).

Workload at N = 1 (BASELINE.json configs[2], the headline): 64-ring HDL-64-style synthetic scans (~130k points),
local map prefilled with 200k edge+surf points through initMapWithPoints, steady state (the warm-up covers the
optimization_count 12 -> 2 ramp).

--gpus N > 1 (launched by torch.distributed.run) defaults to --mode shard on C4 (BASELINE.json configs[3]: 128-ring
~260k-point scans, 500k map, points sharded over the GPUs with an RCCL all-reduce of J^T J): every rank runs the same
sequence, the correspondence queries are split into N ranges, and the normal equations are summed with one RCCL
all-reduce per LM evaluation (SURVEY.md §8 e); value = scans of the one sequence per second (strong scaling).  Rank
0 also times the same sequence unsharded on its own GPU first ("same_config_1gpu").  --mode replica runs one
independent pipeline per GPU (value = scans of all ranks per second, weak scaling).

Prints ONE JSON line on rank 0 (contract in the task statement) with
  "roofline": the kNN search kernel (knn_kernel, edge + surf queries in one launch): algorithmic bytes (device-counted,
              SURVEY.md §8 d) / its average launch time from HIP events on the library stream, measured on an
              identical replay of the timed sequence; "traffic" = rocprofv3 FETCH/WRITE bytes per launch of the same
              kernel and config from the committed profiles/<tag>/hbm_traffic.json;
  "cpu_baseline": the CPU oracle (the reference path restated, single-threaded) on a bounded sample of the sequence;
  "secondary": featureExtraction alone (scans/s) and the same sequence with loss "huber" (SURVEY.md §8 d: "a second
              run uses loss=huber").
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


def code_hash():
    """sha256 (16 hex) of the device-code sources — floam_amd/csrc's kernels, headers, host code and Makefile plus
    include/floam_c.h — that the product library is built from.  tools/gpu_prof.sh records it next to a profile, so a
    bench line cites the PMC counters of the code it ran."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "floam_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "floam_amd", "csrc", "*.hpp")) +
                   glob.glob(os.path.join(ROOT, "floam_amd", "csrc", "*.cpp")) +
                   [os.path.join(ROOT, "floam_amd", "csrc", "Makefile"), os.path.join(ROOT, "include", "floam_c.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def hbm_traffic(kernel_substr, config, steps):
    """The committed rocprofv3 profile for the roofline kernel (profiles/<tag>/hbm_traffic.json, written by
    tools/prof_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE runs of this bench): of the SAME config, chosen
    first by the device-code hash the profile records (the code this bench runs), then by its step count, then by
    recency (its `created` stamp; older summaries carry none and rank last).  Returns a dict with the HBM bytes per
    launch, the profile's rocprof average duration of the kernel over its timed region (kernel_stats.csv) and whether
    code and steps match — or None when no profile of the config is committed."""
    import csv
    import glob
    want = code_hash()
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "*", "hbm_traffic.json")):
        d = json.load(open(f))
        if d.get("config", "c3") != config:
            continue
        hit = next(((n, v) for n, v in d.get("kernels", {}).items() if kernel_substr in n), None)
        if hit is None:
            continue
        rank = (d.get("code_hash") == want, d.get("steps") == steps, d.get("created", ""), f)
        if best is None or rank > best[0]:
            best = (rank, f, d, hit)
    if best is None:
        return None
    rank, f, d, (name, v) = best
    avg_us = None
    ks = os.path.join(os.path.dirname(f), "kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            if r["Name"] == name:
                avg_us = float(r["AvgUs"])
    return {"bytes": round(v["total_bytes"]), "source": os.path.relpath(f, ROOT), "rocprof_avg_us": avg_us,
            "code_match": rank[0], "steps_match": rank[1], "profile_code_hash": d.get("code_hash"),
            "profile_steps": d.get("steps")}


def main():
    # stdout carries exactly the one JSON line: the libraries' own stdout chatter (gloo's peer-connection notice,
    # RCCL's version banner) is sent to stderr at the file-descriptor level, before any of them initialises
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default=None, help="c1..c5 (default: c3 at N = 1, c4 for the sharded N > 1 run)")
    ap.add_argument("--mode", choices=["shard", "replica"], default=None,
                    help="N > 1: shard (default) or replica; N = 1: shard runs the sharded solve through a one-rank "
                         "RCCL communicator (the per-evaluation all-reduce measured on one GPU)")
    ap.add_argument("--oracle-scans", type=int, default=12,
                    help="N > 1: scans of the sequence the oracle replays for pose_vs_oracle (untimed)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--precision", choices=["fp64", "fp32", "fp32g"], default="fp64",
                    help="residual / Jacobian precision (floam_odom_set_precision): fp64 = the reference's (default); "
                         "fp32 = float residuals / Jacobians; fp32g = float line / plane fits too (C5 sweep)")
    ap.add_argument("--shard-comm", choices=["peer", "rccl"], default=os.environ.get("FLOAM_SHARD_COMM", "peer"),
                    help="sharded solve: peer = one resident LM launch per solve exchanging the ranks' sums through "
                         "IPC-mapped buffers (floam_odom_set_shard_peers; default), rccl = one launch + one "
                         "ncclAllReduce per LM evaluation (floam_odom_set_shard)")
    ap.add_argument("--no-c3-shard", action="store_true", help="N > 1 shard mode: skip the extra C3 sharded line")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist   # control plane only (barrier, id broadcast, max-time); data: RCCL
        dist.init_process_group(backend="gloo")
    mode = (args.mode or "shard") if world > 1 else ("shard" if args.mode == "shard" else "single")
    cfg = args.config or ("c4" if mode == "shard" else "c3")

    import floam_amd
    import oracle
    from floam_amd import _ffi, synth
    from floam_amd.odom_estimation import comm_unique_id, reset_process_state

    L = _ffi.load()
    dev = int(os.environ.get("FLOAM_BENCH_DEVICE", local_rank))   # override: several ranks on one GPU (testing)
    model = synth.lidar_model(cfg)
    R = model.rings
    target = synth.MAP_PREFILL.get(cfg, 0)
    params = floam_amd.LidarParams(num_lines=R, scan_period=SCAN_PERIOD, vertical_angle=2.0, max_distance=MAX_DIS,
                                   min_distance=MIN_DIS)

    def oracle_fe(raw, R_):   # the CPU baseline leg only
        e, s, _ = oracle.feature_extraction(raw, R_, MIN_DIS, MAX_DIS, canonical=True)
        return e, s

    fe_lp = floam_amd.LaserProcessingClass(device=dev)
    fe_lp.init(params)

    def gpu_fe(raw, R_):   # featureExtraction on the GPU (untimed: the prefill's earlier scans)
        de, ds = floam_amd.DeviceCloud(device=dev), floam_amd.DeviceCloud(device=dev)
        fe_lp.featureExtraction(floam_amd.DeviceCloud(raw, device=dev), de, ds)
        return de.download(), ds.download()

    t0 = time.time()
    n_scans = args.warmup + args.steps
    # every rank runs the same synthetic sequence (replicas: same work per rank as at N = 1; a sequence that starts
    # elsewhere on the trajectory would not match the map prefilled around the origin)
    raws = [synth.generate_scan(cfg, k) for k in range(1, n_scans + 1)]
    mapE, mapS = synth.prefill_map(cfg, gpu_fe, target)
    fe_lp.close()
    log(f"[rank {rank}] generated {n_scans} scans ({raws[0].shape[0]} pts) + map {mapE.shape[0]}+{mapS.shape[0]} "
        f"in {time.time() - t0:.1f}s")

    d_raw = [floam_amd.DeviceCloud(r, device=dev) for r in raws]       # inputs resident in HBM
    d_mapE, d_mapS = floam_amd.DeviceCloud(mapE, device=dev), floam_amd.DeviceCloud(mapS, device=dev)
    allreduce_impl = None
    uid = None
    if mode == "shard":
        # one RCCL communicator per sharded pipeline: timed run, byte-count replay, the C3 line, a fallback rebuild
        uid = [tuple(comm_unique_id() for _ in range(4)) if rank == 0 else None]
        if dist is not None:
            dist.broadcast_object_list(uid, src=0)
    n_pipelines = 0

    peer_ok = [args.shard_comm == "peer"]

    def set_peers(odo):
        """peer sharding: every rank's exchange-buffer IPC handle, gathered over the control plane (gloo); False
        (RCCL instead) when any rank cannot map the others' buffers"""
        ok = True
        try:
            h, _ = odo.shard_exchange()
        except floam_amd.FloamError as e:
            log(f"[rank {rank}] peer exchange buffer unavailable ({e})")
            ok, h = False, b""
        # every rank's GPU must be able to read the others' memory (xGMI peer access) before the solve polls it
        devs = [None] * world
        dist.all_gather_object(devs, dev)
        try:
            import torch
            for d in set(devs):
                if d != dev and not torch.cuda.can_device_access_peer(dev, d):
                    log(f"[rank {rank}] GPU {dev} cannot access GPU {d}: no peer exchange")
                    ok = False
        except Exception as e:   # (no peer query: fall back to RCCL rather than risk a fault)
            log(f"[rank {rank}] peer access query failed ({e})")
            ok = False
        handles = [None] * world
        dist.all_gather_object(handles, h)
        if ok and all(len(x) == 64 for x in handles):
            try:
                odo.set_shard_peers(rank, world, handles=handles)
            except floam_amd.FloamError as e:
                log(f"[rank {rank}] peer mapping failed ({e})")
                ok = False
        import torch
        t = torch.tensor([0 if ok else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item()) == 0

    def make_pipeline(loss=LOSS, sharded=True, params_=None, maps=None):
        nonlocal allreduce_impl, n_pipelines
        params_ = params_ or params
        joint = uid is not None and sharded and dist is not None   # every rank builds this pipeline together
        reset_process_state()
        lp = floam_amd.LaserProcessingClass(device=dev, asynchronous=True)   # the odometry collects the counts
        lp.init(params_)
        odo = floam_amd.OdomEstimationClass(device=dev)
        odo.init(params_, MAP_RES, loss)
        if args.precision != "fp64":
            odo.set_precision(True, geometry=args.precision == "fp32g")
        if uid is not None and sharded and world > 1 and peer_ok[0]:
            if set_peers(odo):
                allreduce_impl = "peer"
                n_pipelines += 1
                sharded = False   # (configured)
            else:
                log(f"[rank {rank}] peer sharding unavailable: RCCL all-reduce instead")
                peer_ok[0] = False
        if uid is not None and sharded:
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
            n_pipelines += 1
        m = maps or (d_mapE, d_mapS)
        odo.initMapWithPoints(m[0], m[1])
        odo.set_async(DEPTH)
        if joint:
            dist.barrier()   # (sharded ranks start their solves together: a peer waits for the others' sums)
        return lp, odo

    # feature buffers: the extraction of scan k+1 (its own stream) is issued before the odometry of scan k, so the
    # two overlap on the device, as the reference's laserProcessingNode runs beside odomEstimationNode.  DEPTH + 1
    # buffers: the extraction into a buffer is issued once the update that last read it has been collected, so it
    # needs no cross-stream wait on the odometry stream
    bufs = [(floam_amd.DeviceCloud(device=dev), floam_amd.DeviceCloud(device=dev)) for _ in range(max(3, DEPTH + 1))]

    def extract(lp, k, src=None):
        e, s = bufs[k % len(bufs)]
        e.clear()
        s.clear()
        lp.featureExtraction((src or d_raw)[k], e, s)

    host_split = [0.0, 0.0]   # host seconds issuing / waiting (diagnostic, FLOAM_BENCH_HOST=1)

    host_trace = [] if os.environ.get("FLOAM_BENCH_HOST_TRACE") else None   # (diagnostic) monotonic ns per scan

    def run(lp, odo, a, b, poses, src=None):
        """scans [a, b): featureExtraction + UpdatePointsToMapSelector each, extraction one scan ahead; the odometry
        streams (floam_odom_set_async): scan k's pose is collected after scan k+1 has been issued"""
        if a < b:
            extract(lp, a, src)
        for k in range(a, b):
            t0 = time.perf_counter()
            m0 = time.monotonic_ns()
            if k + 1 < b:
                extract(lp, k + 1, src)
            m1 = time.monotonic_ns()
            e, s = bufs[k % len(bufs)]
            odo.UpdatePointsToMapSelector(e, s, True)
            t1 = time.perf_counter()
            m2 = time.monotonic_ns()
            poses.extend(odo.wait(DEPTH - 1))
            host_split[0] += t1 - t0
            host_split[1] += time.perf_counter() - t1
            if host_trace is not None:
                host_trace.append((k, m0, m1, m2, time.monotonic_ns()))
        poses.extend(odo.wait(0))

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        _ffi.check(L.floam_device_synchronize(dev))

    def timed_sequence(loss=LOSS, sharded=True):
        lp, odo = make_pipeline(loss, sharded)
        poses = []
        run(lp, odo, 0, args.warmup, poses)
        _ffi.check(L.floam_device_synchronize(dev))
        t_start = time.perf_counter()
        run(lp, odo, args.warmup, n_scans, poses)
        _ffi.check(L.floam_device_synchronize(dev))
        dt = time.perf_counter() - t_start
        odo.close()
        lp.close()
        return dt, poses

    same_cfg_1gpu = None
    if mode == "shard" and rank == 0:   # the same sequence unsharded on this GPU: the strong-scaling reference
        dt1, _ = timed_sequence(sharded=False)
        same_cfg_1gpu = round(args.steps / dt1, 3)
    lp, odo = make_pipeline()
    poses = []
    peer_failed = False
    try:
        run(lp, odo, 0, args.warmup, poses)
    except floam_amd.FloamError as e:   # (the peer exchange is the one path that can fail here on a new node)
        if allreduce_impl != "peer":
            raise
        log(f"[rank {rank}] peer exchange failed in the warm-up ({e})")
        peer_failed = True
    if allreduce_impl == "peer" and dist is not None:
        import torch
        t = torch.tensor([1 if peer_failed else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(t.item()):   # every rank leaves the peer exchange together and shards through RCCL instead
            for h in (odo, lp):
                try:
                    h.close()
                except floam_amd.FloamError:
                    pass
            peer_ok[0] = False
            lp, odo = make_pipeline()
            poses = []
            run(lp, odo, 0, args.warmup, poses)
    barrier_sync()
    _ffi.check(L.floam_profile_mark(dev, 1))   # trace marker: the timed region starts (tools/prof_summary.py)
    barrier_sync()
    host_split[:] = [0.0, 0.0]
    t_start = time.perf_counter()
    run(lp, odo, args.warmup, n_scans, poses)
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    _ffi.check(L.floam_profile_mark(dev, 2))   # ... and ends
    if host_trace is not None:
        json.dump(host_trace, open(os.environ["FLOAM_BENCH_HOST_TRACE"], "w"))
    if os.environ.get("FLOAM_BENCH_HOST"):
        log(f"[host] per timed scan: issue {1e6 * host_split[0] / args.steps:.0f} us, "
            f"wait {1e6 * host_split[1] / args.steps:.0f} us")
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stats = odo.stats()

    def read_timings():
        arr = (_ffi.KernelTiming * 64)()
        n = C.c_int()
        _ffi.check(L.floam_profile_read(dev, arr, 64, C.byref(n)))
        return {arr[i].name.decode(): (arr[i].launches, arr[i].total_ms, arr[i].algorithmic_bytes)
                for i in range(min(n.value, 64))}

    roof = None
    if not args.no_roofline:
        odo.close()
        lp.close()
        # The roofline kernel — the exact 5-NN search (knn_kernel, edge + surf queries in one launch) — measured on an
        # identical replay of the same sequence (the pipeline is deterministic; the poses are checked bit for bit):
        # HIP events on the library stream around every search launch (FLOAM_PROF_KNN_DETAIL) and the byte-counting
        # kernel after each pass (FLOAM_PROF_KNN_BYTES, SURVEY.md §8 d).  The timed run above has no events and no
        # byte counting inside it.
        lp, odo = make_pipeline()
        replay = []
        run(lp, odo, 0, args.warmup, replay)
        _ffi.check(L.floam_profile_reset(dev))
        _ffi.check(L.floam_profile_enable(dev, 1 | 2 | 16 | 32))
        run(lp, odo, args.warmup, n_scans, replay)
        _ffi.check(L.floam_profile_enable(dev, 0))
        timed = read_timings()
        same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(poses, replay))
        kt = timed.get("knn_search")
        if kt is not None and kt[0] > 0:
            # HIP events set by the search launch itself (hipExtLaunchKernel: the dispatch's start / end, the duration
            # rocprofv3 reports); "bracket_avg_us": events recorded on the stream around the launch (+ dispatch gaps)
            avg_ms = kt[1] / kt[0]
            bytes_per = kt[2] / kt[0]
            ach = bytes_per / (avg_ms * 1e-3) / 1e9
            tr = hbm_traffic("knn_kernel<", cfg, args.steps)
            roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": tr["bytes"] if tr else None,
                    "traffic_source": tr["source"] if tr else None,
                    "kernel": "knn_kernel (exact 5-NN search over the hash grid, edge + surf queries)",
                    "avg_us": round(avg_ms * 1e3, 2), "launches": int(kt[0]),
                    "algorithmic_bytes_per_launch": round(bytes_per), "replay_bitwise_identical": bool(same),
                    "code_hash": code_hash()}
            kb = timed.get("knn_search_bracket")
            if kb is not None and kb[0]:
                roof["bracket_avg_us"] = round(kb[1] / kb[0] * 1e3, 2)
            if tr:
                # the committed profile of this code: its rocprof average for the kernel, and the fraction it gives
                roof.update({"traffic_code_match": tr["code_match"], "traffic_steps_match": tr["steps_match"],
                             "rocprof_avg_us": tr["rocprof_avg_us"]})
                if tr["rocprof_avg_us"]:
                    roof["frac_rocprof"] = round(bytes_per / (tr["rocprof_avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
            for sub, key in (("knn", "correspondence_pass_avg_us"), ("knn_geometry", "knn_geometry_avg_us"),
                             ("lm_solve", "lm_solve_avg_us"), ("lm_solve_sharded", "lm_solve_avg_us")):
                ks = timed.get(sub)
                if ks is not None and ks[0]:
                    roof[key] = round(ks[1] / ks[0] * 1e3, 2)
            # the north star prices the kNN search against HBM; the largest kernel by time per scan is the LM solve
            # (4 launches of ~36 us at C3), which moves < 1 MB per launch and is bound by its serial chain (one
            # hand-off + one fp64 control step per LM evaluation), not by a roofline
            roof["largest_kernel_by_time"] = {"kernel": "lm_solve", "avg_us": roof.get("lm_solve_avg_us"),
                                              "bound": "latency (serial fp64 control step + one inter-block "
                                                       "hand-off per LM evaluation)"}

    def dropin_sync(ref_poses):
        """The drop-in contract: host-resident PointXYZIRT scans through exactly the INTEGRATION.md
        adapters' calls, one scan per callback, everything synchronous (src/laserProcessingNode.cpp:129,
        src/odomEstimationNode.cpp:205-244): featureExtraction = raw upload + extraction + edge / surf download (the
        processing node publishes host clouds); UpdatePointsToMapSelector = edge / surf upload + the update (async
        off) + the Q5 write-back downloads (size + download each, as the adapter's download()) + get_pose +
        get_last_pose.  Same scans and prefilled map as the headline run; the poses must equal the resident run's."""
        reset_process_state()
        lp_ = floam_amd.LaserProcessingClass(device=dev)
        lp_.init(params)
        odo_ = floam_amd.OdomEstimationClass(device=dev)
        odo_.init(params, MAP_RES, LOSS)
        odo_.initMapWithPoints(d_mapE, d_mapS)
        hL, h_lp, h_odo = L, lp_._h, odo_._h
        c_in, c_e, c_s = (floam_amd.DeviceCloud(device=dev) for _ in range(3))   # processing node
        o_e, o_s = floam_amd.DeviceCloud(device=dev), floam_amd.DeviceCloud(device=dev)   # odometry node
        he = np.zeros(max(64 * 1024, raws[0].shape[0]), synth.POINT_DTYPE)
        hs = np.zeros(raws[0].shape[0] + 1024, synth.POINT_DTYPE)
        vp = C.c_void_p
        q, t, q2, t2 = np.zeros(4), np.zeros(3), np.zeros(4), np.zeros(3)
        qp, tp = q.ctypes.data_as(C.POINTER(C.c_double)), t.ctypes.data_as(C.POINTER(C.c_double))
        q2p, t2p = q2.ctypes.data_as(C.POINTER(C.c_double)), t2.ctypes.data_as(C.POINTER(C.c_double))
        n_ = C.c_size_t()
        seg = np.zeros(6)   # seconds: raw upload, extraction, FE downloads, odometry uploads, update, write-back + poses
        got = []

        def download(c, buf):
            _ffi.check(hL.floam_cloud_size(c.handle, C.byref(n_)))
            n = n_.value
            _ffi.check(hL.floam_cloud_download(c.handle, vp(buf.ctypes.data), n, C.byref(n_)))
            return n

        def one(k):
            raw = raws[k]
            t0 = time.perf_counter()
            _ffi.check(hL.floam_cloud_upload(c_in.handle, vp(raw.ctypes.data), raw.shape[0], 32))
            t1 = time.perf_counter()
            _ffi.check(hL.floam_cloud_clear(c_e.handle))
            _ffi.check(hL.floam_cloud_clear(c_s.handle))
            _ffi.check(hL.floam_lp_feature_extraction(h_lp, c_in.handle, c_e.handle, c_s.handle))
            t2 = time.perf_counter()
            ne, ns = download(c_e, he), download(c_s, hs)
            t3 = time.perf_counter()
            _ffi.check(hL.floam_cloud_upload(o_e.handle, vp(he.ctypes.data), ne, 32))
            _ffi.check(hL.floam_cloud_upload(o_s.handle, vp(hs.ctypes.data), ns, 32))
            t4 = time.perf_counter()
            _ffi.check(hL.floam_odom_update_selector(h_odo, o_e.handle, o_s.handle, 1))
            t5 = time.perf_counter()
            download(o_e, he)
            download(o_s, hs)
            _ffi.check(hL.floam_odom_get_pose(h_odo, qp, tp))
            _ffi.check(hL.floam_odom_get_last_pose(h_odo, q2p, t2p))
            t6 = time.perf_counter()
            return np.array([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5])

        for k in range(args.warmup):
            one(k)
            got.append((q.copy(), t.copy()))
        t_start = time.perf_counter()
        for k in range(args.warmup, n_scans):
            seg += one(k)
            got.append((q.copy(), t.copy()))
        dt = time.perf_counter() - t_start
        same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(ref_poses, got))
        for c in (c_in, c_e, c_s, o_e, o_s):
            c.close()
        odo_.close()
        lp_.close()
        us = 1e6 / args.steps
        return {"value": round(args.steps / dt, 2), "unit": "scans/s", "ms_per_scan": round(1e3 * dt / args.steps, 3),
                "poses_equal_resident_run": bool(same),
                "segments_us_per_scan": {"raw_upload": round(seg[0] * us, 1), "feature_extraction": round(seg[1] * us, 1),
                                         "fe_downloads": round(seg[2] * us, 1),
                                         "odom_uploads": round(seg[3] * us, 1), "update": round(seg[4] * us, 1),
                                         "writeback_downloads_and_poses": round(seg[5] * us, 1)},
                "calls": "per scan: floam_cloud_upload(raw), floam_lp_feature_extraction (sync), size+download x2, "
                         "floam_cloud_upload x2, floam_odom_update_selector (async off, deskew), size+download x2 (Q5), "
                         "floam_odom_get_pose, floam_odom_get_last_pose (INTEGRATION.md adapters)"}

    def dropin_host(ref_poses):
        """The drop-in contract through the one-call host entry points the INTEGRATION.md adapters use when built
        against ABI 2 (floam_lp_feature_extraction_host, floam_odom_update_selector_host): per scan one upload + the
        extraction + both downloads with one synchronisation, then both uploads + the synchronous update with the
        deskewed records copied back (Q5) on a copy stream while the update's second call runs, + the two pose reads."""
        reset_process_state()
        lp_ = floam_amd.LaserProcessingClass(device=dev)
        lp_.init(params)
        odo_ = floam_amd.OdomEstimationClass(device=dev)
        odo_.init(params, MAP_RES, LOSS)
        odo_.initMapWithPoints(d_mapE, d_mapS)
        hL, h_lp, h_odo = L, lp_._h, odo_._h
        he = np.zeros(R * 120 + 1, synth.POINT_DTYPE)
        hs = np.zeros(raws[0].shape[0] + 1024, synth.POINT_DTYPE)
        vp = C.c_void_p
        q, t, q2, t2 = np.zeros(4), np.zeros(3), np.zeros(4), np.zeros(3)
        qp, tp = q.ctypes.data_as(C.POINTER(C.c_double)), t.ctypes.data_as(C.POINTER(C.c_double))
        q2p, t2p = q2.ctypes.data_as(C.POINTER(C.c_double)), t2.ctypes.data_as(C.POINTER(C.c_double))
        ne, ns = C.c_size_t(), C.c_size_t()
        seg = np.zeros(3)
        got = []

        def one(k):
            raw = raws[k]
            t0 = time.perf_counter()
            _ffi.check(hL.floam_lp_feature_extraction_host(h_lp, vp(raw.ctypes.data), raw.shape[0], 32,
                                                           vp(he.ctypes.data), he.shape[0], C.byref(ne),
                                                           vp(hs.ctypes.data), hs.shape[0], C.byref(ns)))
            t1 = time.perf_counter()
            _ffi.check(hL.floam_odom_update_selector_host(h_odo, vp(he.ctypes.data), ne.value, vp(hs.ctypes.data),
                                                          ns.value, 32, 1))
            t2_ = time.perf_counter()
            _ffi.check(hL.floam_odom_get_pose(h_odo, qp, tp))
            _ffi.check(hL.floam_odom_get_last_pose(h_odo, q2p, t2p))
            t3 = time.perf_counter()
            return np.array([t1 - t0, t2_ - t1, t3 - t2_])

        for k in range(args.warmup):
            one(k)
            got.append((q.copy(), t.copy()))
        t_start = time.perf_counter()
        for k in range(args.warmup, n_scans):
            seg += one(k)
            got.append((q.copy(), t.copy()))
        dt = time.perf_counter() - t_start
        same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(ref_poses, got))
        odo_.close()
        lp_.close()
        us = 1e6 / args.steps
        return {"value": round(args.steps / dt, 2), "unit": "scans/s", "ms_per_scan": round(1e3 * dt / args.steps, 3),
                "poses_equal_resident_run": bool(same),
                "segments_us_per_scan": {"feature_extraction_host": round(seg[0] * us, 1),
                                         "update_selector_host": round(seg[1] * us, 1),
                                         "poses": round(seg[2] * us, 1)},
                "calls": "per scan: floam_lp_feature_extraction_host, floam_odom_update_selector_host (deskew), "
                         "floam_odom_get_pose, floam_odom_get_last_pose"}

    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary:
        odo.close()
        lp.close()
        # featureExtraction alone over the timed scans (its own stream, no odometry behind it)
        fe = floam_amd.LaserProcessingClass(device=dev, asynchronous=True)
        fe.init(params)
        for k in range(args.warmup):
            extract(fe, k)
        _ffi.check(L.floam_device_synchronize(dev))
        t1 = time.perf_counter()
        for k in range(args.warmup, n_scans):
            extract(fe, k)
        _ffi.check(L.floam_device_synchronize(dev))
        fe_dt = time.perf_counter() - t1
        fe.close()
        # the same sequence with loss "huber" (HuberLoss(0.1), src/odomEstimationClass.cpp:84-87)
        hub_dt, hub_poses = timed_sequence("huber")
        secondary = {"feature_extraction_alone": {"value": round(args.steps / fe_dt, 2), "unit": "scans/s"},
                     "huber": {"value": round(args.steps / hub_dt, 3), "unit": "scans/s",
                               "loss": "huber (HuberLoss(0.1))"},
                     "dropin_sync": dropin_sync(poses), "dropin_host": dropin_host(poses)}

    cpu = None
    pose_err = None
    if rank == 0 and world > 1 and args.oracle_scans > 0:
        # N > 1: the poses of the sharded (or replicated) run against the oracle over the first scans of the same
        # sequence (untimed; the CPU baseline itself is an N = 1 figure)
        oracle.reset_process_statics()
        ref = oracle.Odometry(R, SCAN_PERIOD, MIN_DIS, MAX_DIS, MAP_RES, LOSS, stable_voxel=True)
        ref.init_map(mapE, mapS)
        errs = []
        for k in range(min(n_scans, args.oracle_scans)):
            e, s = oracle_fe(raws[k], R)
            ref.update_selector(e, s, True)
            qr, tr = ref.pose()
            qg, tg = poses[k]
            errs.append((float(np.linalg.norm(tr - tg)), 2 * math.acos(min(1.0, abs(float(np.dot(qr, qg)))))))
        pose_err = {"scans_compared": len(errs), "max_dt_m": max(e[0] for e in errs),
                    "max_drot_rad": max(e[1] for e in errs)}
    elif rank == 0 and args.cpu_baseline_seconds > 0:
        # the reference path restated (oracle), single-threaded, same scans from scan 1 and the same prefilled
        # map; warm-up scans (optimization_count ramp) untimed, then steady-state scans for ~N seconds.
        oracle.reset_process_statics()
        ref = oracle.Odometry(R, SCAN_PERIOD, MIN_DIS, MAX_DIS, MAP_RES, LOSS, stable_voxel=True)   # fp64 always
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
        if os.environ.get("FLOAM_BENCH_POSE_LOG"):   # per-scan agreement (diagnostic)
            for k, (et, er) in enumerate(errs):
                log(f"[pose] scan {k + 1}: {et:.3e} m {er:.3e} rad")

    c3_line = None
    if mode == "shard" and world > 1 and cfg != "c3" and not args.no_c3_shard:
        # the headline config sharded too, beside the C4 line (same scheme: max over ranks of the
        # timed region; rank 0 first times it unsharded on its own GPU)
        odo.close()
        lp.close()
        m3 = synth.lidar_model("c3")
        p3 = floam_amd.LidarParams(num_lines=m3.rings, scan_period=SCAN_PERIOD, vertical_angle=2.0,
                                   max_distance=MAX_DIS, min_distance=MIN_DIS)
        fe3 = floam_amd.LaserProcessingClass(device=dev)
        fe3.init(p3)

        def gpu_fe3(raw, R_):
            de, ds = floam_amd.DeviceCloud(device=dev), floam_amd.DeviceCloud(device=dev)
            fe3.featureExtraction(floam_amd.DeviceCloud(raw, device=dev), de, ds)
            return de.download(), ds.download()

        raws3 = [synth.generate_scan("c3", k) for k in range(1, n_scans + 1)]
        mE3, mS3 = synth.prefill_map("c3", gpu_fe3, synth.MAP_PREFILL.get("c3", 0))
        fe3.close()
        d_raw3 = [floam_amd.DeviceCloud(r, device=dev) for r in raws3]
        maps3 = (floam_amd.DeviceCloud(mE3, device=dev), floam_amd.DeviceCloud(mS3, device=dev))
        c3_1gpu = None
        if rank == 0:
            lp3, odo3 = make_pipeline(sharded=False, params_=p3, maps=maps3)
            ps3 = []
            run(lp3, odo3, 0, args.warmup, ps3, d_raw3)
            _ffi.check(L.floam_device_synchronize(dev))
            t1 = time.perf_counter()
            run(lp3, odo3, args.warmup, n_scans, ps3, d_raw3)
            _ffi.check(L.floam_device_synchronize(dev))
            c3_1gpu = round(args.steps / (time.perf_counter() - t1), 3)
            odo3.close()
            lp3.close()
        lp3, odo3 = make_pipeline(params_=p3, maps=maps3)
        ps3 = []
        run(lp3, odo3, 0, args.warmup, ps3, d_raw3)
        barrier_sync()
        t1 = time.perf_counter()
        run(lp3, odo3, args.warmup, n_scans, ps3, d_raw3)
        barrier_sync()
        import torch
        t = torch.tensor([time.perf_counter() - t1], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        odo3.close()
        lp3.close()
        c3_line = {"value": round(args.steps / float(t.item()), 3), "unit": "scans/s",
                   "config": f"c3: {m3.rings}-ring synthetic scans ({raws3[0].shape[0]} pts), map prefilled "
                             f"{synth.MAP_PREFILL.get('c3', 0)} pts, sharded like the main line ({allreduce_impl})",
                   "same_config_1gpu": c3_1gpu}
        # the deployment that scales: every rank runs its own C3 sequence unsharded (one odometry per
        # sensor); the aggregate is all ranks' scans over the max-over-ranks time of the same timed region
        lp3, odo3 = make_pipeline(sharded=False, params_=p3, maps=maps3)
        ps3 = []
        run(lp3, odo3, 0, args.warmup, ps3, d_raw3)
        barrier_sync()
        t1 = time.perf_counter()
        run(lp3, odo3, args.warmup, n_scans, ps3, d_raw3)
        barrier_sync()
        t = torch.tensor([time.perf_counter() - t1], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        odo3.close()
        lp3.close()
        c3_line["replica"] = {"value": round(world * args.steps / float(t.item()), 3), "unit": "scans/s",
                              "scaling": "weak", "note": f"replica x{world}: every rank its own unsharded c3 "
                                                         f"sequence (all ranks' scans / max-over-ranks time)"}
        for c in list(d_raw3) + list(maps3):
            c.close()
        lp, odo = None, None

    if rank == 0:
        gt_err = []
        for k, (q, t) in enumerate(poses):
            T = synth.gt_pose_matrix(k + 1)
            gt_err.append(float(np.linalg.norm(T[:3, 3] - t)))
        total_scans = args.steps * (world if mode == "replica" else 1)
        value = total_scans / elapsed
        if mode == "shard" and allreduce_impl == "peer":
            par = (f"query-shard x{world} (resident LM solve: the ranks' J^T J / J^T r / cost exchanged through "
                   f"IPC-mapped peer buffers once per LM evaluation, no collective launch)")
        elif mode == "shard":
            par = f"query-shard x{world} ({allreduce_impl} all-reduce of J^T J per LM evaluation)"
        else:
            par = f"replica x{world}" if world > 1 else "single GPU"
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "scans/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if mode == "shard" else "weak", "vs_baseline": None,
            "dtype": "fp32+fp64" if args.precision == "fp64" else "fp32",
            "data": "synthetic (seeded ring-lidar ray-cast scene, floam_amd/synth.py)",
            "config": {"workload": f"{cfg}: {R}-ring synthetic scans ({raws[0].shape[0]} pts), map prefilled "
                                   f"{target} pts, deskew on, loss {LOSS} (no robust loss, Q3), map_res {MAP_RES}",
                       "rings": R, "points_per_scan": int(raws[0].shape[0]), "map_prefill": target,
                       "parallelism": par, "precision": args.precision},
            "roofline": roof,
            "cpu_baseline": cpu,
            "pose_vs_oracle": pose_err,
            "pose_vs_ground_truth_rmse_m": round(math.sqrt(sum(e * e for e in gt_err) / len(gt_err)), 5),
            "secondary": secondary,
            "last_scan_stats": {k: (int(v) if isinstance(v, int) else v) for k, v in stats.items()},
        }
        if c3_line is not None:
            out["c3_sharded"] = c3_line
        if same_cfg_1gpu is not None:
            out["same_config_1gpu"] = {"value": same_cfg_1gpu, "unit": "scans/s",
                                       "note": f"{cfg} unsharded on rank 0's GPU before the sharded run"}
        line = json.dumps(out)
        print(line, file=json_out, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if odo is not None:
        odo.close()
        lp.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
