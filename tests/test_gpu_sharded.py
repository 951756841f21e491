"""Sharded odometry on the GPU: two ranks (processes) shard the correspondence queries and sum the normal
equations once per LM evaluation.  On the one-GPU test box RCCL cannot put two ranks on one device, so the
all-reduce goes through floam_odom_set_shard_callback + torch.distributed/gloo; everything else (query ranges,
per-rank partial sums, LM control on the reduced sums) is the production sharded kernel path.  Poses must match
the unsharded GPU run and be identical on both ranks."""
import math
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NSCAN = 5


def _run(rank, world, port, q, rccl_world1=False, loss="Cauchy", fp32=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import floam_amd
        from floam_amd import synth
        from floam_amd.odom_estimation import reset_process_state
        p = floam_amd.LidarParams(num_lines=16, scan_period=0.1, max_distance=90.0, min_distance=0.5)
        lp = floam_amd.LaserProcessingClass(device=0)
        lp.init(p)
        odo = floam_amd.OdomEstimationClass(device=0)
        odo.init(p, 0.1, loss)
        if fp32:
            odo.set_precision(True)
        reset_process_state()
        if rccl_world1:   # the sharded solve through a one-rank RCCL communicator (ncclAllReduce on the stream)
            from floam_amd.odom_estimation import comm_unique_id
            odo.set_shard(0, 1, comm_unique_id())
        if world > 1:
            def allreduce(arr):
                t = torch.from_numpy(arr)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
            odo.set_shard_callback(rank, world, allreduce)
        poses = []
        for k in range(NSCAN):
            de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
            lp.featureExtraction(floam_amd.DeviceCloud(synth.generate_scan("c1", k), device=0), de, ds)
            if k == 0:
                odo.initMapWithPoints(de, ds)
            else:
                odo.UpdatePointsToMapSelector(de, ds, True)
            q_, t_ = odo.pose()
            poses.append(np.r_[q_, t_])
        if q is not None:
            q.put((rank, np.array(poses)))
        return np.array(poses)
    finally:
        if world > 1:
            dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_two_ranks_match_unsharded(floam_gpu):
    import torch.multiprocessing as mp
    ref = _run(0, 1, _free_port(), None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert np.array_equal(res[0], res[1])   # every rank takes the same LM decisions
    for k in range(NSCAN):
        dt = np.linalg.norm(res[0][k][4:] - ref[k][4:])
        dr = 2 * math.acos(min(1.0, abs(float(np.dot(res[0][k][:4], ref[k][:4])))))
        assert dt < 1e-9 and dr < 1e-9, (k, dt, dr)


C4_SCANS = 2


def _run_c4(rank, world, port, q, mapE, mapS, rccl_world1=False):
    """BASELINE.json configs[3] (C4: 128 rings, ~262k-point scans, 500k prefill): the sharded path on scans
    1..C4_SCANS, extraction on the GPU, the map prefilled through initMapWithPoints."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import floam_amd
        from floam_amd import synth
        from floam_amd.odom_estimation import comm_unique_id, reset_process_state
        p = floam_amd.LidarParams(num_lines=128, scan_period=0.1, max_distance=90.0, min_distance=0.5)
        lp = floam_amd.LaserProcessingClass(device=0)
        lp.init(p)
        odo = floam_amd.OdomEstimationClass(device=0)
        odo.init(p, 0.1, "Cauchy")
        reset_process_state()
        if rccl_world1:
            odo.set_shard(0, 1, comm_unique_id())
        if world > 1:
            def allreduce(arr):
                t = torch.from_numpy(arr)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
            odo.set_shard_callback(rank, world, allreduce)
        odo.initMapWithPoints(floam_amd.DeviceCloud(mapE, device=0), floam_amd.DeviceCloud(mapS, device=0))
        poses = []
        for k in range(1, C4_SCANS + 1):
            de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
            lp.featureExtraction(floam_amd.DeviceCloud(synth.generate_scan("c4", k), device=0), de, ds)
            odo.UpdatePointsToMapSelector(de, ds, True)
            q_, t_ = odo.pose()
            poses.append(np.r_[q_, t_])
        out = (np.array(poses), odo.map_sizes())
        if q is not None:
            q.put((rank, out))
        return out
    finally:
        if world > 1:
            dist.destroy_process_group()


def _c4_oracle(oracle_lib, mapE, mapS):
    from floam_amd import synth
    ref = oracle_lib.Odometry(128, 0.1, 0.5, 90.0, 0.1, "Cauchy", stable_voxel=True)
    oracle_lib.reset_process_statics()
    ref.init_map(mapE, mapS)
    poses = []
    for k in range(1, C4_SCANS + 1):
        e, s, _ = oracle_lib.feature_extraction(synth.generate_scan("c4", k), 128, 0.5, 90.0, canonical=True)
        ref.update_selector(e, s, True)
        q_, t_ = ref.pose()
        poses.append(np.r_[q_, t_])
    return np.array(poses), (ref.map(0).shape[0], ref.map(1).shape[0])


def _assert_close_to_oracle(got, ref, what, tol=1e-6):
    for k in range(len(ref)):
        dt = float(np.linalg.norm(got[k][4:] - ref[k][4:]))
        dr = 2 * math.acos(min(1.0, abs(float(np.dot(got[k][:4], ref[k][:4])))))
        assert dt < tol and dr < tol, (what, k + 1, dt, dr)


def test_sharded_two_ranks_c4_match_oracle(floam_gpu, oracle_lib, prefilled_map):
    """the query-sharded path at the config the north star shards (C4, 500k prefill): two ranks on
    one GPU (the host all-reduce over gloo stands in for RCCL, which refuses two ranks on one device), poses
    identical on both ranks and within 1e-6 m / rad of the oracle; map sizes equal to the oracle's."""
    import torch.multiprocessing as mp
    mapE, mapS = prefilled_map("c4")
    ref, ref_sizes = _c4_oracle(oracle_lib, mapE, mapS)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_c4, args=(r, 2, port, q, mapE, mapS)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert np.array_equal(res[0][0], res[1][0])   # every rank takes the same LM decisions
    assert res[0][1] == res[1][1] == ref_sizes, (res[0][1], res[1][1], ref_sizes)
    _assert_close_to_oracle(res[0][0], ref, "2-rank shard")


def test_rccl_world1_c4_matches_oracle(floam_gpu, oracle_lib, prefilled_map):
    """The sharded solve through a one-rank RCCL communicator (ncclAllReduce on the library stream) at C4."""
    mapE, mapS = prefilled_map("c4")
    ref, ref_sizes = _c4_oracle(oracle_lib, mapE, mapS)
    got, sizes = _run_c4(0, 1, _free_port(), None, mapE, mapS, rccl_world1=True)
    assert sizes == ref_sizes
    _assert_close_to_oracle(got, ref, "RCCL world 1")


@pytest.mark.parametrize("loss,fp32", [("Cauchy", False), ("huber", False), ("Cauchy", True)])
def test_rccl_world1_matches_unsharded(floam_gpu, loss, fp32):
    """The sharded solve (one launch + one ncclAllReduce of the 29 sums per LM evaluation, the control step folded
    into the next launch) on a one-rank RCCL communicator: the same partition and fixed-order reductions as the
    resident single-GPU solve.  lm.hip is compiled with FMA contraction, which the compiler may apply differently
    in the two kernels, so the fp64 poses agree to the last few ulps (observed <= 1e-15 m) rather than bit for bit,
    with identical LM decisions; fp32 residuals: see below."""
    ref = _run(0, 1, _free_port(), None, loss=loss, fp32=fp32)
    got = _run(0, 1, _free_port(), None, rccl_world1=True, loss=loss, fp32=fp32)
    if fp32:
        # float residuals: a contraction difference between the two kernels moves the float sums by ~1e-7 relative,
        # which can flip a borderline tolerance test (|x_cost - cand_cost| <= 1e-6 x_cost) and end a solve one
        # iteration apart (observed 1.9e-5 in r04e); the fp32 variant's bar against the oracle is 5e-3 m (test_gpu_parity)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-4)
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-14)


def _run_peer(rank, world, port, q, config, nscan, maps=None, env=None):
    """Peer sharding (floam_odom_set_shard_peers): one process per rank, the ranks' exchange buffers shared as IPC
    handles (gathered over gloo), the resident solve exchanging the 29 sums through them.  On the one-GPU box both
    ranks are processes on device 0 (the same IPC path as one process per GPU).  env: per-rank variables set before
    the library is loaded (e.g. the diagnostic build and its hooks, tests/diag.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if env and rank in env:
        os.environ.update(env[rank])
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import floam_amd
        from floam_amd import synth
        from floam_amd.odom_estimation import reset_process_state
        R = synth.lidar_model(config).rings
        p = floam_amd.LidarParams(num_lines=R, scan_period=0.1, max_distance=90.0, min_distance=0.5)
        lp = floam_amd.LaserProcessingClass(device=0)
        lp.init(p)
        odo = floam_amd.OdomEstimationClass(device=0)
        odo.init(p, 0.1, "Cauchy")
        reset_process_state()
        handle, _ = odo.shard_exchange()
        handles = [None] * world
        dist.all_gather_object(handles, handle)
        odo.set_shard_peers(rank, world, handles=handles)
        dist.barrier()
        poses = []
        first = 0
        if maps is not None:
            odo.initMapWithPoints(floam_amd.DeviceCloud(maps[0], device=0), floam_amd.DeviceCloud(maps[1], device=0))
            first = 1
        for k in range(first, first + nscan):
            de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
            lp.featureExtraction(floam_amd.DeviceCloud(synth.generate_scan(config, k), device=0), de, ds)
            if k == 0:
                odo.initMapWithPoints(de, ds)
            else:
                odo.UpdatePointsToMapSelector(de, ds, True)
            q_, t_ = odo.pose()
            poses.append(np.r_[q_, t_])
        out = (np.array(poses), odo.map_sizes())
        dist.barrier()   # (no rank closes its exchange buffer while another may still read it)
        odo.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _peer_ranks(config, nscan, maps=None, world=2, env=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run_peer, args=(r, world, port, q, config, nscan, maps, env)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    return res


def test_peer_two_ranks_match_unsharded(floam_gpu):
    """Peer sharding, two ranks (processes, IPC-mapped exchange buffers): poses identical on both ranks and within
    1e-9 of the unsharded run (C1, 5 scans: the first is the map)."""
    ref = _run(0, 1, _free_port(), None)
    res = _peer_ranks("c1", NSCAN)
    assert np.array_equal(res[0][0], res[1][0])
    for k in range(NSCAN):
        dt = np.linalg.norm(res[0][0][k][4:] - ref[k][4:])
        dr = 2 * math.acos(min(1.0, abs(float(np.dot(res[0][0][k][:4], ref[k][:4])))))
        assert dt < 1e-9 and dr < 1e-9, (k, dt, dr)


def test_peer_two_ranks_c4_match_oracle(floam_gpu, oracle_lib, prefilled_map):
    """the resident solve sharded over two ranks through peer-mapped exchange buffers at C4
    (128 rings, 500k prefill): poses identical on both ranks and within 1e-6 m / rad of the oracle, map sizes equal."""
    mapE, mapS = prefilled_map("c4")
    ref, ref_sizes = _c4_oracle(oracle_lib, mapE, mapS)
    res = _peer_ranks("c4", C4_SCANS, maps=(mapE, mapS))
    assert np.array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] == ref_sizes, (res[0][1], res[1][1], ref_sizes)
    _assert_close_to_oracle(res[0][0], ref, "2-rank peer shard")


def test_peer_world1_is_the_resident_solve(floam_gpu):
    """world = 1 peers: the plain resident solve (no exchange), bit-identical to the unsharded run."""
    import floam_amd
    from floam_amd import synth
    from floam_amd.odom_estimation import reset_process_state
    ref = _run(0, 1, _free_port(), None)
    p = floam_amd.LidarParams(num_lines=16, scan_period=0.1, max_distance=90.0, min_distance=0.5)
    lp = floam_amd.LaserProcessingClass(device=0)
    lp.init(p)
    odo = floam_amd.OdomEstimationClass(device=0)
    odo.init(p, 0.1, "Cauchy")
    reset_process_state()
    h, ptr = odo.shard_exchange()
    assert len(h) == 64 and ptr
    odo.set_shard_peers(0, 1, ptrs=[ptr])
    for k in range(NSCAN):
        de, ds = floam_amd.DeviceCloud(device=0), floam_amd.DeviceCloud(device=0)
        lp.featureExtraction(floam_amd.DeviceCloud(synth.generate_scan("c1", k), device=0), de, ds)
        if k == 0:
            odo.initMapWithPoints(de, ds)
        else:
            odo.UpdatePointsToMapSelector(de, ds, True)
        q_, t_ = odo.pose()
        assert np.array_equal(np.r_[q_, t_], ref[k]), k


def test_peer_late_blocks_across_solves(floam_gpu, oracle_lib, prefilled_map):
    """VERDICT r04 item 1 / Weak 6: the peer exchange's slot reuse must hold across solve boundaries.  Rank 1's
    non-zero solve blocks wait ~200 us before every poll of the other ranks' sums (FLOAM_PEER_DELAY_US, diagnostic
    build), so rank 0 finishes each solve and publishes the next solve's first exchange while rank 1's late blocks still
    poll for the last one — with a per-solve slot counter (it & 1) they then saw the new tag and spun to the 20-s
    timeout.  Deterministic: C1 (5 scans) and C4 (128 rings, 500k prefill) complete, no handle fails, poses identical
    on both ranks and equal to the undelayed two-rank run / within 1e-6 of the oracle."""
    diag = {"FLOAM_AMD_LIB": "diag"}
    env = {0: diag, 1: {**diag, "FLOAM_PEER_DELAY_US": "200"}}
    ref = _peer_ranks("c1", NSCAN)
    res = _peer_ranks("c1", NSCAN, env=env)
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][0], ref[0][0])
    mapE, mapS = prefilled_map("c4")
    oref, ref_sizes = _c4_oracle(oracle_lib, mapE, mapS)
    res = _peer_ranks("c4", C4_SCANS, maps=(mapE, mapS), env=env)
    assert np.array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] == ref_sizes, (res[0][1], res[1][1], ref_sizes)
    _assert_close_to_oracle(res[0][0], oref, "2-rank peer shard, late blocks on rank 1")


def test_peer_five_ranks_match_unsharded(floam_gpu):
    """world > 4 puts more than 256 exchange granules in a block's poll (58 per rank); every rank's
    sums must still be read.  Five ranks (processes sharing the one GPU, IPC-mapped buffers) on C1: poses identical on
    all ranks and within 1e-9 of the unsharded run."""
    ref = _run(0, 1, _free_port(), None)
    res = _peer_ranks("c1", NSCAN, world=5)
    for r in range(1, 5):
        assert np.array_equal(res[0][0], res[r][0]), r
    for k in range(NSCAN):
        dt = np.linalg.norm(res[0][0][k][4:] - ref[k][4:])
        dr = 2 * math.acos(min(1.0, abs(float(np.dot(res[0][0][k][:4], ref[k][:4])))))
        assert dt < 1e-9 and dr < 1e-9, (k, dt, dr)


def test_peer_eight_ranks_match_unsharded(floam_gpu, oracle_lib, prefilled_map):
    """world = kMaxShardRanks = 8, the world the driver's 8-GPU run uses, as eight processes on
    the one GPU (IPC-mapped exchange buffers; every rank's set_shard_peers probes the seven others' mappings first).
    C1 (5 scans): poses identical on all ranks and within 1e-9 of the unsharded run; C4 (128 rings, 500k prefill):
    identical on all ranks, map sizes equal to the oracle's and poses within 1e-6 of it."""
    ref = _run(0, 1, _free_port(), None)
    res = _peer_ranks("c1", NSCAN, world=8)
    for r in range(1, 8):
        assert np.array_equal(res[0][0], res[r][0]), r
    for k in range(NSCAN):
        dt = np.linalg.norm(res[0][0][k][4:] - ref[k][4:])
        dr = 2 * math.acos(min(1.0, abs(float(np.dot(res[0][0][k][:4], ref[k][:4])))))
        assert dt < 1e-9 and dr < 1e-9, (k, dt, dr)
    mapE, mapS = prefilled_map("c4")
    oref, ref_sizes = _c4_oracle(oracle_lib, mapE, mapS)
    res = _peer_ranks("c4", C4_SCANS, maps=(mapE, mapS), world=8)
    for r in range(1, 8):
        assert np.array_equal(res[0][0], res[r][0]), r
        assert res[r][1] == ref_sizes, (r, res[r][1], ref_sizes)
    _assert_close_to_oracle(res[0][0], oref, "8-rank peer shard")


def _probe_lonely_rank(q):
    """One rank of a two-rank peer group whose other rank never calls set_shard_peers (its mapping never answers)."""
    import floam_amd
    p = floam_amd.LidarParams(num_lines=16, scan_period=0.1, max_distance=90.0, min_distance=0.5)
    odo = floam_amd.OdomEstimationClass(device=0)
    odo.init(p, 0.1, "Cauchy")
    other = floam_amd.OdomEstimationClass(device=0)   # a second handle: its buffer exists but never answers
    other.init(p, 0.1, "Cauchy")
    _, mine = odo.shard_exchange()
    _, theirs = other.shard_exchange()
    import time
    t0 = time.time()
    try:
        odo.set_shard_peers(0, 2, ptrs=[mine, theirs])
        q.put(("no error", time.time() - t0))
    except floam_amd.FloamError as e:
        q.put((str(e), time.time() - t0))


def test_peer_probe_fails_fast(floam_gpu):
    """a peer mapping that never answers fails floam_odom_set_shard_peers in seconds with
    FLOAM_ERR_COMM (bench.py then takes the RCCL form), instead of the first solve's ~20-s hand-off timeout."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_probe_lonely_rank, args=(q,))
    pr.start()
    msg, dt = q.get(timeout=120)
    pr.join(timeout=60)
    assert pr.exitcode == 0
    assert "probe" in msg and "rank(s) 1" in msg, msg
    assert 1.5 < dt < 10.0, dt
