"""N > 1 path on CPU (gloo, world_size 2): query sharding + one all-reduce of the normal equations.

The HIP path splits each correspondence set into `world` contiguous ranges [n*r/W, n*(r+1)/W) (corr_kernel) and
all-reduces the 29 sums (cost, J^T J upper triangle, J^T r, count) once per LM evaluation (host.cpp
allreduce_sums).  Here each rank computes its shard's sums with the reference cost functions (oracle), the sums
are all-reduced over gloo, and the result must equal the unsharded sums and be bitwise identical on every rank
(so every rank takes the same LM decision).  The control-plane broadcast bench.py uses for the RCCL unique id is
exercised too.
"""
import os
import socket

import numpy as np
import pytest

WORLD = 2


def _records(seed=0, ne=37, ns=91):
    rng = np.random.default_rng(seed)
    edges = []
    for _ in range(ne):
        cp = rng.uniform(-20, 20, 3)
        a = rng.uniform(-20, 20, 3)
        edges.append((cp, a, a + rng.standard_normal(3) * 0.2))
    surfs = []
    for _ in range(ns):
        n = rng.standard_normal(3)
        surfs.append((rng.uniform(-20, 20, 3), n / np.linalg.norm(n), rng.uniform(-3, 3)))
    return edges, surfs


def shard_range(n, rank, world):
    return (n * rank) // world, (n * (rank + 1)) // world


def partial_sums(oracle, edges, surfs, x, rank, world, huber=False):
    s = np.zeros(29)
    lo, hi = shard_range(len(edges), rank, world)
    rows = [oracle.edge_residual(cp, a, b, x) for cp, a, b in edges[lo:hi]]
    lo, hi = shard_range(len(surfs), rank, world)
    rows += [oracle.surf_residual(cp, n, d, x) for cp, n, d in surfs[lo:hi]]
    for r, J in rows:
        sq = r * r
        if huber and sq > 0.01:
            rr = np.sqrt(sq)
            rho0, rho1 = 0.2 * rr - 0.01, 0.1 / rr
        else:
            rho0, rho1 = sq, 1.0
        s[0] += 0.5 * rho0
        r, J = r * np.sqrt(rho1), J * np.sqrt(rho1)
        s[1:22] += np.outer(J, J)[np.triu_indices(6)]
        s[22:28] += J * r
        s[28] += 1
    return s


def _worker(rank, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import oracle
        edges, surfs = _records()
        x = np.array([0.01, -0.02, 0.03, 0.0, 0.5, -0.2, 0.1])
        x[3] = np.sqrt(1 - np.sum(x[:3] ** 2))
        out = {}
        for huber in (False, True):
            part = torch.tensor(partial_sums(oracle, edges, surfs, x, rank, WORLD, huber), dtype=torch.float64)
            dist.all_reduce(part, op=dist.ReduceOp.SUM)
            out[huber] = part.numpy().copy()
        uid = [bytes(range(128)) if rank == 0 else None]   # RCCL unique id broadcast (bench.py)
        dist.broadcast_object_list(uid, src=0)
        q.put((rank, out, uid[0]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_normal_equations_gloo(oracle_lib):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    edges, surfs = _records()
    x = np.array([0.01, -0.02, 0.03, 0.0, 0.5, -0.2, 0.1])
    x[3] = np.sqrt(1 - np.sum(x[:3] ** 2))
    for huber in (False, True):
        full = partial_sums(oracle_lib, edges, surfs, x, 0, 1, huber)
        for _, out, _ in res:
            np.testing.assert_allclose(out[huber], full, rtol=1e-12, atol=1e-12)
        assert np.array_equal(res[0][1][huber], res[1][1][huber])   # identical on every rank
        assert res[0][1][huber][28] == len(edges) + len(surfs)
    assert res[1][2] == bytes(range(128))


@pytest.mark.parametrize("n", [0, 1, 2, 5, 37, 1000])
def test_shard_ranges_partition(n):
    cover = []
    for w in (1, 2, 3, 8):
        cover = []
        for r in range(w):
            lo, hi = shard_range(n, r, w)
            cover.extend(range(lo, hi))
        assert cover == list(range(n))
