"""Multi-rank path on CPU: world_size 2 (and 3) over gloo.

Each rank generates only its block of groups, runs the per-group step for that block (here the
CPU oracle stands in for the GPU kernel: this test checks the partition and the collective, the
kernel itself is covered by the GPU parity tests), builds the fused watermark vector with -1 on
groups it does not own, and max-all-reduces it. Every rank must end with exactly the watermarks
of a single-process run over all groups.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from minpaxos_amd import shard, synth
from minpaxos_amd import records as R

G_TOTAL, IPG = 48, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from oracle_lib import Oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g0, g1 = shard.block_range(G_TOTAL, world, rank)
        b = synth.group_batch(g1 - g0, IPG, 5, 4, 32, seed=45, first_group=g0)
        out = Oracle(5, R.MODE_MIN).group_step(b)
        wm = shard.watermark_vector(G_TOTAL, g0, out["committed_out"], out["executed_out"])
        wm = shard.allreduce_watermarks(wm)
        q.put((rank, wm.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_watermark_allreduce_gloo(world):
    from oracle_lib import Oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = synth.group_batch(G_TOTAL, IPG, 5, 4, 32, seed=45)
    want = Oracle(5, R.MODE_MIN).group_step(full)
    ref = np.concatenate([want["committed_out"], want["executed_out"]])
    for r in range(world):
        assert np.array_equal(np.array(got[r], np.int32), ref), r


def test_block_partition():
    for n in (1, 7, 64, 65536, 100003):
        for w in (1, 2, 3, 8):
            seen = np.zeros(n, np.int32)
            for r in range(w):
                a, b = shard.block_range(n, w, r)
                seen[a:b] += 1
            assert (seen == 1).all()
            for gidx in (0, n // 2, n - 1):
                a, b = shard.block_range(n, w, shard.owner_of(gidx, n, w))
                assert a <= gidx < b


def test_rank_block_equals_global_slice():
    """a rank's generated block is byte-identical to the same block of the whole job"""
    full = synth.group_batch(16, 32, 5, 4, 32, seed=45)
    part = synth.group_batch(6, 32, 5, 4, 32, seed=45, first_group=5)
    assert np.array_equal(full["recs"][5 * 32 * 4:11 * 32 * 4], part["recs"])
    assert np.array_equal(full["key"][5 * 32 * 4:11 * 32 * 4], part["key"])
    assert np.array_equal(full["op"][5 * 32 * 4:11 * 32 * 4], part["op"])


def _ranks_worker(rank, world, port, q):
    """bench.Ranks over gloo: RCCL unique-id broadcast, barrier, max over ranks"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import bench
    rk = bench.Ranks()
    try:
        uid = rk.bcast(bytes(range(128)) if rank == 0 else None)
        rk.barrier()
        q.put((rank, uid, rk.max(1.5 * (rank + 1))))
    finally:
        rk.close()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_ranks_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ranks_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, uid, mx in got:
        assert uid == bytes(range(128)) and mx == 1.5 * world


def test_strong_scaling_partition_covers_groups():
    """--scaling strong: block ranges of groups_total over P ranks tile [0, G) exactly"""
    for g_total in (65536, 1000, 7):
        for world in (1, 2, 4, 8):
            rs = [shard.block_range(g_total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == g_total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
