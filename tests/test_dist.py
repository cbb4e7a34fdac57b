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


# ---- bench.py --gpus N: the launcher and the engine's multi-rank step (nranks > 1) ----------
def _bench(stub_lib, *args, devices=2, timeout=240):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MPX_LIB=stub_lib, MPX_STUB_DEVICES=str(devices))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args],
                          capture_output=True, text=True, env=env, timeout=timeout, cwd=root)


def _expected_step(g_total, ipg=256, n=5, b=4, keys=256):
    """one step of every group of the job in ONE process through the oracle: the fused
    watermark vector every rank must hold after the all-reduce, and the summed totals"""
    import hashlib

    from oracle_lib import Oracle
    full = synth.group_batch(g_total, ipg, n, b, keys, p_ok=0.7, p_put=0.5, seed=45)
    want = Oracle(n, R.MODE_MIN, kv_per_group=256).group_step(full)
    wm = np.concatenate([want["committed_out"], want["executed_out"]]).astype(np.int32)
    ei = full["executed_in"].astype(np.int64)
    eo = want["executed_out"].astype(np.int64)
    lo = np.maximum(ei + 1, 0)
    coff = full["cmd_off"].astype(np.int64)
    g0 = np.arange(g_total, dtype=np.int64) * ipg
    ran = eo >= lo
    xi = int(np.where(ran, eo - lo + 1, 0).sum())
    xc = int(np.where(ran, coff[g0 + np.where(ran, eo, 0) + 1] - coff[g0 + lo], 0).sum())
    return (hashlib.sha256(wm.tobytes()).hexdigest(),
            (int(want["n_decided"].sum()), xi, xc))


@pytest.mark.parametrize("scaling,extra,g_total", [
    ("strong", ["--groups-total", "64"], 64),
    ("weak", ["--groups", "24"], 48),
    ("strong", ["--groups-total", "37"], 37),  # ragged blocks: 18 + 19 groups
])
def test_bench_gpus2_multirank_step(stub_lib, scaling, extra, g_total):
    """`bench.py --gpus 2` starts two rank processes itself; each runs the engine's real
    multi-rank step sequence (engine.cpp: comm init over the broadcast unique id, group step,
    step totals, the fused max + sum RCCL group on a second stream, double-buffered watermark
    vectors reset to -1 outside the rank's block) for 1 + 1 warm-up + 3 timed steps, so both
    buffers are reused. The buffers start poisoned, so a missing -1 fill would survive the max.
    Every rank must end with the single-process oracle's vector and the line's totals must be
    the oracle's sums."""
    r = _bench(stub_lib, "--gpus", "2", "--scaling", scaling, *extra, "--steps", "3",
               "--warmup", "1", "--no-cpu-baseline")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    import json
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["config"]["groups_total"] == g_total
    assert line["parity"]["bit_exact"], line["parity"]
    sha, (nd, xi, xc) = _expected_step(g_total)
    assert line["watermarks_identical_on_all_ranks"]
    assert line["watermarks_sha256"] == sha
    assert line["watermark_allreduce_ok"]
    assert (line["decided_instances_per_step"], line["executed_instances_per_step"],
            line["executed_commands_per_step"]) == (nd, xi, xc)


def test_bench_gpus1_line_shape(stub_lib):
    """--gpus 1 runs in-process (no launcher) and prints the same keys as the 2-rank line"""
    r1 = _bench(stub_lib, "--gpus", "1", "--groups-total", "16", "--steps", "2", "--warmup", "1",
                "--no-cpu-baseline", devices=1)
    r2 = _bench(stub_lib, "--gpus", "2", "--groups-total", "16", "--steps", "2", "--warmup", "1",
                "--no-cpu-baseline")
    assert r1.returncode == 0 and r2.returncode == 0, r1.stderr[-2000:] + r2.stderr[-2000:]
    import json
    l1, l2 = (json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
              for r in (r1, r2))
    assert l1["n_gpus"] == 1 and l2["n_gpus"] == 2
    assert sorted(l1) == sorted(l2)
    sha, _ = _expected_step(16)
    assert l1["watermarks_sha256"] == sha == l2["watermarks_sha256"]
    # achieved from min(event mean, ms_per_step): the kernel never gets more time than its step
    for ln in (l1, l2):
        rf = ln["roofline"]
        assert 0 < rf["kernel_ms_bound"] <= ln["ms_per_step"]
        assert rf["kernel_ms_bound"] == min(rf["kernel_ms_avg"], ln["ms_per_step"])


def test_bench_kernel_events_inline(stub_lib):
    """--kernel-events inline: the event pairs sit in the timed steps themselves"""
    import json
    r = _bench(stub_lib, "--groups-total", "16", "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline", "--kernel-events", "inline", devices=1)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["roofline"]["kernel_ms_avg"] > 0 and line["parity"]["bit_exact"]


def test_bench_launcher_rank_failure_exits_nonzero(stub_lib):
    """one rank failing (rank 1 has no device: the stub reports one) ends the job non-zero
    instead of leaving rank 0 blocked in a collective"""
    r = _bench(stub_lib, "--gpus", "2", "--groups-total", "16", "--steps", "2", "--warmup", "1",
               "--no-cpu-baseline", devices=1, timeout=180)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("P,g_total", [(2, 64), (3, 37)])
def test_bench_emulate_world(stub_lib, P, g_total):
    """`--emulate-world P`: one process runs rank 0's share of a P-rank job (groups
    [0, ceil(g_total / P)) under the launcher's block split) with the full watermark vector
    through the engine's all-reduce; the owned range must hold the oracle's watermarks and every
    foreign entry must stay -1 (watermark_allreduce_ok), and the line names the emulation"""
    r = _bench(stub_lib, "--emulate-world", str(P), "--groups-total", str(g_total), "--steps", "2",
               "--warmup", "1", "--no-cpu-baseline", devices=1)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    emu = line["emulated_world"]
    assert emu["ranks"] == P and emu["groups_total"] == g_total
    assert 0 < emu["groups_on_this_rank"] < g_total
    assert line["watermark_allreduce_ok"] and line["parity"]["bit_exact"], line["parity"]
    assert "EMULATED" in line["config"]["workload"]
